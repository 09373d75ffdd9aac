"""Timeline of the persistent MU launch from the diagnostic stamps build (s_memrealtime, 100 MHz).

    python -m cnmf_amd.build --stamps
    CNMF_HIP_LIB=cnmf_amd/libcnmf_hip_stamps.so python tools/timeline_persist.py [--iters 20]

Per steady-state iteration: the streaming span of each workgroup (basis ready -> rows published),
the arrival skew (first -> last workgroup), the reduction tail (last arrival -> AB published) and
the resume latency (AB published -> basis ready in each workgroup).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TL_IT, TL_WG = 64, 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1000, help="iterations before the stamped launch (clock ramp)")
    ap.add_argument("--solver", default="mu", choices=["mu", "als", "wmu"],
                    help="als: the persistent constrained ALS (sum_to_one 1, smoothness 0.5); wmu: the "
                         "persistent weighted MU (30 %% zero weights)")
    ap.add_argument("--layout", type=int, default=0, help="the plan's persistent layout (0 = default)")
    ap.add_argument("--tol", type=float, default=0.0,
                    help="> 0: the stamped launch is the device tolerance test's (cnmf_mu_fit_tol); a tol "
                         "small enough never stops it")
    ap.add_argument("--exchange", action="store_true",
                    help="the multi-GPU launch exchanging with itself (world-1 gloo group)")
    a = ap.parse_args()
    import torch
    from cnmf_amd import _lib
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    X = iop_spectra(a.rows, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, a.k, 42)
    lib = _lib.load()
    fn = lib.cnmf_debug_timeline
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    group = None
    if a.exchange:
        import socket
        import torch.distributed as dist
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        group = dist.group.WORLD
    if a.solver == "als":
        from cnmf_amd.solver import ALSPlan
        plan = ALSPlan(torch.from_numpy(X).cuda(), a.k, sum_to_one=1.0, smoothness=0.5)
    elif a.solver == "wmu":
        from cnmf_amd.solver import WeightedMUPlan
        rng = np.random.default_rng(0)
        M = (rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= 0.3)).astype(np.float32)
        plan = WeightedMUPlan(torch.from_numpy(X).cuda(), torch.from_numpy(M).cuda(), a.k)
    else:
        plan = MUPlan(torch.from_numpy(X).cuda(), a.k, group=group)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    if a.layout and hasattr(plan, "layout"):
        plan.layout = a.layout
    if a.exchange:
        plan.enable_exchange()
    assert plan.persistent
    plan.iterate(a.warmup)
    torch.cuda.synchronize()
    fph = getattr(lib, "cnmf_debug_resume_phases", None)
    if fph is not None:  # the ALS resume path's phase sums (workgroup 0), from this launch only
        fph.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fph.restype = ctypes.c_int
        _lib.check(fph(np.zeros(16, dtype=np.uint64).ctypes.data, 1), "resume phases")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if a.tol > 0:
        plan.fit_device_tol(a.iters, a.tol)
    else:
        plan.iterate(a.iters)
    e1.record()
    torch.cuda.synchronize()
    launch_us = e0.elapsed_time(e1) * 1e3
    buf = np.zeros(TL_IT * TL_WG * 2 + TL_IT + TL_WG + TL_WG, dtype=np.uint64)
    _lib.check(fn(buf.ctypes.data), "timeline")
    G = plan.n_parts
    from cnmf_amd.solver import MUPlan as _M  # noqa: F401
    tl = buf[:TL_IT * TL_WG * 2].reshape(TL_IT, TL_WG, 2).astype(np.int64)
    pub = buf[TL_IT * TL_WG * 2:TL_IT * TL_WG * 2 + TL_IT].astype(np.int64)
    start = buf[TL_IT * TL_WG * 2 + TL_IT:TL_IT * TL_WG * 2 + TL_IT + TL_WG].astype(np.int64)
    hw = buf[TL_IT * TL_WG * 2 + TL_IT + TL_WG:].view(np.uint32).reshape(TL_WG, 2)
    # the grid actually launched: workgroups with a start stamp in this launch
    g = int(np.count_nonzero(start[:G] >= start[:G].max() - 10_000_000))
    n = min(a.iters, TL_IT)
    arr = tl[:n, :g, 0]
    res = tl[:n, :g, 1]
    t0 = start[:g].min()
    rows = []
    for it in range(1, n - 1):
        span = (arr[it] - res[it - 1]) * 10 / 1e3  # us
        rows.append({
            "it": it,
            "period_us": (pub[it] - pub[it - 1]) * 10 / 1e3,
            "stream_med_us": float(np.median(span)), "stream_min_us": float(span.min()),
            "stream_max_us": float(span.max()),
            "skew_us": (arr[it].max() - arr[it].min()) * 10 / 1e3,
            "tail_us": (pub[it] - arr[it].max()) * 10 / 1e3,
            "resume_med_us": float(np.median(res[it] - pub[it])) * 10 / 1e3,
            "resume_max_us": float((res[it] - pub[it]).max()) * 10 / 1e3,
        })
    summary = {k: round(float(np.median([r[k] for r in rows])), 2) for k in rows[0] if k != "it"}
    # is the skew systematic?  per-workgroup stream time, iterations 1..n-2
    spans = np.stack([(arr[it] - res[it - 1]) * 10 / 1e3 for it in range(1, n - 1)])  # [it][wg]
    mean_wg = spans.mean(axis=0)
    half = spans.shape[0] // 2
    corr = float(np.corrcoef(spans[:half].mean(axis=0), spans[half:].mean(axis=0))[0, 1])
    nbt = np.array([(plan.n_rows // 64 - b + g - 1) // g for b in range(g)])
    by_xcd = [round(float(mean_wg[np.arange(g) % 8 == x].mean()), 2) for x in range(8)]
    summary.update({"wg_stream_corr_between_halves": round(corr, 3), "stream_by_b_mod_8": by_xcd,
                    "stream_by_tiles": {int(v): round(float(mean_wg[nbt == v].mean()), 2) for v in np.unique(nbt)},
                    "per_wg_mean_min_max": [round(float(mean_wg.min()), 2), round(float(mean_wg.max()), 2)],
                    "within_wg_std_us": round(float(spans.std(axis=0).mean()), 2)})
    # physical placement: HW_ID bits cu_id [11:8], sh_id [12], se_id [15:13]; XCC_ID [3:0]
    hwid, xcc = hw[:g, 0].astype(np.int64), hw[:g, 1].astype(np.int64) & 0xF
    cu = (hwid >> 8) & 0xF
    se = (hwid >> 13) & 0x7
    sh = (hwid >> 12) & 0x1
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    per_cu = np.bincount(inv, weights=mean_wg) / cnt
    co = cnt[inv]  # workgroups sharing this block's CU
    summary.update({"n_cus_used": int(len(uk)), "wgs_per_cu_hist": {int(c): int((cnt == c).sum()) for c in np.unique(cnt)},
                    "stream_by_wgs_on_cu": {int(c): round(float(mean_wg[co == c].mean()), 2) for c in np.unique(co)},
                    "stream_by_xcc": [round(float(mean_wg[xcc == x].mean()), 2) for x in range(8)],
                    "stream_by_se": [round(float(mean_wg[se == x].mean()), 2) if (se == x).any() else None for x in range(8)],
                    "cu_mean_min_max": [round(float(per_cu.min()), 2), round(float(per_cu.max()), 2)],
                    "same_cu_pair_corr": round(float(np.corrcoef(mean_wg, per_cu[inv])[0, 1]), 3),
                    "b_mod_8_equals_xcc_frac": round(float(np.mean((np.arange(g) % 8) == xcc)), 3)})
    slow = np.argsort(mean_wg)[-8:]
    summary["slowest_wgs"] = [(int(b), int(xcc[b]), int(se[b]), int(cu[b]), round(float(mean_wg[b]), 1)) for b in slow]
    summary.update({"grid": g, "iters": a.iters, "launch_us": round(launch_us, 1),
                    "us_per_iter": round(launch_us / a.iters, 2),
                    "first_arrival_it0_us": round((arr[0].min() - t0) * 10 / 1e3, 2)})
    if a.exchange:
        fx = lib.cnmf_debug_xtimeline
        fx.argtypes = [ctypes.c_void_p]
        fx.restype = ctypes.c_int
        xb = np.zeros(TL_IT * 4, dtype=np.uint64)
        _lib.check(fx(xb.ctypes.data), "xtimeline")
        x = xb.reshape(TL_IT, 4).astype(np.int64)[1:n - 1]
        p_ = pub[1:n - 1]
        summary["exchange_us_median"] = {
            "group_sum_to_start": None,
            "slot_stores": round(float(np.median(x[:, 1] - x[:, 0])) * 10 / 1e3, 2),
            "flag_wait": round(float(np.median(x[:, 2] - x[:, 1])) * 10 / 1e3, 2),
            "slot_loads_sum": round(float(np.median(x[:, 3] - x[:, 2])) * 10 / 1e3, 2),
            "to_publish": round(float(np.median(p_ - x[:, 3])) * 10 / 1e3, 2),
            "arrival_to_start": round(float(np.median(x[:, 0] - arr[1:n - 1].max(axis=1))) * 10 / 1e3, 2)}
    flv = getattr(lib, "cnmf_debug_levels", None)
    if flv is not None and a.solver == "mu" and a.k in (4, 8):  # the reduction tree, level by level
        flv.argtypes = [ctypes.c_void_p]
        flv.restype = ctypes.c_int
        LVG = 64
        nlv = TL_IT * (LVG + 1) * 2
        lb = np.zeros(nlv + 4 * TL_IT * TL_WG, dtype=np.uint64)
        _lib.check(flv(lb.ctypes.data), "levels")
        lv = lb[:nlv].reshape(TL_IT, LVG + 1, 2).astype(np.int64)
        pre = lb[nlv:nlv + TL_IT * TL_WG].reshape(TL_IT, TL_WG).astype(np.int64)[:, :g]
        seen = lb[nlv + TL_IT * TL_WG:nlv + 2 * TL_IT * TL_WG].reshape(TL_IT, TL_WG).astype(np.int64)[:, :g]
        abl = lb[nlv + 2 * TL_IT * TL_WG:nlv + 3 * TL_IT * TL_WG].reshape(TL_IT, TL_WG).astype(np.int64)[:, :g]
        upd = lb[nlv + 3 * TL_IT * TL_WG:].reshape(TL_IT, TL_WG).astype(np.int64)[:, :g]
        ng = int(np.count_nonzero(lv[1, :LVG, 0]))
        us = lambda v: round(float(np.median(v)) * 10 / 1e3, 2)  # noqa: E731
        its = range(1, n - 1)
        last_arr = np.array([arr[i].max() for i in its])
        grp_t = np.array([lv[i, :ng, 0].max() for i in its])
        grp_d = np.array([lv[i, :ng, 1].max() for i in its])
        top_t = np.array([lv[i, LVG, 0] for i in its])
        top_d = np.array([lv[i, LVG, 1] for i in its])
        pubs = np.array([pub[i] for i in its])
        last_wg = [int(np.argmax(arr[i])) for i in its]
        summary["tree_us_median"] = {
            "groups": ng,
            "partial_row_store_median_wg": us(np.concatenate([arr[i] - pre[i] for i in its])),
            "partial_row_store_last_arriver": us([arr[i][w] - pre[i][w] for i, w in zip(its, last_wg)]),
            "last_arrival_to_last_group_ticket": us(grp_t - last_arr),
            "group_combine_median": us(np.concatenate([lv[i, :ng, 1] - lv[i, :ng, 0] for i in its])),
            "last_group_combine": us([lv[i, np.argmax(lv[i, :ng, 0]), 1] - lv[i, :ng, 0].max() for i in its]),
            "last_group_row_to_top_ticket": us(top_t - grp_d),
            "top_combine": us(top_d - top_t),
            "top_done_to_flag": us(pubs - top_d),
        }
        nt_ = [np.nonzero(seen[i] > pub[i] - 10)[0] for i in its]  # the workgroups that polled the flag
        summary["resume_us_median"] = {
            "flag_to_seen": us(np.concatenate([seen[i][m] - pub[i] for i, m in zip(its, nt_)])),
            "seen_to_ab_in_lds": us(np.concatenate([abl[i][m] - seen[i][m] for i, m in zip(its, nt_)])),
            "ab_to_basis_ready": us(np.concatenate([res[i][m] - abl[i][m] for i, m in zip(its, nt_)])),
            "ab_to_update_done": us(np.concatenate([upd[i][m] - abl[i][m] for i, m in zip(its, nt_)])),
            "update_done_to_ready": us(np.concatenate([res[i][m] - upd[i][m] for i, m in zip(its, nt_)])),
        }
    if a.solver == "als":  # H-step of workgroup 0: BPP iterations and cycles per row, per call
        fh = lib.cnmf_debug_hstep
        fh.argtypes = [ctypes.c_void_p]
        fh.restype = ctypes.c_int
        hb = np.zeros(64 * 4 * 2, dtype=np.uint64)
        _lib.check(fh(hb.ctypes.data), "hstep")
        hs = hb.reshape(64, 4, 2).astype(np.int64)
        used = hs[:, :, 1].sum(axis=1) > 0
        it_ = hs[used][-5:, :, 0]
        summary["hstep_bpp_iters_per_row_last_calls"] = (it_ & 0xFFFF).tolist()
        summary["hstep_kcycles_per_row_last_calls"] = (hs[used][-5:, :, 1] / 1e3).round(1).tolist()
        rt = (it_ >> 16) * 10 / 1e3  # the one-wave form: the row's s_memrealtime ticks (100 MHz) above bit 16
        if rt.max() > 0:
            summary["hstep_us_per_row_last_calls"] = rt.round(2).tolist()
            summary["hstep_shader_mhz"] = round(float(hs[used][-5:, :, 1].sum() / (rt.sum() * 1e3) * 1e3), 0)
        if fph is not None:
            pb = np.zeros(16, dtype=np.uint64)
            _lib.check(fph(pb.ctypes.data, 0), "resume phases")
            cnt = int(pb[15])
            if cnt:
                # the stamps present, in time order (cnmf_hip.hip PH(slot)): 0 flag seen, 1 AB in LDS,
                # 2 barrier, 3 (unused), 4 rows done, 5 after the H-step, 6 table done, 7 basis ready
                sums = pb.astype(np.int64)
                present = [q for q in range(8) if sums[q] > 0]
                summary["resume_phases_us_wg0"] = {
                    f"{a_}->{b_}": round(float(sums[b_] - sums[a_]) / cnt * 10 / 1e3, 3)
                    for a_, b_ in zip(present, present[1:])}
                summary["resume_phases_n"] = cnt
        fp = getattr(lib, "cnmf_debug_hstep_phases", None)
        if fp is not None:  # the wave H-step's phases per row: setup, gather, PCR, check (k cycles)
            fp.argtypes = [ctypes.c_void_p]
            fp.restype = ctypes.c_int
            pb = np.zeros(64 * 4 * 4, dtype=np.uint64)
            _lib.check(fp(pb.ctypes.data), "hstep phases")
            ph = pb.reshape(64, 4, 4).astype(np.int64)
            summary["hstep_phase_kcycles_setup_gather_pcr_check_last_calls"] = (ph[used][-3:] / 1e3).round(2).tolist()
    print(json.dumps(summary), flush=True)
    for r in rows[:5]:
        print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
