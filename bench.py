"""Benchmark of the MI355X MU hot path (BASELINE.json metric: MU iterations/sec & achieved HBM
GB/s vs peak, V = 1e6 x 81, k = 4, at 1/2/4/8 GPUs; configs[1] = cfg2 at one GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
    python bench.py --rows 10000000 --k 8             # cfg3's rows on one GPU
    python bench.py --rows 10000000 --k 8 --scaling strong   # cfg3 as one 1e7-row problem over the GPUs
    python bench.py --solver als                      # cfg5, the constrained ALS
    python bench.py --features 300 --k 16 --dtype bf16   # cfg4, the bf16 matrix-core pass

One "step" = one MU iteration (sample pass over X + cross-workgroup reduction + basis update) on
synthetic IOP spectra (cnmf_amd.synthetic), fp32, tol = 0, inputs resident in HBM before the timed
region.

Default --scaling weak (the task's rule for a path that shards its units): every rank owns --rows
rows of the sample axis (rank 0's rows are exactly cfg2's X), and the k(F+k) fp64 accumulators —
the path's one exchange — are all-reduced every iteration, inside the persistent launch over xGMI
when validated, else RCCL.  value = ranks x K / time in the unit "<rows>-row it/s" (cfg2: "1e6-row
it/s"): the iterations of one <rows>-row shard that all ranks completed per second (at N = 1 exactly
the it/s of the problem run).  --scaling strong: V = --rows x 81 is ONE problem (cfg2's X, or
cfg3's) split over the N ranks in 64-row-aligned shards, value = iterations/s of that problem
(unit "it/s").

At N > 1 the line also carries `strong`: the metric's own V = --strong-rows (default 1e6) x 81
problem — cfg2's X and start, split over the same ranks — timed in the same run, and the same
problem on rank 0's GPU alone, so `strong.speedup_vs_n1` is north_star's strong-scaling figure
measured on one clock.  At N = 1 `strong` is the line itself.

The bench refuses to report a broken run: a non-finite final error, or a non-finite or negative
entry of W or H on any rank, exits with status 3 and prints no line.

Extra keys: roofline (the dominant kernel timed with HIP events on its launch stream inside the
timed region: at N = 1 the ONE persistent launch that runs all K iterations, else each per-iteration
launch; achieved = algorithmic bytes of this GPU's shard n·(F·4 + 2·k·4) per iteration × iterations
per launch ÷ the slowest rank's launch time, peak = one MI355X's 8 TB/s), cpu_baseline (the NumPy /
scipy oracle, rank 0 at N = 1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
EXIT_BROKEN = 3  # a run whose final state is not a valid factorisation: no line is printed


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (one rank each); default: WORLD_SIZE when a launcher set it, else 1")
    p.add_argument("--steps", type=int, default=500)
    # 1000 warmup iterations (~70 ms at cfg2): after idle the chip runs its first ~35 ms of work at
    # lower clocks (tools/bench_trend.py: 73.7 us/iteration on the first 500-iteration launch,
    # 66 us on the following ones), so a short warmup would time the clock ramp, not the solver
    p.add_argument("--warmup", type=int, default=1000)
    p.add_argument("--rows", type=int, default=1_000_000,
                   help="rows of V: the whole problem (--scaling strong) or per GPU (--scaling weak)")
    p.add_argument("--scaling", default="weak", choices=["strong", "weak"],
                   help="weak (default): every GPU owns --rows rows, value = ranks x iterations/s in "
                        "'<rows>-row it/s'; strong: --rows is ONE problem split over the GPUs, value = "
                        "iterations/s of that problem")
    p.add_argument("--strong-rows", type=int, default=None,
                   help="at N > 1: also time this V (x F) as ONE problem split over the ranks, and on "
                        "rank 0's GPU alone (the line's `strong` key); 0 = skip; default 1e6 (the "
                        "metric's V), skipped when ranks share a GPU (their 1e6-row persistent grids "
                        "are not co-resident on one device; ADVICE r5)")
    p.add_argument("--features", type=int, default=81)
    p.add_argument("--k", type=int, default=4)
    p.add_argument("--dtype", default="f32", choices=["f32", "f64", "bf16"])
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--weighted", action="store_true",
                   help="the weighted / masked MU (SURVEY §8(f) row 2): synthetic weights, 30 %% zero")
    p.add_argument("--solver", default="mu", choices=["mu", "als"],
                   help="mu: cfg2 (the headline); als: cfg5, the constrained ALS")
    p.add_argument("--sum-to-one", type=float, default=1.0, help="ALS sum-to-one weight (delta)")
    p.add_argument("--smoothness", type=float, default=0.5, help="ALS smoothness penalty (lambda)")
    p.add_argument("--dist", action="store_true",
                   help="use the multi-GPU code path even at one rank (diagnostic; a world-size-1 "
                        "nccl group): the in-launch exchange with itself, or with --exchange off "
                        "shard step + RCCL all_reduce per iteration")
    p.add_argument("--exchange", default="auto", choices=["auto", "off"],
                   help="multi-GPU MU: auto = the all-reduce inside the persistent launch (peer "
                        "exchange over xGMI), validated against the RCCL path before timing and "
                        "replaced by it on any failure; off = shard step + RCCL all_reduce")
    p.add_argument("--ramp-seconds", type=float, default=0.5,
                   help="untimed clock ramp after the warmup: iterations on copies of W and H until "
                        "this much GPU time has passed (the chip holds a low clock for its first "
                        "tens of ms of work; the state is restored, the timed K steps are unchanged)")
    p.add_argument("--settle-ms", type=float, default=2.0,
                   help="idle pause (ms) between the last untimed launch and the timed region: right "
                        "behind a busy launch a short timed launch reads up to 13 %% slower, after a "
                        "1-300 ms pause it reads the steady 500-step rate (tools/driver_form_probe.py, "
                        "DESIGN §5)")
    p.add_argument("--no-tune", action="store_true",
                   help="skip timing the persistent-launch layouts (MUPlan.tune) before the run")
    p.add_argument("--layout", type=int, default=0,
                   help="> 0: run this persistent layout (include/cnmf_hip.h) instead of tuning")
    p.add_argument("--tol", type=float, default=0.0,
                   help="> 0: the timed fit runs sklearn's tolerance test (SK:872-884) on the device "
                        "(cnmf_mu_fit_tol: ONE launch, the error every 10 iterations inside it); value = "
                        "iterations done / time (the fit may stop before --steps)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="torch.distributed backend at N > 1: nccl (= RCCL over xGMI, the default) or "
                        "gloo (host-side collectives: lets two ranks share one GPU, as the N > 1 tests do)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="PMC traffic summary written by tools/pmc_traffic.py (optional)")
    return p.parse_args(argv)


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline line."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _time_oracle_mu(X, W0, H0, budget_s):
    """Iterations per second of oracle/mu_ref.py's fp32 MU on the host: (it/s, iterations, seconds)."""
    from oracle import mu_ref
    W, H = W0.copy(), H0.copy()

    def one():
        nonlocal W, H
        W, _, _ = mu_ref.update_w(X, W, H)
        H = mu_ref.update_h(X, W, H)

    t0 = time.perf_counter()
    one()
    per = max(time.perf_counter() - t0, 1e-6)
    n = int(max(2, min(200, budget_s / per)))
    t0 = time.perf_counter()
    for _ in range(n):
        one()
    el = time.perf_counter() - t0
    return n / el, n, el


def cpu_baseline(X, W0, H0, budget_s):
    """Oracle fp32 MU iterations (SK:526-728 arithmetic via oracle/mu_ref.py) on the host cores:
    with the BLAS threads this process is granted (reported as `cores`) and with ONE thread (SURVEY
    §8(d)); the CPU model and BLAS vendor are named.  SURVEY §8(d) asks for os.cpu_count() threads;
    on the GPU box os.cpu_count() counts the whole machine (256 logical CPUs) while one GPU's job is
    granted a 16-CPU share (OMP_NUM_THREADS=16, which the box's rules say to leave as set), so the
    granted share is what is used and `cpu_share` says so."""
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        info = threadpool_info()
        threads = max((i.get("num_threads", 1) for i in info if i.get("user_api") == "blas"), default=1)
        blas = ",".join(sorted({f"{i.get('internal_api')}" for i in info if i.get("user_api") == "blas"}))
    except Exception:  # pragma: no cover
        threadpool_limits = None
        threads, blas = os.cpu_count() or 1, "unknown"
    value, n, el = _time_oracle_mu(X, W0, H0, budget_s)
    one_thread = None
    if threadpool_limits is not None:
        with threadpool_limits(limits=1, user_api="blas"):
            v1, n1, el1 = _time_oracle_mu(X, W0, H0, max(budget_s / 3.0, 1.0))
        one_thread = {"value": round(v1, 4), "unit": "it/s", "cores": 1, "iterations": n1,
                      "seconds": round(el1, 3)}
    return {"value": round(value, 4), "unit": "it/s", "cores": int(threads), "kind": "port",
            "sample": f"{n} MU iterations (after 1 untimed) of oracle/mu_ref.py update_w+update_h, "
                      f"NumPy fp32 ({blas} BLAS, {threads} threads), on the same "
                      f"{X.shape[0]}x{X.shape[1]} k={W0.shape[1]} X as the GPU run",
            "seconds": round(el, 3), "cpu_model": cpu_model(), "logical_cpus": os.cpu_count(),
            "blas": blas, "one_thread": one_thread,
            "cpu_share": (f"{threads} BLAS threads = the CPU share granted to this job "
                          f"(OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}); "
                          f"os.cpu_count() = {os.cpu_count()} counts the whole host")}


def cpu_baseline_als(X, W0, H0, delta, lam, budget_s):
    """The ALS oracle (oracle/als_ref.py, scipy NNLS per sample) on a bounded row sample, scaled
    to iterations/s of the full problem (the per-sample solves dominate and scale linearly)."""
    from oracle import als_ref
    n = X.shape[0]
    rows = 2000
    Xs = X[:rows].astype(np.float64)
    H = H0.astype(np.float64)
    t0 = time.perf_counter()
    it = 0
    while True:
        W = als_ref.fcls_w(Xs, H, delta)
        H = als_ref.smooth_h_sweep(W.T @ Xs, W.T @ W, H, lam)
        it += 1
        el = time.perf_counter() - t0
        if el > budget_s or it >= 50:
            break
    per_it_full = el / it * (n / rows)
    return {"value": round(1.0 / per_it_full, 6), "unit": "it/s", "cores": 1, "kind": "port",
            "sample": f"{it} ALS iterations of oracle/als_ref.py (scipy.optimize.nnls per sample, "
                      f"fp64, 1 thread) on the first {rows} of the {n} rows, scaled by {n}/{rows}",
            "seconds": round(el, 3), "cpu_model": cpu_model(), "logical_cpus": os.cpu_count()}


def validate_exchange(plan, W0, H0d, n=20):
    """Set up the in-launch exchange and check it against the RCCL path from the same start:
    n iterations each way; every rank must end with bit-identical H, both paths must agree to fp64
    summation-order noise, and no launch may report an error.  Leaves the plan at (W0, H0) on the
    path to time.  Returns a status string."""
    import torch
    import torch.distributed as dist
    dev = plan.device
    try:
        plan.enable_exchange()
    except Exception as e:  # every rank raises together (enable_exchange agrees collectively)
        return f"unavailable ({str(e)[:300]}); RCCL path timed"
    fail, why = 0.0, ""
    try:
        plan.iterate(n)
        torch.cuda.synchronize()
        plan.check_sync_error()
    except Exception as e:
        fail, why = 1.0, str(e)[:200]
    Hx, Wx = plan.H64.clone(), plan.W.clone()
    plan.exchange, plan.persistent = False, False
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(H0d)
    plan.iterate(n)  # shard steps + RCCL all_reduce
    torch.cuda.synchronize()
    dH = float((Hx - plan.H64).norm() / plan.H64.norm())
    dW = float((Wx.double() - plan.W.double()).norm() / max(float(plan.W.double().norm()), 1e-300))
    hmax, hmin = Hx.clone(), Hx.clone()
    dist.all_reduce(hmax, op=dist.ReduceOp.MAX, group=plan.group)
    dist.all_reduce(hmin, op=dist.ReduceOp.MIN, group=plan.group)
    same = bool(torch.equal(hmax, hmin))
    # the two paths may run different kernels (the exchange: the persistent launch; RCCL: one
    # shard-step launch per iteration), whose fp32 partial sums are grouped differently: agreement
    # to that noise, the parity bar's hundredth
    # (the constrained ALS and the weighted MU: their per-iteration kernels sum differently again and
    # the ALS's exact FCLS amplifies that noise by cond(Q_PP): the parity bar itself)
    bar = 1e-6 if type(plan).__name__ == "MUPlan" else 1e-5
    bad = fail or (not same) or not (dH < bar and dW < bar)
    st = torch.tensor([1.0 if bad else 0.0, dH, dW], dtype=torch.float64, device=dev)
    dist.all_reduce(st, op=dist.ReduceOp.MAX, group=plan.group)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(H0d)
    torch.cuda.synchronize()
    if float(st[0]) != 0.0:
        plan.disable_exchange()
        return (f"failed validation (error: {why or 'none'}, ranks identical: {same}, rel diff vs "
                f"RCCL path H {float(st[1]):.2e} W {float(st[2]):.2e}); RCCL path timed")
    plan.exchange, plan.persistent = True, True
    return (f"validated over {n} iterations: H identical on all ranks, rel diff vs the RCCL path "
            f"H {float(st[1]):.2e} W {float(st[2]):.2e}")


def any_rank(flag: bool, world: int, dev) -> bool:
    """True on every rank when `flag` is True on any rank (a MAX all-reduce; identity at N = 1)."""
    if world == 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64,
                     device="cpu" if dist.get_backend() == "gloo" else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]) != 0.0


def rank0_says(flag: bool, world: int, dev) -> bool:
    """Rank 0's `flag`, on every rank (a broadcast; identity at N = 1)."""
    if world == 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64,
                     device="cpu" if dist.get_backend() == "gloo" else dev)
    dist.broadcast(t, src=0)
    return float(t[0]) != 0.0


def clock_ramp(plan, seconds: float, world: int, dev, sync, trip: int = 100) -> tuple[float, int]:
    """Untimed iterations on copies of W / H until `seconds` of wall time have passed on RANK 0's
    clock: before every trip rank 0 broadcasts whether to go on, so every rank issues the same
    launches (per-rank clocks could give one rank an extra 100-iteration trip, which on
    the exchange path spins its launch into a timeout and on the RCCL path mis-pairs collectives).
    The plan's state is restored afterwards.  Returns (seconds, trips)."""
    W_keep = plan.W.clone()
    H_keep = plan.H64.clone()
    t_r = time.perf_counter()
    trips = 0
    while rank0_says(time.perf_counter() - t_r < seconds, world, dev):
        plan.iterate(trip)
        sync()
        trips += 1
    el = time.perf_counter() - t_r
    plan.W.copy_(W_keep)
    plan.H64.copy_(H_keep)
    if hasattr(plan, "refresh_basis"):
        plan.refresh_basis()
    sync()
    return el, trips


def load_traffic(path, n_rows, F, k, variant=""):
    """PMC-measured HBM bytes of ONE iteration of the dominant kernel (tools/pmc_traffic.py), keyed by
    the shape and the solver variant ("_als", "_w" for the weighted MU, "" for the MU)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None, None
    key = f"{n_rows}x{F}_k{k}{variant}"
    ent = d.get(key)
    if not ent:
        return None, None
    per_it = ent.get("hbm_bytes_per_iteration", ent.get("hbm_bytes_per_launch"))
    return per_it, ent.get("source")


def launcher_decision(gpus, env, device_count: int, backend: str):
    """How `bench.py --gpus N` runs (never time one rank and call it N):
    ("run", None) — this process is a rank of a world of exactly N (a launcher set WORLD_SIZE = N, or
    N = 1 without one; --gpus omitted: whatever WORLD_SIZE the launcher set); ("spawn",
    None) — no launcher and N > 1: start N ranks as children through torch.distributed.run;
    ("refuse", why) — WORLD_SIZE disagrees with --gpus, or RCCL would need more devices than are
    visible."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if gpus is not None and int(ws) != gpus:
            return "refuse", (f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks: the line would "
                              f"report the wrong GPU count")
        return "run", None
    if gpus is None or gpus <= 1:
        return "run", None
    if backend == "nccl" and device_count < gpus:
        return "refuse", (f"--gpus {gpus} needs {gpus} visible devices for RCCL, {device_count} visible "
                          f"(--backend gloo lets ranks share a device)")
    return "spawn", None


def spawn_ranks(gpus: int) -> int:
    """Start `gpus` ranks of this script through torch.distributed.run (one process per GPU, the
    driver's own launch line) from this parent, which never touches the GPU; returns their exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] no launcher: starting {gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def state_problem(err, W, H) -> str | None:
    """Why the measured state is not a valid factorisation (None when it is): the final Frobenius
    error must be finite, and W / H finite and non-negative (a NaN-producing
    kernel variant was once timed and reported with exit status 0).  W, H: torch tensors or arrays."""
    import torch
    if err is None or not math.isfinite(float(err)):
        return f"final Frobenius error is {err}"
    for name, t in (("W", W), ("H", H)):
        t = torch.as_tensor(t)
        if t.numel() == 0:
            continue
        if not bool(torch.isfinite(t).all()):
            return f"{name} has a non-finite entry"
        if bool((t < 0).any()):
            return f"{name} has a negative entry"
    return None


def final_verdict(plan, world: int, dev):
    """(final error, problem or None) of the plan's measured state, agreed over the ranks: when any
    rank's state is not a valid factorisation every rank gets a problem (and refuses together)."""
    err = plan.frobenius_error()
    problem = state_problem(err, plan.W, plan.H64)
    if any_rank(problem is not None, world, dev):
        problem = problem or "another rank's state is not a valid factorisation"
    return err, problem


def refuse_result(why: str, rank: int):
    """Exit with EXIT_BROKEN and no JSON line (every rank calls it together)."""
    print(f"[bench] rank {rank}: refusing to report: {why}", file=sys.stderr, flush=True)
    sys.exit(EXIT_BROKEN)


def row_unit(n_rows: int) -> str:
    """Label of the weak-scaling unit: the rows of one shard ('1e6' for cfg2's 1,000,000)."""
    m = math.log10(n_rows) if n_rows > 0 else 0.0
    if n_rows > 0 and abs(m - round(m)) < 1e-12:
        return f"1e{int(round(m))}"
    return str(n_rows)


def line_value(scaling: str, world: int, n_rows: int, k_done: int, elapsed: float):
    """(value, unit) of the JSON line.  weak: world x k_done / elapsed in '<rows>-row it/s' — the
    iterations of one <rows>-row shard completed per second over all ranks (at N = 1 the it/s of the
    problem run; ADVICE r4: no rescaling by rows / 1e6); strong: k_done / elapsed in it/s of the
    whole problem."""
    if scaling == "strong":
        return k_done / elapsed, "it/s"
    return world * k_done / elapsed, f"{row_unit(n_rows)}-row it/s"


class Ctx:
    """Where a measurement runs: this process's rank in a world (group None at world 1)."""

    def __init__(self, world, rank, dev, group, dist_path, backend):
        self.world, self.rank, self.dev, self.group = world, rank, dev, group
        self.dist_path, self.backend = dist_path, backend

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier(group=self.group)


def make_problem(args, rows_total: int, lo: int, hi: int, seed: int):
    """Host arrays of rows [lo, hi) of the seeded synthetic problem with rows_total rows (X, W0, H0,
    weights or None).  Rows are drawn for the whole problem, so any split of it sees the same X."""
    from cnmf_amd.synthetic import iop_spectra, random_init
    np_dt = np.float64 if args.dtype == "f64" else np.float32
    X = iop_spectra(rows_total, args.features, seed=seed, dtype=np_dt)
    W0, H0 = random_init(X, args.k, 42 + seed)
    Mw = None
    if args.weighted:
        rng = np.random.default_rng(seed)
        Mw = (rng.uniform(0.2, 2.0, X.shape) * (rng.random(X.shape) >= 0.3)).astype(np.float32)[lo:hi]
    if lo != 0 or hi != rows_total:
        X, W0 = np.ascontiguousarray(X[lo:hi]), np.ascontiguousarray(W0[lo:hi])
    return X, W0, H0, Mw


def make_plan(args, ctx, X, W0, H0, Mw, Xd=None):
    """The plan of one measurement on ctx's device (X copied to HBM unless Xd is given); H0 is
    broadcast from rank 0.  Returns (plan, Xt host tensor, H0 on the device)."""
    import torch
    import torch.distributed as dist
    from cnmf_amd.solver import ALSPlan, MUPlan, WeightedMUPlan
    Xt = torch.from_numpy(X)
    if args.dtype == "bf16":
        Xt = Xt.to(torch.bfloat16)
    if Xd is None:
        Xd = Xt.to(ctx.dev)
    H0d = torch.from_numpy(H0).to(ctx.dev)
    if ctx.world > 1:
        dist.broadcast(H0d, src=0, group=ctx.group)
    if args.weighted:
        plan = WeightedMUPlan(Xd, torch.from_numpy(Mw).to(ctx.dev), args.k, group=ctx.group)
    elif args.solver == "als":
        plan = ALSPlan(Xd, args.k, sum_to_one=args.sum_to_one, smoothness=args.smoothness, group=ctx.group)
    else:
        plan = MUPlan(Xd, args.k, group=ctx.group)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(H0d)
    return plan, Xt, H0d


def measure(args, ctx, plan, W0, H0d, K, warmup, ramp_seconds, tune=True):
    """Warm up, ramp the clock, tune the layout, then time exactly K steps of `plan` bracketed by a
    barrier + synchronisation on both sides (max over ranks).  Returns a dict of the timing, the
    paths taken and the measured state's verdict (`problem`, agreed over the ranks)."""
    import torch
    from cnmf_amd.solver import agree_max
    world, rank, dev = ctx.world, ctx.rank, ctx.dev
    exchange = None
    if ctx.dist_path and args.exchange == "auto" and plan.exchange_shape:
        exchange = validate_exchange(plan, W0, H0d)
        print(f"[rank {rank}] in-launch exchange ({plan.n_rows} rows): {exchange}", file=sys.stderr, flush=True)
    elif args.dist and args.solver == "mu" and not args.weighted:
        plan.use_shard_steps()
    torch.cuda.synchronize()

    plan.iterate(warmup)
    torch.cuda.synchronize()
    if getattr(plan, "exchange", False):  # a failed warmup launch falls back before anything is timed
        fail = False
        try:
            plan.check_sync_error()
        except Exception as e:
            fail = True
            print(f"[rank {rank}] exchange warmup failed: {e}", file=sys.stderr, flush=True)
        if any_rank(fail, world, dev):
            plan.disable_exchange()
            exchange = "failed in warmup; RCCL path timed"
            plan.set_W(torch.from_numpy(W0))
            plan.set_H(H0d)
            plan.iterate(warmup)
            torch.cuda.synchronize()

    # clock ramp: after idle the chip runs its first tens of ms of work at lower clocks (r01/r02:
    # a 20-step timing after a 5-step warmup read 66 us per iteration against 57-58 us once warm);
    # run untimed iterations on copies of W / H until ramp_s of GPU time has passed
    ramp_s, ramp_trips = 0.0, 0
    if ramp_seconds > 0:
        ramp_s, ramp_trips = clock_ramp(plan, ramp_seconds, world, dev, torch.cuda.synchronize)
        plan.check_sync_error()

    # the persistent launch has several layouts whose order can differ between boxes: time them on
    # this box (warm clocks; copies of W / H, so the state is unchanged) and keep the fastest.  The
    # choice is collective (MUPlan.tune max-reduces the times over the ranks): every rank launches
    # the same layout
    tuned = {}
    if args.layout > 0 and args.solver == "mu" and not args.weighted:
        plan.set_layout(args.layout)
    elif tune and args.solver == "mu" and getattr(plan, "layouts", ()) and not args.no_tune and not args.weighted:
        tuned = plan.tune(n_iter=100, rounds=2)
        print(f"[rank {rank}] persistent layouts (us/iteration): {tuned}", file=sys.stderr, flush=True)
    layout = plan.describe() if plan.persistent else None
    layouts = [getattr(plan, "layout", None)]
    if world > 1:
        import torch.distributed as dist
        layouts = [None] * world
        dist.all_gather_object(layouts, getattr(plan, "layout", None), group=ctx.group)

    tol_result = {}

    def timed():
        persistent = plan.persistent and (world == 1 or plan.exchange)
        # two events around the whole timed stretch for the single-GPU MU launches too (cfg4's pass +
        # reduction + update per iteration): an event record between every iteration's launches
        # stretched cfg4's timed iterations by ~14 us over tune()'s (profiles/r04/e/)
        whole = persistent or (world == 1 and type(plan).__name__ == "MUPlan" and not plan.shard_steps)
        events = [torch.cuda.Event(enable_timing=True) for _ in range(2 if whole else 2 * K)]
        stream = torch.cuda.current_stream(dev)
        for e in events:  # creates the HIP events (outside the timed region)
            e.record(stream)
        # the K iterations' library call with its arguments marshalled here, outside the timed region
        prep = plan.prepare_device_tol(K, args.tol, pass_events=events) if (
            args.tol > 0 and persistent and hasattr(plan, "prepare_device_tol")) else None
        if args.tol > 0 and prep is None:
            raise SystemExit("--tol needs a plan whose shape takes the device tolerance test (wave tiles)")
        if prep is not None:
            launch, finish = prep

            def run():
                launch()
                tol_result["n_iter"], tol_result["errors"] = finish()  # the one synchronisation
        else:
            run = plan.prepare(K, pass_events=events)
        torch.cuda.synchronize()
        if args.settle_ms > 0:
            time.sleep(args.settle_ms / 1e3)
        ctx.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        return persistent, events, elapsed, whole

    persistent, events, elapsed, whole = timed()
    if getattr(plan, "exchange", False):  # a failed exchange launch: every rank re-times on RCCL
        fail = False
        try:
            plan.check_sync_error()
        except Exception as e:
            fail = True
            print(f"[rank {rank}] exchange launch failed: {e}", file=sys.stderr, flush=True)
        if any_rank(fail, world, dev):
            plan.disable_exchange()
            exchange = "failed in the timed launch; RCCL path re-timed"
            plan.set_W(torch.from_numpy(W0))
            plan.set_H(H0d)
            plan.iterate(warmup)
            torch.cuda.synchronize()
            persistent, events, elapsed, whole = timed()
    plan.check_sync_error()
    if persistent:  # ONE launch ran all K iterations (pass + in-launch reduction + basis update)
        launches = 1
        avg_launch_s = events[0].elapsed_time(events[1]) / 1e3
    elif whole:  # K iterations of launches between two events: the average iteration
        launches = K
        avg_launch_s = events[0].elapsed_time(events[1]) / 1e3 / K
    else:
        launches = K
        avg_launch_s = float(np.mean([events[2 * i].elapsed_time(events[2 * i + 1])
                                      for i in range(K)])) / 1e3
    elapsed, avg_launch_s_max = agree_max([elapsed, avg_launch_s], ctx.group if world > 1 else None, dev)

    err, problem = final_verdict(plan, world, dev)
    return {"persistent": persistent, "whole": whole, "elapsed": elapsed, "avg_launch_s": avg_launch_s,
            "avg_launch_s_max": avg_launch_s_max, "launches": launches, "exchange": exchange,
            "layout": layout, "layouts": layouts, "tuned": tuned, "ramp_s": ramp_s,
            "ramp_trips": ramp_trips, "tol_result": tol_result, "err": err, "problem": problem,
            "k_done": tol_result.get("n_iter", K)}


def bytes_per_iteration(args, n_rows: int) -> int:
    """Algorithmic HBM bytes of one pass over n_rows: X once, W read and written
    (+ the weights for the weighted MU)."""
    sx = {"f32": 4, "f64": 8, "bf16": 2}[args.dtype]
    sw = 8 if args.dtype == "f64" else 4
    return n_rows * (args.features * sx + 2 * args.k * sw) + (n_rows * args.features * 4 if args.weighted else 0)


def strong_block(args, res, n_rows_shard: int, rows: int, world: int, n1=None):
    """The line's `strong` key: the fixed rows x F problem over `world` ranks (res) and on one GPU
    (n1: the same problem on rank 0's GPU alone, in the same run; at N = 1 res itself)."""
    us = res["elapsed"] / res["k_done"] * 1e6
    per_launch = res["avg_launch_s_max"] / (res["k_done"] if res["persistent"] else 1)
    frac = bytes_per_iteration(args, n_rows_shard) / per_launch / 1e9 / HBM_PEAK_GBS
    out = {"rows": rows, "ranks": world, "rows_per_gpu_max": n_rows_shard,
           "it_s": round(res["k_done"] / res["elapsed"], 2), "us_per_iteration": round(us, 3),
           "frac": round(frac, 4), "exchange": res["exchange"],
           "layout": res["layout"]}
    if n1 is not None:
        us1 = n1["elapsed"] / n1["k_done"] * 1e6
        out["n1_it_s"] = round(n1["k_done"] / n1["elapsed"], 2)
        out["n1_us_per_iteration"] = round(us1, 3)
        out["speedup_vs_n1"] = round(us1 / us, 3)
    return out


def main():
    args = parse()
    import torch
    # decided before any HIP call (device_count does not initialise the runtime on this image)
    how, why = launcher_decision(args.gpus, os.environ, torch.cuda.device_count(), args.backend)
    if how == "refuse":
        print(f"[bench] refused: {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    if how == "spawn":
        sys.exit(spawn_ranks(args.gpus))
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    dist_path = world > 1 or args.dist
    # one GPU per rank; with --backend gloo several ranks may share a GPU (local % device count)
    n_dev = max(torch.cuda.device_count(), 1)
    local_dev = local % n_dev
    if dist_path:
        torch.cuda.set_device(local_dev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_dev)
    torch.cuda.set_device(dev)
    ctx = Ctx(world, rank, dev, dist.group.WORLD if dist_path else None, dist_path, args.backend)

    from cnmf_amd.distributed import shard_bounds

    F, k, K = args.features, args.k, args.steps
    if args.scaling == "strong":  # the fixed problem (cfg2's X), 64-row-aligned shards (persistent tiles)
        lo, hi = shard_bounds(args.rows, world, rank, align=64)
        X, W0, H0, Mw = make_problem(args, args.rows, lo, hi, seed=0)
    else:  # every rank its own rows (seed = rank: rank 0's are exactly cfg2's X)
        X, W0, H0, Mw = make_problem(args, args.rows, 0, args.rows, seed=rank)
    n_rows = X.shape[0]
    plan, Xt, H0d = make_plan(args, ctx, X, W0, H0, Mw)
    res = measure(args, ctx, plan, W0, H0d, K, args.warmup, args.ramp_seconds)
    if res["problem"]:
        refuse_result(res["problem"], rank)

    # north_star's strong-scaling figure on one clock: the metric's V = strong_rows problem split over
    # the same ranks, and on rank 0's GPU alone (ranks > 0 wait at the barrier meanwhile)
    strong = None
    S = args.strong_rows
    # ranks that share a device (--backend gloo on fewer GPUs): the default 1e6-row split is not
    # co-resident there, so it is recorded as not measured unless --strong-rows asks for it
    n_gpus = min(world, n_dev) if args.backend == "gloo" and dist_path else world
    strong_skipped = None
    if S is None:
        S = 1_000_000
        if world > 1 and n_gpus < world:
            S, strong_skipped = 0, (f"not measured: {world} ranks share {n_gpus} GPU(s) (pass --strong-rows "
                                    f"to split a problem whose per-rank grids are co-resident)")
    if world > 1 and S > 0:
        if args.scaling == "strong" and S == args.rows:
            sres, s_rows, s_plan = res, n_rows, None
        else:
            slo, shi = shard_bounds(S, world, rank, align=64)
            Xs, W0s, H0s, Mws = make_problem(args, S, slo, shi, seed=0)
            s_plan, _, H0sd = make_plan(args, ctx, Xs, W0s, H0s, Mws)
            sres = measure(args, ctx, s_plan, W0s, H0sd, K, min(args.warmup, 200), 0.1)
            s_rows = Xs.shape[0]
            if sres["problem"]:
                refuse_result("strong split: " + sres["problem"], rank)
        s_rows_max = int(max(shard_bounds(S, world, r, align=64)[1] - shard_bounds(S, world, r, align=64)[0]
                             for r in range(world)))
        n1 = None
        if s_plan is not None:
            s_plan.release()
        if rank == 0:
            ctx1 = Ctx(1, 0, dev, None, False, args.backend)
            X1, W01, H01, Mw1 = make_problem(args, S, 0, S, seed=0)
            p1, _, H01d = make_plan(args, ctx1, X1, W01, H01, Mw1)
            n1 = measure(args, ctx1, p1, W01, H01d, K, min(args.warmup, 200), 0.1)
            del p1
        n1_bad = rank == 0 and n1["problem"] is not None
        if any_rank(n1_bad, world, dev):
            refuse_result("one-GPU reference of the strong split: " + (n1["problem"] if n1_bad else "rank 0"), rank)
        if rank == 0:
            strong = strong_block(args, sres, s_rows_max, S, world, n1)
    elif strong_skipped:
        strong = {"skipped": strong_skipped}
    elif world == 1 and S > 0 and n_rows == S and not args.dist:
        strong = strong_block(args, res, n_rows, S, 1)
        strong["n1_it_s"], strong["n1_us_per_iteration"], strong["speedup_vs_n1"] = (
            strong["it_s"], strong["us_per_iteration"], 1.0)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    persistent = res["persistent"]
    tol_result = res["tol_result"]
    elapsed, avg_pass_s, avg_pass_s_max = res["elapsed"], res["avg_launch_s"], res["avg_launch_s_max"]
    bytes_per_pass = bytes_per_iteration(args, n_rows)
    iters_per_launch = tol_result.get("n_iter", K) if persistent else 1
    bytes_per_launch = bytes_per_pass * iters_per_launch
    achieved = bytes_per_launch / avg_pass_s_max / 1e9
    layout = res["layout"]

    variant = "_als" if args.solver == "als" else ("_w" if args.weighted else "")
    traffic, traffic_src = load_traffic(args.traffic_json, n_rows, F, k, variant)
    if traffic is not None:
        traffic = traffic * iters_per_launch
    if args.weighted and persistent:
        kname = ("wmu_iter_wt_kernel (persistent: K weighted iterations of pass + in-launch reduction + "
                 "H-step per launch)")
    elif args.weighted:
        kname = "weighted MU pass (wmu_pass_kernel: W-step + [W'ᵀ(M∘X) | W'ᵀ(M∘(W'H))])"
    elif args.solver == "als" and persistent:
        kname = ("als_iter_wt_kernel (persistent: K constrained-ALS iterations of W-step pass + in-launch "
                 "reduction + NNLS H-step per launch)")
    elif args.solver == "als":
        kname = "constrained-ALS W-step pass (mu_pass_kernel<..., ALS>: exact FCLS per sample + [WᵀX|WᵀW])"
    elif persistent:
        kbase = (layout or "").split("<")[0].split(":")[0].strip() or "persistent kernel"
        if world == 1:
            kname = (f"{kbase} (persistent: K iterations of pass + in-launch reduction + basis "
                     "update per launch)")
        else:
            kname = (f"{kbase}<..., MULTI> (persistent, one launch per rank: K iterations of "
                     "pass + in-launch reduction + peer all-reduce over xGMI + basis update)")
    elif plan.persistent_shape:
        kname = ("mu_iter_sl_kernel shard step (one iteration per launch: pending basis update, "
                 "pass, in-launch reduction; all_reduce between launches)")
    else:
        kname = ("iteration as launches (sample pass + reduction + basis update; events around the whole "
                 "iteration)")
    roofline = {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "algorithmic_bytes_per_iteration": bytes_per_pass,
                "launches_timed": res["launches"], "iterations_per_launch": iters_per_launch,
                "avg_launch_us": round(avg_pass_s * 1e6, 2),
                "avg_us_per_iteration_in_launch": round(avg_pass_s / iters_per_launch * 1e6, 2),
                "max_over_ranks_avg_launch_us": round(avg_pass_s_max * 1e6, 2)}

    cpu = None
    if world == 1 and not args.no_cpu and not args.weighted:
        Xc = X if args.dtype != "bf16" else Xt.float().numpy()
        if args.solver == "als":
            cpu = cpu_baseline_als(Xc, W0, H0, args.sum_to_one, args.smoothness, args.cpu_seconds)
        else:
            cpu = cpu_baseline(Xc, W0, H0, args.cpu_seconds)

    K_done = res["k_done"]  # --tol: the iterations the fit actually ran
    value, unit = line_value(args.scaling, world, n_rows, K_done, elapsed)
    n_rows_total = args.rows if args.scaling == "strong" else world * n_rows
    if args.weighted:
        metric = "weighted MU iterations/sec (V=1e6x81 k=4 with per-element weights, 30 % zero)"
        workload = (f"weighted / masked MU (SURVEY 8f row 2, tol=0) on V={n_rows}x{F} per GPU, k={k}, "
                    f"f32 synthetic IOP spectra, synthetic weights U(0.2, 2) with 30 % zeros")
    elif args.solver == "als":
        metric = ("constrained-ALS iterations/sec (cfg5: V=1e6x81 k=4, sum-to-one + smoothness) & "
                  "achieved HBM GB/s of the W-step pass vs peak")
        workload = (f"cfg5: constrained ALS (FCLS W-step delta={args.sum_to_one}, smoothness "
                    f"lambda={args.smoothness} NNLS basis sweep, tol=0) on V={n_rows}x{F} per GPU, k={k}, "
                    f"{args.dtype} synthetic IOP spectra")
    else:
        cfg = {(1_000_000, 81, 4, "f32"): "cfg2", (10_000_000, 81, 8, "f32"): "cfg3",
               (1_250_000, 81, 8, "f32"): "cfg3 (one GPU's shard)",
               (1_000_000, 300, 16, "bf16"): "cfg4"}.get((args.rows, F, k, args.dtype), "custom")
        metric = ("MU iterations/sec & achieved HBM GB/s vs peak, V=1e6×81 k=4, 1/2/4/8 GPU"
                  if cfg == "cfg2" else f"MU iterations/sec & achieved HBM GB/s vs peak, {cfg}")
        if args.scaling == "strong":
            workload = (f"{cfg}: MU (Frobenius, tol={args.tol:g}) on V={args.rows}x{F} in total, k={k}, "
                        f"{args.dtype} synthetic IOP spectra, rows split over {world} GPU(s) in "
                        f"64-row-aligned shards (strong scaling: the problem is fixed; value = its it/s)")
        else:
            workload = (f"{cfg}: MU (Frobenius, tol={args.tol:g}) on V={n_rows}x{F} per GPU, k={k}, "
                        f"{args.dtype} synthetic IOP spectra (weak scaling: every GPU owns its own "
                        f"{n_rows} rows of one {world * n_rows}-row problem, [WᵀX | WᵀW] all-reduced "
                        f"every iteration; value = {world} x the it/s of that problem = iterations of "
                        f"one {n_rows}-row shard per second over all ranks)")
    # ranks that share a device (--backend gloo on fewer GPUs) are not more GPUs: n_gpus above
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": n_gpus,
        "ranks": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / max(K_done, 1) * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": {"f32": "f32", "f64": "f64", "bf16": "bf16 X / f32 W"}[args.dtype],
        "data": "synthetic",
        "config": {"workload": workload,
                   "n_rows_total": n_rows_total,
                   "n_rows_per_gpu": n_rows, "n_features": F, "k": k,
                   "parallelism": f"dp{world} (row shards, all_reduce of k(F+k) fp64"
                                  + (", in-launch over xGMI)" if plan.exchange else ", RCCL)")
                                  + (" [--dist: multi-GPU path at one rank]" if args.dist and world == 1 else "")
                                  + (f" [{world} ranks on {n_gpus} GPU(s): diagnostic]" if n_gpus < world else ""),
                   "exchange": res["exchange"],
                   "persistent_layout": layout if plan.persistent else None,
                   "layout_per_rank": res["layouts"],
                   "backend": (args.backend if dist_path else None),
                   "layout_tuning_us_per_iteration": {str(kk): round(v, 2) for kk, v in res["tuned"].items()} or None,
                   "clock_ramp_s": round(res["ramp_s"], 3), "clock_ramp_trips": res["ramp_trips"],
                   "tol": args.tol or None,
                   "tol_n_iter": tol_result.get("n_iter"),
                   "tol_errors": tol_result.get("errors")},
        "roofline": roofline,
        "strong": strong,
        "cpu_baseline": cpu,
        "final_frobenius_error": res["err"],
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
