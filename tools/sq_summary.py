"""Per-tile instruction mix and stall shares of one kernel from three rocprofv3 --pmc SQ passes.

    python tools/sq_summary.py --db gpurun_out/<dir>/{p1,p2,p3}/run_results.db --kernel als_iter_wt \\
        --tiles 1250000 --out profiles/r06/sq/als_sq_summary.json [--note "..."]

--tiles: wave tiles per launch (the pass kernel's launches are averaged).  Counter passes (each its own
run, rocprofv3 never splits a pass):
  p1  SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_LDS, SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES, SQ_WAIT_ANY,
      SQ_WAIT_INST_ANY, SQ_WAVES, SQ_WAVE_CYCLES
  p2  SQ_INSTS_LDS, SQ_INSTS_SALU, SQ_INSTS_SMEM, SQ_INSTS_VALU, SQ_INSTS_VMEM_RD, SQ_INSTS_VMEM_WR,
      SQ_LDS_BANK_CONFLICT, SQ_WAIT_INST_LDS
  p3  GRBM_COUNT, GRBM_GUI_ACTIVE, SQ_ACTIVE_INST_MISC, SQ_INSTS_FLAT, SQ_INSTS_MFMA,
      SQ_INSTS_VALU_FMA_F64, SQ_INSTS_VALU_MFMA_F64, SQ_VALU_MFMA_BUSY_CYCLES
"""
import argparse
import json
import sqlite3


def per_launch(db, kernel):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                     "group by dispatch_id, counter_name").fetchall()
    acc, disp = {}, set()
    for d, name, ctr, v in rows:
        if kernel in name:
            acc[ctr] = acc.get(ctr, 0.0) + float(v)
            disp.add(d)
    n = max(1, len(disp))
    return {k: v / n for k, v in acc.items()}, len(disp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--db", nargs=3, required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--tiles", type=float, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    raw, launches = {}, []
    for db in a.db:
        d, n = per_launch(db, a.kernel)
        raw.update(d)
        launches.append(n)
    T = a.tiles
    g = raw.get
    out = {
        "kernel_substring": a.kernel,
        "launches_per_pass": launches,
        "tiles_per_launch": T,
        "valu_per_tile": round(g("SQ_INSTS_VALU", 0) / T, 1),
        "mfma_per_tile": round(g("SQ_INSTS_MFMA", 0) / T, 1),
        "lds_per_tile": round(g("SQ_INSTS_LDS", 0) / T, 1),
        "salu_per_tile": round(g("SQ_INSTS_SALU", 0) / T, 1),
        "vmem_rd_per_tile": round(g("SQ_INSTS_VMEM_RD", 0) / T, 2),
        "vmem_wr_per_tile": round(g("SQ_INSTS_VMEM_WR", 0) / T, 2),
        "valu_fma_f64_per_tile": round(g("SQ_INSTS_VALU_FMA_F64", 0) / T, 1),
        "lds_bank_conflict_cycles_per_lds_instr": round(g("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, g("SQ_INSTS_LDS", 1)), 3),
        "lds_bank_conflict_share_of_lds_active": round(g("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, g("SQ_ACTIVE_INST_LDS", 1)), 3),
        "wait_any_over_wave_cycles": round(g("SQ_WAIT_ANY", 0) / max(1.0, g("SQ_WAVE_CYCLES", 1)), 3),
        "valu_active_over_wave_cycles": round(g("SQ_ACTIVE_INST_VALU", 0) / max(1.0, g("SQ_WAVE_CYCLES", 1)), 3),
        "note": a.note,
        "raw_per_launch": {k: round(v, 1) for k, v in sorted(raw.items())},
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "raw_per_launch"}))


if __name__ == "__main__":
    main()
