#!/bin/bash
# k = 8 (cfg3's 1.25e6-row shard, W streamed): counter passes of the VALU wave tiles (layout 4) and
# the matrix-core wave tiles (layout 5), each pass its own run (<= 8 SQ / 2 GRBM counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-pmc_mf8}
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv"
for L in 4 5; do
  A="--rows 1250000 --k 8 --iters 20 --layout $L"
  $P --stats -d $D/s$L -o s$L -- python3 tools/prof_pass.py $A > $D/s$L.log 2>&1 &&
  $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $D/a$L -o a$L -- python3 tools/prof_pass.py $A > $D/a$L.log 2>&1 &&
  $P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC -d $D/b$L -o b$L -- python3 tools/prof_pass.py $A > $D/b$L.log 2>&1 &&
  $P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE GRBM_COUNT -d $D/c$L -o c$L -- python3 tools/prof_pass.py $A > $D/c$L.log 2>&1 || { echo "failed at layout $L"; exit 1; }
done
python3 - $D <<'PY'
import csv, glob, sys, collections
D = sys.argv[1]
for L in (4, 5):
    tot = collections.defaultdict(float)
    for f in glob.glob(f"{D}/[abc]{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "iter" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print("layout", L, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
