#!/bin/bash
# GPU: per-tile vs per-item cost of the hand-placed kernels (sequence scaling at fixed tokens,
# hp and old kernels) and SQ / GRBM counters of the hp forward and backward at cfg3.
# usage: bash scripts/gpu_hp_diag.sh TAG
set -o pipefail
TAG=${1:-diag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export FA2_DKDV_HP=1 FA2_DQ_HP=1
for c in 1 0; do
  timeout -k 10 200 python -u scripts/hp_scaling.py --causal $c > $OUT/scaling_hp_c$c.jsonl 2>&1 || exit $?
  FA2_FWD_HP=0 FA2_DKDV_HP=0 FA2_DQ_HP=0 timeout -k 10 200 python -u scripts/hp_scaling.py --causal $c > $OUT/scaling_old_c$c.jsonl 2>&1 || exit $?
done
cat $OUT/scaling_*.jsonl
n=0
for c in 1 0; do
  for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$n -o run --output-format csv -- python3 scripts/run_kernels.py --reps 3 --causal $c > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT/p$n.log; exit 1; }
    python3 - $OUT/p$n $c <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fa2::" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("<")[0].replace("void fa2::", "") + ":" + r["Counter_Name"]].append(float(r["Counter_Value"]))
print("causal", sys.argv[2], {k: f"{sum(v)/len(v):.4g}" for k, v in sorted(d.items())})
PY
  done
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 scripts/run_kernels.py --reps 5 --causal 1 > $OUT/trace.log 2>&1 || exit $?
cat $(find $OUT/trace -name "*kernel_stats.csv") | cut -c1-200
