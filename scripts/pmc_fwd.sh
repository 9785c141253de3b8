#!/bin/bash
# SQ / GRBM counters of the forward kernel at cfg3 (causal and not), one pass per counter set.
# usage: bash scripts/pmc_fwd.sh TAG [lib.so]
set -o pipefail
TAG=$1; LIB=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export FA2_AMD_LIB=$LIB
n=0
for c in 0 1; do
  for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$n -o run --output-format csv -- python3 scripts/run_kernels.py --what ${WHAT:-fwd} --reps 3 --causal $c > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT/p$n.log; exit 1; }
    python3 - $OUT/p$n $c <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fa2::" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("<")[0].replace("void fa2::", "") + ":" + r["Counter_Name"]].append(float(r["Counter_Value"]))
print("causal", sys.argv[2], {k: f"{sum(v)/len(v):.4g}" for k, v in d.items()})
PY
  done
done
