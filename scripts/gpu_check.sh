#!/bin/bash
# GPU round-trip used during development: parity tests, bench, rocprofv3 kernel stats.
# usage: bash scripts/gpu_check.sh TAG [stride]
set -o pipefail
TAG=${1:-dev}
STRIDE=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FA2_GRID_STRIDE=$STRIDE timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --maxfail=20 -rf > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 $OUT/tests.log | cut -c1-300
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | head -6
