#!/bin/bash
# GPU parity suite + default bench line, each step under its own time limit.
# usage: bash scripts/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export FA2_RTOL_LOG=$OUT/rtol.jsonl
rm -f $FA2_RTOL_LOG
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
fi
rc=$?
tail -25 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
