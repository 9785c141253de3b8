#!/bin/bash
# GPU: hand-placed kernels dev loop -- numerics check (fwd/bwd vs the old kernels and the oracle),
# cfg3 bench A/B (FA2_FWD_HP / FA2_DKDV_HP), optional full suite.
# usage: bash scripts/gpu_hp.sh TAG [fwd,bwd] [suite]
set -o pipefail
TAG=${1:-hp}
WHAT=${2:-fwd,bwd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u tests/hp_check.py $WHAT > $OUT/check.log 2>&1
rc=$?; cat $OUT/check.log; [ $rc -eq 0 ] || exit $rc
export FA2_DKDV_HP=1 FA2_DQ_HP=1
timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench_c.json 2> $OUT/bench_c.err || exit $?
timeout -k 10 240 python bench.py --no-causal --no-cpu-baseline > $OUT/bench_nc.json 2> $OUT/bench_nc.err || exit $?
FA2_DKDV_HP=0 FA2_DQ_HP=0 timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench_c_oldbwd.json 2> $OUT/bench_c_oldbwd.err || exit $?
FA2_FWD_EXACT=0 timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench_c_ps.json 2> $OUT/bench_c_ps.err || exit $?
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], 'fwd', d['fwd_tflops'], 'bwd', d['bwd_tflops'], d['kernels'])"; done
if [ "$3" = "suite" ]; then
  # the suite with the hand-placed backward switched on
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
