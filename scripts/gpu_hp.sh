#!/bin/bash
# GPU: hand-placed forward dev loop -- numerics check, forward A/B bench (hp vs fwd_pipe), suite.
# usage: bash scripts/gpu_hp.sh TAG [suite]
set -o pipefail
TAG=${1:-hp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python -u tests/hp_check.py > $OUT/check.log 2>&1
rc=$?; cat $OUT/check.log; [ $rc -eq 0 ] || exit $rc
for hp in 1 0; do
  FA2_FWD_HP=$hp timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench_c_hp$hp.json 2> $OUT/bench_c_hp$hp.err || exit $?
  FA2_FWD_HP=$hp timeout -k 10 240 python bench.py --no-causal --no-cpu-baseline > $OUT/bench_nc_hp$hp.json 2> $OUT/bench_nc_hp$hp.err || exit $?
done
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], 'fwd', d['fwd_tflops'], d['kernels']['fwd_kernel'])"; done
if [ "$2" = "suite" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
