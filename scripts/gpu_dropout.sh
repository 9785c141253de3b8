#!/bin/bash
# GPU: dropout / Philox parity tests, then the cfg3 bench plain and with dropout 0.1.
# usage: bash scripts/gpu_dropout.sh TAG
set -o pipefail
TAG=${1:-dropout}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "dropout or philox" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for leg in "dropout:--dropout 0.1" "plain:"; do
  n=${leg%%:*}; a=${leg#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', d['value'], 'fwd', d['fwd_tflops'], 'bwd', d['bwd_tflops'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
