#!/bin/bash
# GPU: full parity suite, then the cfg3 bench with and without the reference tests' [1,1,S,S]
# bias (causal and not), per-kernel times.  usage: bash scripts/gpu_bias.sh TAG
set -o pipefail
TAG=${1:-bias}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for leg in "plain:" "bias:--bias" "bias_nc:--bias --no-causal" "dropout:--dropout 0.1"; do
  n=${leg%%:*}; a=${leg#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  python -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', d['value'], 'fwd', d['fwd_tflops'], 'bwd', d['bwd_tflops'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
