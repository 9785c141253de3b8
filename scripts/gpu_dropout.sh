#!/bin/bash
# GPU: dropout / Philox / full-size tests, then the cfg3 dropout bench leg.
set -o pipefail
TAG=${1:-dropout2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "dropout or philox or full_size" --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dropout 0.1 --no-cpu-baseline > $OUT/bench_dropout.json 2> $OUT/bench_dropout.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_dropout.json')); print('dropout', d['value'], 'fwd', d['fwd_tflops'], 'bwd', d['bwd_tflops'], {k: v['ms'] for k, v in d['kernels'].items()})"
