#!/bin/bash
# One GPU call of round evidence: full parity suite, smoke(), a bench line per BASELINE config
# (cfg3 default, cfg2, cfg5) and the bias / dropout legs of cfg3, each step under its own limit.
# usage: bash scripts/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export FA2_RTOL_LOG=$OUT/rtol.jsonl
rm -f $FA2_RTOL_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || exit $?
cat $OUT/bench_cfg3.json
timeout -k 10 400 python bench.py --config cfg2 > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || exit $?
cat $OUT/bench_cfg2.json
timeout -k 10 400 python bench.py --config cfg5 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || exit $?
cat $OUT/bench_cfg5.json
timeout -k 10 300 python bench.py --bias --no-cpu-baseline > $OUT/bench_cfg3_bias.json 2> $OUT/bench_bias.err || exit $?
timeout -k 10 300 python bench.py --dropout 0.1 --no-cpu-baseline > $OUT/bench_cfg3_dropout.json 2> $OUT/bench_dropout.err || exit $?
timeout -k 10 300 python bench.py --no-causal --no-cpu-baseline > $OUT/bench_cfg3_noncausal.json 2> $OUT/bench_nc.err || exit $?
for f in bias dropout noncausal; do python -c "import json,sys; d=json.load(open('$OUT/bench_cfg3_$f.json')); print('$f', d['value'], d['fwd_tflops'], d['bwd_tflops'], d['kernels'])"; done
