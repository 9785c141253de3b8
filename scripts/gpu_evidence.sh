#!/bin/bash
# One GPU call of round evidence: full parity suite (rtol log), smoke(), a bench line per BASELINE
# config (cfg3 default, cfg2, cfg5), the bias / dropout / non-causal legs of cfg3, a two-rank
# rehearsal of the multi-GPU launcher on this one GPU, then scripts/profile_round.sh (rocprofv3
# kernel stats + PMC passes), each step under its own limit.
# usage: bash scripts/gpu_evidence.sh TAG    then   python scripts/summarize_profiles.py TAG
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
timeout -k 10 300 python bench.py --bias --no-causal --no-cpu-baseline > $OUT/bench_cfg3_bias_noncausal.json 2> $OUT/bench_bias_nc.err || exit $?
for f in bias dropout noncausal bias_noncausal; do python -c "import json,sys; d=json.load(open('$OUT/bench_cfg3_$f.json')); print('$f', d['value'], d['fwd_tflops'], d['bwd_tflops'], d['kernels'])"; done
# two ranks on the one GPU of this box: the self-launching multi-GPU path end to end (gloo
# coordination, per-rank shards, max-over-ranks timing); the 8-GPU run is the driver's
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --no-cpu-baseline > $OUT/bench_cfg3_2ranks.json 2> $OUT/bench_2ranks.err || exit $?
cat $OUT/bench_cfg3_2ranks.json
bash scripts/profile_round.sh $TAG
