#!/bin/bash
# GPU: end-of-round evidence in one call -- the GPU suite (with the tolerance-escape count), smoke,
# rocprofv3 stats + PMC of the default bench (profile_round.sh), and the bench lines of every
# configuration.  usage: bash scripts/gpu_final.sh TAG   (then python scripts/summarize_profiles.py TAG)
set -o pipefail
TAG=${1:-r04h}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# PART=tests | bench (default both: one call may not hold both within gpurun's limit)
PART=${PART:-all}
if [ "$PART" != bench ]; then
FA2_TOL_REPORT=$OUT/tolerance_escapes.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
[ "$PART" = tests ] && exit 0
fi
bash scripts/profile_round.sh $TAG || exit $?
for leg in "" "--no-causal" "--dropout 0.1" "--bias" "--config cfg2" "--config refbench" "--config cfg5" "--bias-grad --steps 3 --warmup 1"; do
  f=$OUT/bench_$(echo "x$leg" | tr -d ' -.').json
  timeout -k 10 400 python bench.py $leg > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$leg', d['value'], d.get('fwd_tflops'), d.get('bwd_tflops'), {k: v['ms'] for k, v in d.get('kernels', {}).items()}, d.get('roofline_valu', {}).get('frac'))"
done
