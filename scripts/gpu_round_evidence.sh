#!/bin/bash
# GPU: the round's committed evidence -- rocprofv3 stats + PMC of the default bench (profile_round.sh),
# the HBM copy and MFMA microbenchmarks, and the bench lines of the other configurations.
# usage: bash scripts/gpu_round_evidence.sh TAG   (then python scripts/summarize_profiles.py TAG here)
set -o pipefail
TAG=${1:-r04f}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/profile_round.sh $TAG || exit $?
timeout -k 10 120 ./bench_micro/hbm_copy > $OUT/hbm_copy.txt 2>&1 || exit $?
timeout -k 10 120 ./bench_micro/mfma_peak > $OUT/mfma_peak.txt 2>&1 || exit $?
for leg in "--config refbench" "--config cfg2" "--dropout 0.1" "--bias" "--no-causal"; do
  f=$OUT/bench_$(echo $leg | tr -d ' -' ).json
  timeout -k 10 300 python bench.py --no-cpu-baseline $leg > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$leg', d['value'], d.get('fwd_tflops'), d.get('bwd_tflops'), {k: v['ms'] for k, v in d.get('kernels', {}).items()})"
done
cat $OUT/hbm_copy.txt $OUT/mfma_peak.txt
