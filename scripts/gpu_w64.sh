#!/bin/bash
# GPU: forward-variant check, then interleaved A/B timing (cfg3 causal / non-causal, S=8192).
set -o pipefail
TAG=${1:-w64a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/fwd_variant_check.py ab_libs/base.so ab_libs/w64.so:FA2_FWD_W64=1 > $OUT/check.log 2>&1
rc=$?; tail -4 $OUT/check.log; [ $rc -ne 0 ] && exit $rc
for cz in 1 0; do
  WHAT=fwd CAUSAL=$cz timeout -k 10 240 python scripts/ab.py ab_libs/base.so ab_libs/w64.so:FA2_FWD_W64=1 > $OUT/ab_c$cz.log 2>&1 || exit $?
  echo "causal=$cz"; cat $OUT/ab_c$cz.log
done
SHAPE=4,32,8192,128 WHAT=fwd CAUSAL=1 timeout -k 10 240 python scripts/ab.py ab_libs/base.so ab_libs/w64.so:FA2_FWD_W64=1 > $OUT/ab_s8k.log 2>&1 || exit $?
echo "S=8192 causal"; cat $OUT/ab_s8k.log
