#!/bin/bash
# GPU: forward variants against ab_libs/base.so -- variant check, then interleaved A/B timing
# (cfg3 causal / non-causal, S=8192 causal, cfg2).  usage: gpu_ab_fwd.sh TAG arm1 [arm2 ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for a in "$@"; do
  n=$(basename ${a%%:*} .so)
  timeout -k 10 240 python -u scripts/fwd_variant_check.py ab_libs/base.so $a > $OUT/check_$n.log 2>&1
  rc=$?; echo "$a: $(tail -1 $OUT/check_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
for cz in 1 0; do
  WHAT=fwd CAUSAL=$cz timeout -k 10 240 python scripts/ab.py ab_libs/base.so "$@" > $OUT/ab_c$cz.log 2>&1 || exit $?
  echo "causal=$cz"; grep -v amdgpu.ids $OUT/ab_c$cz.log
done
SHAPE=4,32,8192,128 WHAT=fwd CAUSAL=1 timeout -k 10 240 python scripts/ab.py ab_libs/base.so "$@" > $OUT/ab_s8k.log 2>&1 || exit $?
echo "S=8192 causal"; grep -v amdgpu.ids $OUT/ab_s8k.log
SHAPE=8,16,1024,64 WHAT=fwd CAUSAL=0 timeout -k 10 240 python scripts/ab.py ab_libs/base.so "$@" > $OUT/ab_cfg2.log 2>&1 || exit $?
echo "cfg2"; grep -v amdgpu.ids $OUT/ab_cfg2.log
