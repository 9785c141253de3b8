#!/bin/bash
# GPU: interleaved A/B timing only (no tests).  usage: bash scripts/ab_time.sh TAG lib.so ...  (env WHAT)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
WHAT=${WHAT:-fwd} CAUSAL=1 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_causal.log 2>&1 || exit $?
cat $OUT/ab_causal.log
WHAT=${WHAT:-fwd} CAUSAL=0 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_noncausal.log 2>&1 || exit $?
cat $OUT/ab_noncausal.log
