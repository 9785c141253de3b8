#!/bin/bash
# GPU: full parity suite on the in-tree library, then interleaved A/B timing of library builds.
# usage: bash scripts/gpu_ab.sh TAG WHAT lib_a.so lib_b.so ...
set -o pipefail
TAG=$1; WHAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -15 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
WHAT=$WHAT CAUSAL=1 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_causal.log 2>&1 || exit $?
cat $OUT/ab_causal.log
WHAT=$WHAT CAUSAL=0 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_noncausal.log 2>&1 || exit $?
cat $OUT/ab_noncausal.log
