#!/bin/bash
# GPU A/B of library builds: quick parity of the candidate (first lib) then interleaved timing.
# usage: bash scripts/ab_run.sh TAG cand.so [other.so ...]   (env WHAT, STRIDE)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FA2_AMD_LIB=$1 FA2_GRID_STRIDE=${STRIDE:-9} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
WHAT=${WHAT:-fwd} CAUSAL=1 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_causal.log 2>&1 || exit $?
cat $OUT/ab_causal.log
WHAT=${WHAT:-fwd} CAUSAL=0 timeout -k 10 300 python scripts/ab.py "$@" > $OUT/ab_noncausal.log 2>&1 || exit $?
cat $OUT/ab_noncausal.log
