#!/bin/bash
# GPU: parity (reference grids at stride STRIDE, default 9, plus everything else) of each candidate
# library, then interleaved A/B timing of all of them, causal and not, at cfg3 and at SHAPE2.
# usage: bash scripts/gpu_ab3.sh TAG WHAT cand1.so [cand2.so ...] -- base.so [...]
set -o pipefail
TAG=$1; WHAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CANDS=(); while [ "$1" != "--" ]; do CANDS+=("$1"); shift; done; shift
for c in "${CANDS[@]}"; do
  n=$(basename $c .so)
  FA2_AMD_LIB=$c FA2_GRID_STRIDE=${STRIDE:-9} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_$n.log 2>&1
  rc=$?; echo "$n: $(tail -1 $OUT/tests_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
for cz in 1 0; do
  WHAT=$WHAT CAUSAL=$cz timeout -k 10 300 python scripts/ab.py "${CANDS[@]}" "$@" > $OUT/ab_c$cz.log 2>&1 || exit $?
  echo "causal=$cz"; cat $OUT/ab_c$cz.log
done
if [ -n "$SHAPE2" ]; then
  SHAPE=$SHAPE2 WHAT=fwd CAUSAL=${CAUSAL2:-0} timeout -k 10 300 python scripts/ab.py "${CANDS[@]}" "$@" > $OUT/ab_shape2.log 2>&1 || exit $?
  echo "shape2=$SHAPE2"; cat $OUT/ab_shape2.log
fi
