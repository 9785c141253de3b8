#!/bin/bash
# GPU: full parity suite, then SQ/GRBM counters of the forward at cfg3 (causal, non-causal).
# usage: bash scripts/gpu_hp_pmc.sh TAG [nosuite]
set -o pipefail
TAG=${1:-hpp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "nosuite" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
WHAT=fwd bash scripts/pmc_fwd.sh $TAG/pmc > $OUT/pmc.txt 2>&1 || { cat $OUT/pmc.txt; exit 1; }
cat $OUT/pmc.txt
