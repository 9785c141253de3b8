#!/bin/bash
# GPU: full parity suite + smoke, then forward scaling sweeps (per-item vs per-tile cost).
# usage: bash scripts/gpu_suite.sh TAG
set -o pipefail
TAG=${1:-suite}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python scripts/fwd_scaling.py --d 64 --heads 16 --tokens 8192 --seqlens 256,512,1024,2048,4096 --causal 0 > $OUT/scaling_d64.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/fwd_scaling.py --d 128 --heads 32 --tokens 32768 --seqlens 1024,2048,4096,8192 > $OUT/scaling_d128.txt 2>&1 || exit $?
cat $OUT/scaling_d64.txt $OUT/scaling_d128.txt
