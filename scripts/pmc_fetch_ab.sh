#!/bin/bash
# HBM read bytes (FETCH_SIZE) of the backward launches at the bench workload, per library build.
# usage: bash scripts/pmc_fetch_ab.sh TAG lib_a.so lib_b.so ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  FA2_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$n -o run --output-format csv -- python3 scripts/run_kernels.py --reps 3 --what bwd > $OUT/fetch_$n.log 2>&1 || exit $?
  echo "== $n"; python3 scripts/sum_pmc.py $OUT/fetch_$n
done
echo done
