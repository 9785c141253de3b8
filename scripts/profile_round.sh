#!/bin/bash
# Profiles committed under profiles/: rocprofv3 kernel stats of the default bench command and
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the forward / backward launches.
# usage: bash scripts/profile_round.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_stdout.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 scripts/run_kernels.py --reps 3 > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 scripts/run_kernels.py --reps 3 > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 scripts/run_kernels.py --reps 3 > $OUT/sq.log 2>&1 || exit $?
echo done
