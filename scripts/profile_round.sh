#!/bin/bash
# Profiles committed under profiles/: rocprofv3 kernel stats of the default bench command and
# PMC counters of the forward / backward launches at the bench workload (each pass its own
# run: FETCH_SIZE and WRITE_SIZE apart, SQ counters in two passes of <= 8, GRBM beside them).
# usage: bash scripts/profile_round.sh TAG   then   python scripts/summarize_profiles.py TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RK="python3 scripts/run_kernels.py --reps 3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_stdout.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_dropout -o run --output-format csv -- python3 bench.py --dropout 0.1 --no-cpu-baseline > $OUT/bench_dropout_stdout.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $RK > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $RK > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/sq1 -o run --output-format csv -- $RK > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC -d $OUT/sq2 -o run --output-format csv -- $RK > $OUT/sq2.log 2>&1 || echo "sq2 pass failed (optional counters)"
echo done
