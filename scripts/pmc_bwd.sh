#!/bin/bash
# PMC counters of the backward launches at the bench workload (one rocprofv3 pass per group).
# usage: bash scripts/pmc_bwd.sh TAG [WHAT]
set -o pipefail
TAG=${1:-pmc}
WHAT=${2:-bwd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RK="python3 scripts/run_kernels.py --reps 3 --what $WHAT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $RK > $OUT/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/sq1 -o run --output-format csv -- $RK > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC -d $OUT/sq2 -o run --output-format csv -- $RK > $OUT/sq2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_IFETCH SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_SMEM -d $OUT/sq3 -o run --output-format csv -- $RK > $OUT/sq3.log 2>&1 || echo "sq3 optional pass failed"
echo done
