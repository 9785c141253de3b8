set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
OUT=gpurun_out/pmc_dbias; mkdir -p $OUT
RK="python3 bench.py --bias-grad --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/sq1 -o run --output-format csv -- $RK > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC -d $OUT/sq2 -o run --output-format csv -- $RK > $OUT/sq2.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $RK > $OUT/fetch.log 2>&1 || exit $?
# (optional) the address path and the LDS array: TA_BUSY (twice the fragment-load rate shows there,
# cdna_hip_programming.md), LDS cycles and stalls
timeout -s KILL 150 rocprofv3 --pmc TA_BUSY_avr SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE -d $OUT/ta -o run --output-format csv -- $RK > $OUT/ta.log 2>&1 || echo "ta pass failed (optional counters)"
python3 scripts/sum_pmc.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
