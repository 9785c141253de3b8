#!/bin/bash
# round-2 check: GPU suite + bench, then the context comparison (SDPA, Flex) and the MQA split A/B
set -o pipefail
bash scripts/gpu_tests.sh r02b || exit $?
OUT=gpurun_out/r02b
timeout -k 10 240 env FA2_DKV_SPLIT=0 python scripts/compare_sdpa.py --no-flex --only mqa-b1 > $OUT/mqa_nosplit.jsonl 2> $OUT/mqa_nosplit.err || exit $?
timeout -k 10 900 python -u scripts/compare_sdpa.py > $OUT/compare.jsonl 2> $OUT/compare.err || exit $?
cat $OUT/mqa_nosplit.jsonl $OUT/compare.jsonl
