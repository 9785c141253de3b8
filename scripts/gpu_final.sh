#!/bin/bash
# Round-end evidence in one GPU call: full parity suite (rtol log), smoke(), the default bench
# line (with cpu_baseline), then scripts/profile_round.sh (rocprofv3 kernel stats + PMC passes).
# usage: bash scripts/gpu_final.sh TAG     then   python scripts/summarize_profiles.py TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export FA2_RTOL_LOG=$OUT/rtol.jsonl
rm -f $FA2_RTOL_LOG
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_line.json 2> $OUT/bench.err || exit $?
cat $OUT/bench_line.json
bash scripts/profile_round.sh $TAG
