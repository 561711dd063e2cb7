#!/bin/bash
# rocprofv3 kernel trace of the bench step (single stream unless WS=1), summarised per kernel family.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export KDL_ENGINE=side=${WS:-0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --direct --steps ${STEPS:-8} --warmup 4 > gpurun_out/prof_bench.log 2>&1
rc=$?; tail -2 gpurun_out/prof_bench.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" $(( ${STEPS:-8} + 4 )) > gpurun_out/prof_summary.txt
head -45 gpurun_out/prof_summary.txt
