#!/bin/bash
# Round 5 baseline: job-path bench twice, then a two-stream kernel trace of the direct step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/base_bench$i.json 2> gpurun_out/r05/base_bench$i.err || exit $?
  tail -1 gpurun_out/r05/base_bench$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/prof -o run -- python bench.py --direct --steps 8 --warmup 4 > gpurun_out/r05/prof_bench.log 2>&1 || exit $?
f=$(find gpurun_out/r05/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 12 > gpurun_out/r05/prof_summary.txt
head -60 gpurun_out/r05/prof_summary.txt
