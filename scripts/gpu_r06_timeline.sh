#!/bin/bash
# Round 6: kernel trace of the ResNet-50 two-stream step (bench.py --direct, 10 steps after 4) -> the critical-path
# timeline (scripts/timeline.py) and the per-kernel stats of the step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/tl_prof -o run -- python3 bench.py --direct --steps 10 --warmup 4 > gpurun_out/r06/tl_prof.log 2>&1 || { tail -5 gpurun_out/r06/tl_prof.log; exit 1; }
f=$(find gpurun_out/r06/tl_prof -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline.py "$f" --steps 4 > gpurun_out/r06/timeline.txt 2>&1 || { tail -5 gpurun_out/r06/timeline.txt; exit 1; }
cat gpurun_out/r06/timeline.txt | head -80
