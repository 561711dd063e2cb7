#!/bin/bash
# Round 5: per-kernel stats, bn_bwd_fuse=3 vs 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for m in 3 1; do
  KDL_ENGINE=bn_bwd_fuse=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/prof_gram$m -o run -- python3 bench.py --direct --steps 10 --warmup 4 > gpurun_out/r05/prof_gram$m.log 2>&1 || exit $?
done
find gpurun_out/r05 -name '*kernel_stats.csv' | head -5
