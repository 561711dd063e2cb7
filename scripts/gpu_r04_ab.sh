#!/bin/bash
# Round 4 A/B pricing runs (bench --direct, interleaved): default vs the
# slab reduce skipped (timing only) vs fewer weight-gradient blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for spec in "base:X=1" "noreduce:KDL_PRICE_WGRAD_REDUCE=0" "wg256:KDL_WGRAD_BLOCKS=256" "wg384:KDL_WGRAD_BLOCKS=384"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/ab4_${name}_r$r.log 2>&1 || exit $?
    echo "$name r$r $(grep -o '"value": [0-9.]*' gpurun_out/ab4_${name}_r$r.log)"
  done
done
