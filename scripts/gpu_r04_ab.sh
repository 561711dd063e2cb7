#!/bin/bash
# Round 4 A/B pricing runs (bench --direct, interleaved): default vs the slab
# reduce skipped (timing only) vs the world-1 DDP rehearsal with a bucket-sized
# RCCL op per bucket on the process group's stream; then a kernel trace of the
# rehearsal (which stream the RCCL copies run on, what overlaps them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for spec in ${AB:-"base:X=1" "noreduce:KDL_TUNE=price_wgrad_reduce=0" "ddpcopy:KDL_TUNE=ddp_world1=copy"}; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/ab4_${name}_r$r.log 2>&1 || exit $?
    echo "$name r$r $(grep -o '"value": [0-9.]*' gpurun_out/ab4_${name}_r$r.log) $(grep -o '"exposed_ms_per_step": [0-9.a-z]*' gpurun_out/ab4_${name}_r$r.log)"
  done
done
KDL_TUNE=ddp_world1=copy timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r04_prof_ddpcopy -o run -- python bench.py --direct --steps 8 --warmup 4 > gpurun_out/r04_prof_ddpcopy.log 2>&1 || exit $?
f=$(find gpurun_out/r04_prof_ddpcopy -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --steps 6 > gpurun_out/r04_ddpcopy_timeline.txt
cat gpurun_out/r04_ddpcopy_timeline.txt
