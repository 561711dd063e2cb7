#!/bin/bash
# Round 4: world-1 DDP rehearsal.  Job-path bench (default), then direct A/B of
# KDL_TUNE ddp_world1=0/1 (two interleaved rounds), then a kernel trace of the
# two-stream step with the bucketed RCCL all-reduces on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/r04_job.log 2>&1 || exit $?
tail -1 gpurun_out/r04_job.log
for r in 1 2; do
  for w in 0 1; do
    KDL_TUNE=ddp_world1=$w timeout -k 10 180 python bench.py --direct --steps 20 --warmup 8 > gpurun_out/r04_ddp${w}_r$r.log 2>&1 || exit $?
    echo "ddp_world1=$w r$r $(grep -o '"value": [0-9.]*' gpurun_out/r04_ddp${w}_r$r.log)"
  done
done
KDL_TUNE=ddp_world1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof_ddp -o run -- python bench.py --direct --steps 8 --warmup 4 > gpurun_out/r04_prof_ddp.log 2>&1 || exit $?
f=$(find gpurun_out/r04_prof_ddp -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --steps 6 > gpurun_out/r04_ddp_timeline.txt
cat gpurun_out/r04_ddp_timeline.txt
s=$(find gpurun_out/r04_prof_ddp -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$s" 12 > gpurun_out/r04_ddp_summary.txt
head -60 gpurun_out/r04_ddp_summary.txt
python3 scripts/stray_kernels.py "$f" > gpurun_out/r04_stray.txt
tail -30 gpurun_out/r04_stray.txt
