#!/bin/bash
# Round 4 iteration: new-kernel numerics tests, then the bench (job path x2),
# a kernel trace of the step, then (PMC=1) the whole-step PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests/test_head_gpu.py tests/test_stem_gpu.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T > gpurun_out/r04_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/r04_job_$r.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r04_job_$r.log') if l.startswith('{')][-1]); print('job', $r, {k: d.get(k) for k in ('value','ms_per_step','comm_init_s','time_to_first_step_s','first_pod_launch_delay_s','node_prefetch_s')})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof -o run -- python bench.py --direct --steps 8 --warmup 4 > gpurun_out/r04_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r04_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" --steps 6 > gpurun_out/r04_timeline.txt
python3 scripts/stray_kernels.py "$f" > gpurun_out/r04_stray.txt
python3 scripts/main_gaps.py "$f" 15 > gpurun_out/r04_main_gaps.txt
cat gpurun_out/r04_timeline.txt; tail -12 gpurun_out/r04_stray.txt; head -12 gpurun_out/r04_main_gaps.txt
timeout -k 10 300 rocprofv3 --hip-runtime-trace --output-format csv -d gpurun_out/r04_host -o run -- python bench.py --direct --steps 6 --warmup 4 > gpurun_out/r04_host.log 2>&1 || exit $?
h=$(find gpurun_out/r04_host -name "*hip_api_trace.csv" | head -1)
[ -n "$h" ] && python3 scripts/host_api_summary.py "$h" > gpurun_out/r04_host_summary.txt && head -40 gpurun_out/r04_host_summary.txt
if [ "${PMC:-0}" = "1" ]; then bash scripts/gpu_r04_pmc.sh || exit $?; fi
exit 0
