#!/bin/bash
# Round 5: CTR re-measured after the dedup memset moved into the insert kernel:
# fixed-exchange world-1 rehearsal vs the sync-free path (interleaved) and a kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  for ex in fixed auto; do
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r05/ctr3_$ex$i.log 2>&1 || { tail -20 gpurun_out/r05/ctr3_$ex$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/ctr3_$ex$i.log') if l.startswith('{')][-1]);print('$ex', d.get('exchange'), round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,2),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'))"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/ctr3_fixed_prof -o run -- python3 -u -m kubedl_amd.workers.xdl_ctr --steps 60 --warmup 10 --exchange fixed > gpurun_out/r05/ctr3_fixed_prof.log 2>&1 || exit $?
# which HIP API calls issue the fill / copy kernels (runtime trace, no counters)
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d gpurun_out/r05/ctr3_fixed_api -o run -- python3 -u -m kubedl_amd.workers.xdl_ctr --steps 60 --warmup 10 --exchange fixed > gpurun_out/r05/ctr3_fixed_api.log 2>&1 || exit $?
