#!/bin/bash
# Round 5: owner update without de-duplication (a2a_owner_update) -- CTR GPU tests, then the
# fixed-exchange world-1 rehearsal vs the sync-free path (interleaved) and a kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_ctr.py -m gpu > gpurun_out/r05/ctr2_tests.log 2>&1 || { tail -30 gpurun_out/r05/ctr2_tests.log; exit 1; }
tail -2 gpurun_out/r05/ctr2_tests.log
for i in 1 2; do
  for ex in fixed auto; do
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r05/ctr2_$ex$i.log 2>&1 || { tail -20 gpurun_out/r05/ctr2_$ex$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/ctr2_$ex$i.log') if l.startswith('{')][-1]);print('$ex', d.get('exchange'), round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,2),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'))"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/ctr2_fixed_prof -o run -- python3 -u -m kubedl_amd.workers.xdl_ctr --steps 60 --warmup 10 --exchange fixed > gpurun_out/r05/ctr2_fixed_prof.log 2>&1 || exit $?
