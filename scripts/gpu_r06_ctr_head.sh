#!/bin/bash
# Round 6: head backward with every row's loads in flight per batch (csrc/ctr.hip head_bce_bwd_kernel) --
# the CTR GPU tests, the kernel's time in a kernel trace, then the CTR step (sync-free x2, fixed x1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu -p no:cacheprovider > gpurun_out/r06/ctr_head_tests.log 2>&1 || { tail -30 gpurun_out/r06/ctr_head_tests.log; exit 1; }
tail -1 gpurun_out/r06/ctr_head_tests.log
rm -rf gpurun_out/r06/ctr_head_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/ctr_head_prof -o run -- python3 -m kubedl_amd.workers.xdl_ctr --steps 200 --warmup 20 > gpurun_out/r06/ctr_head_prof.log 2>&1 || { tail -5 gpurun_out/r06/ctr_head_prof.log; exit 1; }
f=$(find gpurun_out/r06/ctr_head_prof -name '*kernel_stats.csv' | head -1)
grep -i -E "head_bce|segment_reduce" "$f" | cut -c1-200
for i in 1 2; do
  for ex in auto fixed; do
    [ $ex = fixed ] && [ $i = 2 ] && continue
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r06/ctr_head_$ex$i.log 2>&1 || { tail -20 gpurun_out/r06/ctr_head_$ex$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctr_head_$ex$i.log') if l.startswith('{')][-1]);print('$ex run $i:', round(d['steps_per_sec'],1), 'steps/s', round(d['samples_per_sec']/1e6,3),'M samples/s  host', d.get('host_issue_ms_per_step'), 'ms/step  loss_last', d['loss_last'])"
  done
done
