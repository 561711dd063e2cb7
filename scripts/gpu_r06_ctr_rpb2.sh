#!/bin/bash
# Round 6: the CTR head backward's rows per block (KDL_TUNE ctr_head_rpb) re-swept after its batched row loads,
# interleaved x2, sync-free CTR step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
for i in 1 2; do
  for rpb in 64 32 128; do
    KDL_TUNE="ctr_head_rpb=$rpb" timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 > gpurun_out/r06/ctr_rpb2_${rpb}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctr_rpb2_${rpb}_$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctr_rpb2_${rpb}_$i.log') if l.startswith('{')][-1]);print('head_rpb=$rpb run $i:', round(d['steps_per_sec'],1), 'steps/s', round(d['samples_per_sec']/1e6,3),'M samples/s  host', d.get('host_issue_ms_per_step'), 'ms/step  loss_last', d['loss_last'])"
  done
done
