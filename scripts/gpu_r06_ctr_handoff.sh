#!/bin/bash
# Round 6: the CTR split reductions' hand-off without fences (KDL_TUNE ctr_handoff=1: sc1 partials) -- CTR GPU tests
# under it, then the sync-free step over ctr_handoff 0/1 x ctr_fused_relu_bwd 0/1, interleaved x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
KDL_TUNE=ctr_handoff=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ctr.py -m gpu > gpurun_out/r06/ctrh_tests.log 2>&1 || { tail -30 gpurun_out/r06/ctrh_tests.log; exit 1; }
tail -1 gpurun_out/r06/ctrh_tests.log
for i in 1 2; do
  for h in 0 1; do
    for fz in 0 1; do
      KDL_TUNE=ctr_handoff=$h,ctr_fused_relu_bwd=$fz timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 > gpurun_out/r06/ctrh_${h}_${fz}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctrh_${h}_${fz}_$i.log; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctrh_${h}_${fz}_$i.log') if l.startswith('{')][-1]);print('handoff=$h fused=$fz run $i:', round(d['steps_per_sec'],1),'steps/s', round(d['samples_per_sec']/1e6,3),'M samples/s  host', d.get('host_issue_ms_per_step'),'ms/step  loss_last', d.get('loss_last'))"
    done
  done
done
