#!/bin/bash
# Round 6: CTR small-kernel occupancy: the optimizer's chunk size now adaptive (2048-element chunks for the 2.4M-parameter
# tower) and the head backward's rows per block (KDL_TUNE ctr_head_rpb 64 = before / 32 / 16), CTR tests, interleaved x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ctr.py tests/test_ops_gpu.py -m gpu > gpurun_out/r06/ctrs_tests.log 2>&1 || { tail -30 gpurun_out/r06/ctrs_tests.log; exit 1; }
tail -1 gpurun_out/r06/ctrs_tests.log
for i in 1 2; do
  for r in 64 32 16; do
    KDL_TUNE=ctr_head_rpb=$r timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 > gpurun_out/r06/ctrs_${r}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctrs_${r}_$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctrs_${r}_$i.log') if l.startswith('{')][-1]);print('head_rpb=$r run $i:', round(d['steps_per_sec'],1),'steps/s', round(d['samples_per_sec']/1e6,3),'M samples/s  host', d.get('host_issue_ms_per_step'),'ms/step  loss_last', d.get('loss_last'))"
  done
done
