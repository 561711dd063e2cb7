#!/bin/bash
# Round 6: CTR forward GEMMs on the LDS-DMA igemm loop (BIAS / BIAS_RELU epilogues): numerics tests, the
# per-shape probe, then the sync-free and fixed CTR step with KDL_TUNE ctr_igemm=0 / 1 interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu -k "gemm or igemm" > gpurun_out/r06/ctri_tests.log 2>&1 || { tail -30 gpurun_out/r06/ctri_tests.log; exit 1; }
tail -1 gpurun_out/r06/ctri_tests.log
timeout -k 10 200 python -u scripts/ctr_igemm_probe.py 300 > gpurun_out/r06/ctri_probe.log 2>&1 || { tail -20 gpurun_out/r06/ctri_probe.log; exit 1; }
cat gpurun_out/r06/ctri_probe.log
for i in 1 2; do
  for ig in 0 1; do
    for ex in auto fixed; do
      KDL_TUNE=ctr_igemm=$ig timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r06/ctri_${ex}_${ig}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctri_${ex}_${ig}_$i.log; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctri_${ex}_${ig}_$i.log') if l.startswith('{')][-1]);print('ctr_igemm=$ig', '$ex', round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,3),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'), 'loss_last', d.get('loss_last'))"
    done
  done
done
