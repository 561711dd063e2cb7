#!/bin/bash
# Round 6: CTR tower with the ReLU backward + bias gradients fused into the producing launches
# (head_bce_bwd relu_x, gemm_dgrad_relu) and the 1024/512-wide forward layers on igemm: GPU tests,
# then sync-free / fixed CTR A/B (KDL_TUNE ctr_fused_relu_bwd 0 / 1) interleaved x2; then the
# standalone GBDT histogram probe with and without the flush (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ctr.py tests/test_gbdt.py -m gpu > gpurun_out/r06/ctrf_tests.log 2>&1 || { tail -30 gpurun_out/r06/ctrf_tests.log; exit 1; }
tail -1 gpurun_out/r06/ctrf_tests.log
for i in 1 2; do
  for fz in 0 1; do
    for ex in auto fixed; do
      KDL_TUNE=ctr_fused_relu_bwd=$fz timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r06/ctrf_${ex}_${fz}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctrf_${ex}_${fz}_$i.log; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctrf_${ex}_${fz}_$i.log') if l.startswith('{')][-1]);print('fused_relu_bwd=$fz', '$ex', round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,3),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'), 'loss_last', d.get('loss_last'))"
    done
  done
done
timeout -k 10 200 python -u scripts/gbdt_hist_probe.py > gpurun_out/r06/gbdt_probe.log 2>&1 || { tail -20 gpurun_out/r06/gbdt_probe.log; exit 1; }
cat gpurun_out/r06/gbdt_probe.log
KDL_TUNE=gbdt_price_noflush=1 timeout -k 10 200 python -u scripts/gbdt_hist_probe.py > gpurun_out/r06/gbdt_probe_noflush.log 2>&1 || { tail -20 gpurun_out/r06/gbdt_probe_noflush.log; exit 1; }
echo "no flush (timing only):"; cat gpurun_out/r06/gbdt_probe_noflush.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/ctrf_prof -o run -- python3 -m kubedl_amd.workers.xdl_ctr --steps 200 --warmup 20 > gpurun_out/r06/ctrf_prof.log 2>&1 || { tail -5 gpurun_out/r06/ctrf_prof.log; exit 1; }
head -14 gpurun_out/r06/ctrf_prof/run_kernel_stats.csv | cut -c1-160
