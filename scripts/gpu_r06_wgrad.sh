#!/bin/bash
# Round 6: interleaved-DMA weight-gradient main loop (csrc/wgrad_dma.hip) vs the round-5 build (_C_base.so):
# kernel tests, standalone probe on both, then the driver's bench interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_igemm_gpu.py tests/test_dgrad_s2_gpu.py tests/test_resnet_engine.py tests/test_wgrad_dma_gpu.py tests/test_gbdt.py -m gpu > gpurun_out/r06/wg_tests.log 2>&1 || { tail -30 gpurun_out/r06/wg_tests.log; exit 1; }
tail -2 gpurun_out/r06/wg_tests.log
timeout -k 10 200 python -u scripts/wgrad_probe.py > gpurun_out/r06/wg_probe_new.txt 2>&1 || { cat gpurun_out/r06/wg_probe_new.txt; exit 1; }
KDL_C_PATH=$PWD/kubedl_amd/_C_base.so timeout -k 10 200 python -u scripts/wgrad_probe.py > gpurun_out/r06/wg_probe_base.txt 2>&1 || { cat gpurun_out/r06/wg_probe_base.txt; exit 1; }
paste -d'\n' gpurun_out/r06/wg_probe_new.txt gpurun_out/r06/wg_probe_base.txt | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/wg_bench_new_$i.json 2> gpurun_out/r06/wg_bench_new_$i.err || { tail -20 gpurun_out/r06/wg_bench_new_$i.err; exit 1; }
  echo "new: $(tail -1 gpurun_out/r06/wg_bench_new_$i.json | cut -c1-200)"
  KDL_C_PATH=$PWD/kubedl_amd/_C_base.so timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/wg_bench_base_$i.json 2> gpurun_out/r06/wg_bench_base_$i.err || { tail -20 gpurun_out/r06/wg_bench_base_$i.err; exit 1; }
  echo "base: $(tail -1 gpurun_out/r06/wg_bench_base_$i.json | cut -c1-200)"
done
