#!/bin/bash
# Round 6: the LDS-DMA GEMM main loop on v_mfma_f32_16x16x32_bf16 (_C_mf16.so, -DKDL_IGEMM_MF16=1)
# vs 32x32x16 (_C.so): numerics with every tile config forced, the 3x3 probe, the bench interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
M16=$PWD/kubedl_amd/_C_mf16.so
KDL_C_PATH=$M16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_igemm_gpu.py tests/test_dgrad_s2_gpu.py > gpurun_out/r06/mf16_tests.log 2>&1 || { tail -30 gpurun_out/r06/mf16_tests.log; exit 1; }
tail -1 gpurun_out/r06/mf16_tests.log
KDL_C_PATH=$M16 timeout -k 10 200 python -u scripts/igemm_cfg_probe.py 0,1,2,3 > gpurun_out/r06/mf16_probe.txt 2>&1 || { cat gpurun_out/r06/mf16_probe.txt; exit 1; }
timeout -k 10 200 python -u scripts/igemm_cfg_probe.py 0,1,2,3 > gpurun_out/r06/mf32_probe.txt 2>&1 || { cat gpurun_out/r06/mf32_probe.txt; exit 1; }
paste -d'\n' gpurun_out/r06/mf16_probe.txt gpurun_out/r06/mf32_probe.txt | grep -v amdgpu.ids
for i in 1 2; do
  KDL_C_PATH=$M16 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/mf16_bench_$i.json 2> gpurun_out/r06/mf16_bench_$i.err || { tail -20 gpurun_out/r06/mf16_bench_$i.err; exit 1; }
  echo "mf16: $(tail -1 gpurun_out/r06/mf16_bench_$i.json | cut -c1-200)"
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/mf32_bench_$i.json 2> gpurun_out/r06/mf32_bench_$i.err || { tail -20 gpurun_out/r06/mf32_bench_$i.err; exit 1; }
  echo "mf32: $(tail -1 gpurun_out/r06/mf32_bench_$i.json | cut -c1-200)"
done
