#!/bin/bash
# Round 6: interleaved-DMA LDS-DMA GEMM main loop (csrc/igemm.hip) vs the round-5 loop (_C_base.so):
# numerics, the stage 2-4 3x3 probe on both, then the driver's bench interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_igemm_gpu.py tests/test_dgrad_s2_gpu.py > gpurun_out/r06/ilv_tests.log 2>&1 || { tail -30 gpurun_out/r06/ilv_tests.log; exit 1; }
tail -2 gpurun_out/r06/ilv_tests.log
timeout -k 10 200 python -u scripts/igemm_cfg_probe.py 0,1,2,3 > gpurun_out/r06/ilv_probe_new.txt 2>&1 || { cat gpurun_out/r06/ilv_probe_new.txt; exit 1; }
KDL_C_PATH=$PWD/kubedl_amd/_C_base.so timeout -k 10 200 python -u scripts/igemm_cfg_probe.py 0,1,2,3 > gpurun_out/r06/ilv_probe_base.txt 2>&1 || { cat gpurun_out/r06/ilv_probe_base.txt; exit 1; }
paste -d'\n' gpurun_out/r06/ilv_probe_new.txt gpurun_out/r06/ilv_probe_base.txt | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/ilv_bench_new_$i.json 2> gpurun_out/r06/ilv_bench_new_$i.err || { tail -20 gpurun_out/r06/ilv_bench_new_$i.err; exit 1; }
  echo "new: $(tail -1 gpurun_out/r06/ilv_bench_new_$i.json)"
  KDL_C_PATH=$PWD/kubedl_amd/_C_base.so timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/ilv_bench_base_$i.json 2> gpurun_out/r06/ilv_bench_base_$i.err || { tail -20 gpurun_out/r06/ilv_bench_base_$i.err; exit 1; }
  echo "base: $(tail -1 gpurun_out/r06/ilv_bench_base_$i.json)"
done
