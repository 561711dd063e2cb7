#!/bin/bash
# quick GPU loop: engine+conv1x1 numerics, GEMM microbench, fused-engine bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_engine.py tests/test_conv1x1_gpu.py tests/test_ops_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_quick.log 2>&1 || { tail -30 gpurun_out/t_quick.log; exit 1; }
tail -1 gpurun_out/t_quick.log
if [ -n "$MICRO" ]; then timeout -k 10 300 python -u scripts/bench_conv1x1.py > gpurun_out/gemm_micro.log 2>&1 || exit $?; tail -1 gpurun_out/gemm_micro.log; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_quick.log 2>&1 || exit $?
tail -1 gpurun_out/bench_quick.log
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_quick -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_quick.log 2>&1 || exit $?
  echo prof-done
fi
