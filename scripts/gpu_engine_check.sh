mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resnet_engine.py tests/test_conv1x1_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_engine.log 2>&1
rc=$?; tail -30 gpurun_out/t_engine.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 --engine fused > gpurun_out/bench_fused.log 2>&1 || exit $?
tail -1 gpurun_out/bench_fused.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 --engine autograd > gpurun_out/bench_autograd.log 2>&1 || exit $?
tail -1 gpurun_out/bench_autograd.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --engine fused > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.log 2>&1 || exit $?
echo prof-done
