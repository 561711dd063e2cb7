# A/B of the engine's side stream (KDL_ENGINE=side=0|1) + its GPU tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_resnet_engine.py tests/test_p2p.py > gpurun_out/ws_tests.log 2>&1 || { tail -30 gpurun_out/ws_tests.log; exit 1; }
tail -3 gpurun_out/ws_tests.log
for f in 1 1 1; do
  KDL_ENGINE=side=$f timeout -k 10 200 python -u bench.py > gpurun_out/ws_bench_$f.log 2>&1 || exit 1
  echo "ws=$f $(tail -1 gpurun_out/ws_bench_$f.log | cut -c1-200)"
done
