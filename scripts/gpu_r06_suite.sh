#!/bin/bash
# Round 6: the full GPU test suite (one process), smoke(), then one driver-flag bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r06/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || { tail -20 gpurun_out/r06/smoke.log; exit 1; }
tail -1 gpurun_out/r06/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final_bench_${FINAL_TAG:-d}.json 2> gpurun_out/r06/final_bench_${FINAL_TAG:-d}.err || { tail -20 gpurun_out/r06/final_bench_${FINAL_TAG:-d}.err; exit 1; }
tail -1 gpurun_out/r06/final_bench_${FINAL_TAG:-d}.json | cut -c1-300
