#!/bin/bash
# Halo 3x3 kernel: numerics first (own timeout, stop at the first failure), then the existing
# conv suites, then timings of the 3x3 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_halo3x3_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/halo_tests.log 2>&1
rc=$?; tail -15 gpurun_out/halo_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_igemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/time_igemm.py 3x3 > gpurun_out/time_halo.jsonl 2> gpurun_out/time_halo.err
exit $?
