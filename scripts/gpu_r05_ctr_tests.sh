#!/bin/bash
# Round 5: CTR GPU tests only (after a binding change).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu > gpurun_out/r05/ctr_tests_final.log 2>&1 || { tail -30 gpurun_out/r05/ctr_tests_final.log; exit 1; }
tail -1 gpurun_out/r05/ctr_tests_final.log
