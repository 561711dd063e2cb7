#!/bin/bash
# Round 5: GBDT fit with the sort-based cuts and the staged host copy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r05/gbdt_tests4.log 2>&1 || { tail -30 gpurun_out/r05/gbdt_tests4.log; exit 1; }
tail -1 gpurun_out/r05/gbdt_tests4.log
for i in 1 2 3; do
  timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r05/gbdt_f$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/gbdt_f$i.log
done
