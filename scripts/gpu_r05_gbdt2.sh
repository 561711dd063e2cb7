#!/bin/bash
# Round 5: GBDT with quantised integer LDS histograms -- GPU tests, fit x2, kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py tests/test_gpu_jobs.py -m gpu -k "gbdt or xgb or XGB" > gpurun_out/r05/gbdt_tests3.log 2>&1 || { tail -30 gpurun_out/r05/gbdt_tests3.log; exit 1; }
tail -1 gpurun_out/r05/gbdt_tests3.log
for i in 1 2 3; do
  timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r05/gbdt_q$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/gbdt_q$i.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/gbdt_q_prof -o run -- python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 30 > gpurun_out/r05/gbdt_q_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r05/gbdt_q_prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r05/gbdt_q_summary.txt; head -24 gpurun_out/r05/gbdt_q_summary.txt
