#!/bin/bash
# Round 6: GBDT histogram row slots in flight per thread (KDL_TUNE gbdt_unroll 4 / 8 / 16), 2M x 28 depth 6,
# 100 rounds, interleaved x3; then the kernel summary of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtu_tests.log 2>&1 || { tail -20 gpurun_out/r06/gbdtu_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtu_tests.log
for i in 1 2 3; do
  for u in 4 8 16; do
    KDL_TUNE=gbdt_unroll=$u timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtu_${u}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtu_${u}_$i.log') if l.startswith('{')][-1]);print('unroll=$u', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/gbdtu_prof -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtu_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r06/gbdtu_prof -name '*kernel_stats.csv' | head -1); head -6 "$f" | cut -c1-160
