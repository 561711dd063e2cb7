#!/bin/bash
# Round 6: GBDT integer histograms with one 64-bit LDS add per (row, feature) vs two 32-bit adds
# (KDL_TUNE gbdt_pack64=0), interleaved: tests, then the 2M x 28 depth-6 fit three times each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdt_tests.log 2>&1 || { tail -20 gpurun_out/r06/gbdt_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdt_tests.log
for i in 1 2 3; do
  for pk in 1 0; do
    KDL_TUNE=gbdt_pack64=$pk timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdt_p${pk}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdt_p${pk}_$i.log') if l.startswith('{')][-1]);print('pack64=$pk', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','setup_s','logloss','accuracy')})"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/gbdt_prof -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdt_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r06/gbdt_prof -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -c1-200
