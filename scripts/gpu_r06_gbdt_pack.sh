#!/bin/bash
# Round 6: GBDT row-per-lane build with g and h in one 64-bit LDS add (KDL_TUNE gbdt_pack64=1) vs two 32-bit adds:
# the quantised-histogram tests under it, then interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
KDL_TUNE=gbdt_pack64=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtk_tests.log 2>&1 || { tail -30 gpurun_out/r06/gbdtk_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtk_tests.log
for i in 1 2 3; do
  for pk in 0 1; do
    KDL_TUNE=gbdt_pack64=$pk timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtk_${pk}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtk_${pk}_$i.log') if l.startswith('{')][-1]);print('pack64=$pk', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
