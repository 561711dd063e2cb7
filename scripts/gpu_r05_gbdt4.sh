#!/bin/bash
# Round 5: GBDT fit with the cuts computed from the host copy beside the H2D copy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r05/gbdt4_tests.log 2>&1 || { tail -20 gpurun_out/r05/gbdt4_tests.log; exit 1; }
tail -1 gpurun_out/r05/gbdt4_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r05/gbdt4_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/gbdt4_$i.log') if l.startswith('{')][-1]);print({k:round(d[k],4) for k in ('rounds_per_sec','fit_rounds_per_sec','setup_s','setup_h2d_s','setup_cuts_s','logloss')})"
done
