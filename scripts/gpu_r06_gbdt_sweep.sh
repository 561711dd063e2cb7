#!/bin/bash
# Round 6: GBDT rows per chunk x rows in flight on the packed 64-bit build (KDL_TUNE gbdt_rpb / gbdt_hist_rows), x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2; do
  for arm in "gbdt_rpb=4096,gbdt_hist_rows=4" "gbdt_rpb=4096,gbdt_hist_rows=8" "gbdt_rpb=8192,gbdt_hist_rows=4" "gbdt_rpb=2048,gbdt_hist_rows=4"; do
    tag=$(echo "$arm" | tr '=,' '__')
    KDL_TUNE=$arm timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdts_${tag}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdts_${tag}_$i.log') if l.startswith('{')][-1]);print('$arm', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
