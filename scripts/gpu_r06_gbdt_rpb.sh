#!/bin/bash
# Round 6: GBDT rows per histogram chunk (KDL_TUNE gbdt_rpb; default by N = 1024 at 2M rows) with the row-per-lane
# build: the per-block fp32 flush is paid per chunk (profiles/r06_gbdt_hist_probe.txt).  Interleaved x2, 2M x 28, depth 6.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2; do
  for rpb in 0 2048 4096 8192; do
    KDL_TUNE=gbdt_rpb=$rpb timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtb_${rpb}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtb_${rpb}_$i.log') if l.startswith('{')][-1]);print('rpb=$rpb', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
