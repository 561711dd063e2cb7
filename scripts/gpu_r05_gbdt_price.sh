#!/bin/bash
# Round 5: what bounds the GBDT histogram build -- the same fit with both LDS
# atomics (0), the g atomic only (1, timing only) and none (2, loads only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  for pr in 0 1 2 3 4; do
    KDL_TUNE=gbdt_price=$pr timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r05/gbdt_price${pr}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/gbdt_price${pr}_$i.log') if l.startswith('{')][-1]);print('price=$pr', round(d['rounds_per_sec'],1), round(d['fit_rounds_per_sec'],1), round(d['setup_s'],3), round(d.get('setup_cuts_s',0),3))"
  done
done
