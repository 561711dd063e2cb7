#!/bin/bash
# Round 6: GBDT histogram unroll 16 (default) vs 32, and rows per chunk 2048 vs 4096 at unroll 16; x2 interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtu2_tests.log 2>&1 || { tail -20 gpurun_out/r06/gbdtu2_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtu2_tests.log
for i in 1 2; do
  for spec in "u16:gbdt_unroll=16" "u32:gbdt_unroll=32" "u16r4k:gbdt_unroll=16,gbdt_rpb=4096" "u16r1k:gbdt_unroll=16,gbdt_rpb=1024"; do
    name=${spec%%:*}; tune=${spec#*:}
    KDL_TUNE=$tune timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtu2_${name}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtu2_${name}_$i.log') if l.startswith('{')][-1]);print('$name', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
