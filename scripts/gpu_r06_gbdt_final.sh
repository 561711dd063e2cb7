#!/bin/bash
# Round 6: GBDT with the row-per-lane build and 4096 rows per chunk (new defaults): GPU tests, 3 timed fits, the
# rows-in-flight A/B (KDL_TUNE gbdt_hist_rows 4 / 8), and a kernel trace of one fit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtf_tests.log 2>&1 || { tail -30 gpurun_out/r06/gbdtf_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtf_tests.log
for i in 1 2 3; do
  for ru in 4; do
    KDL_TUNE=gbdt_hist_rows=$ru timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtf_${ru}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtf_${ru}_$i.log') if l.startswith('{')][-1]);print('hist_rows=$ru', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/gbdtf_prof -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtf_prof.log 2>&1 || { tail -5 gpurun_out/r06/gbdtf_prof.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r06/gbdtf_prof/run_kernel_stats.csv')))
for r in rows[:16]:
    print('%-70s %5s calls %8.2f ms %8.2f us/call %6s %%' % (r['Name'][:70], r['Calls'], int(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3, r['Percentage'][:5]))
PY
