#!/bin/bash
# Round 6: GBDT quantised histogram feature tile (KDL_TUNE gbdt_ftile 64 = default / 16 / 8), 2M x 28 depth 6,
# interleaved x2; then one driver-flag ResNet bench on this fresh lease (final-bench series).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtf_tests.log 2>&1 || { tail -20 gpurun_out/r06/gbdtf_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtf_tests.log
for i in 1 2; do
  for ft in 64 16 8; do
    KDL_TUNE=gbdt_ftile=$ft timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtf_${ft}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtf_${ft}_$i.log') if l.startswith('{')][-1]);print('ftile=$ft', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json 2> gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err || { tail -20 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err; exit 1; }
tail -1 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json | cut -c1-300
