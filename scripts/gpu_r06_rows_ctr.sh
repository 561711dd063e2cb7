#!/bin/bash
# Round 6: (1) GBDT row-per-lane quantised histogram build (KDL_TUNE gbdt_hist_rows 0 = slot kernel / 4 / 8)
# tests + A/B interleaved x2 with a kernel trace of the default; (2) CTR forward GEMMs on igemm
# (scripts/gpu_r06_ctr_igemm.sh); (3) one driver-flag ResNet bench on this lease.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtr_tests.log 2>&1 || { tail -30 gpurun_out/r06/gbdtr_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtr_tests.log
for i in 1 2; do
  for ru in 0 4 8; do
    KDL_TUNE=gbdt_hist_rows=$ru timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtr_${ru}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtr_${ru}_$i.log') if l.startswith('{')][-1]);print('hist_rows=$ru', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/gbdtr_prof -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtr_prof.log 2>&1 || { tail -5 gpurun_out/r06/gbdtr_prof.log; exit 1; }
head -6 gpurun_out/r06/gbdtr_prof/run_kernel_stats.csv | cut -c1-200
bash scripts/gpu_r06_ctr_igemm.sh || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json 2> gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err || { tail -20 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err; exit 1; }
tail -1 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json | cut -c1-300
