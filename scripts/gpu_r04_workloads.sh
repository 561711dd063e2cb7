#!/bin/bash
# Round 4: XDL CTR and XGBoost GBDT on the GPU -- steps/s, rounds/s and their
# kernel summaries (world 1: the sync-free CTR path, the device-resident grower).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m kubedl_amd.workers.xdl_ctr --steps 200 --warmup 10 > gpurun_out/r04_ctr.log 2>&1 || exit $?
tail -1 gpurun_out/r04_ctr.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_ctr_prof -o run -- python -u -m kubedl_amd.workers.xdl_ctr --steps 20 --warmup 5 > gpurun_out/r04_ctr_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r04_ctr_prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 25 > gpurun_out/r04_ctr_summary.txt; head -25 gpurun_out/r04_ctr_summary.txt
timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r04_gbdt.log 2>&1 || exit $?
tail -1 gpurun_out/r04_gbdt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_gbdt_prof -o run -- python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 30 > gpurun_out/r04_gbdt_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r04_gbdt_prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r04_gbdt_summary.txt; head -25 gpurun_out/r04_gbdt_summary.txt
