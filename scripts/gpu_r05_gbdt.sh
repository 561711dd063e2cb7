#!/bin/bash
# Round 5: GBDT rounds/s with the fused grad/hess kernel, setup phases, and PMC
# passes over the histogram build (LDS atomics / conflicts / occupancy / bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/gbdt_pmc
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r05/gbdt_tests.log 2>&1 || { tail -20 gpurun_out/r05/gbdt_tests.log; exit 1; }
tail -1 gpurun_out/r05/gbdt_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r05/gbdt_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/gbdt_$i.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/gbdt_prof -o run -- python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 30 > gpurun_out/r05/gbdt_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r05/gbdt_prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r05/gbdt_summary.txt; head -20 gpurun_out/r05/gbdt_summary.txt
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
for g in P1 P2; do
  timeout -s KILL 120 rocprofv3 --pmc ${!g} --kernel-include-regex "hist_build|grad_hess" --output-format csv -d gpurun_out/r05/gbdt_pmc/$g -o run -- python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 10 > gpurun_out/r05/gbdt_pmc/$g.log 2>&1
  rc=$?; echo "$g rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05/gbdt_pmc/$g.log; exit $rc; }
done
exit 0
