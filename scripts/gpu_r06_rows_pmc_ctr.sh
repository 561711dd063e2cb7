#!/bin/bash
# Round 6: PMC of the row-per-lane GBDT histogram build (10 rounds), then the CTR igemm tests / probe / A/B
# (scripts/gpu_r06_ctr_igemm.sh), then one driver-flag ResNet bench on this lease.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06/gbdtr_pmc
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
G2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"
for g in G1 G2; do
  timeout -s KILL 120 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/r06/gbdtr_pmc/$g -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 10 > gpurun_out/r06/gbdtr_pmc_$g.log 2>&1 || { echo "pmc $g failed"; tail -5 gpurun_out/r06/gbdtr_pmc_$g.log; exit 1; }
done
python3 scripts/pmc_quick.py gpurun_out/r06/gbdtr_pmc/G1 gpurun_out/r06/gbdtr_pmc/G2 | grep -A1 "hist_build" || true
bash scripts/gpu_r06_ctr_igemm.sh || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json 2> gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err || { tail -20 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.err; exit 1; }
tail -1 gpurun_out/r06/final_bench_${FINAL_TAG:-c}.json | cut -c1-300
