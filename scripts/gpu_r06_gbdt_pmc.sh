#!/bin/bash
# Round 6: PMC passes over the GBDT fit (2M x 28, depth 6, 10 rounds): where hist_build_wq_kernel waits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06/gbdt_pmc
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
G2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"
G3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max"
for g in G1 G2 G3; do
  timeout -s KILL 120 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/r06/gbdt_pmc/$g -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 10 > gpurun_out/r06/gbdt_pmc_$g.log 2>&1 || { echo "pmc $g failed"; tail -5 gpurun_out/r06/gbdt_pmc_$g.log; exit 1; }
done
python3 scripts/pmc_quick.py gpurun_out/r06/gbdt_pmc/G1 gpurun_out/r06/gbdt_pmc/G2 gpurun_out/r06/gbdt_pmc/G3 | grep -A1 "hist_build\|route_flags\|partition_kernel"
