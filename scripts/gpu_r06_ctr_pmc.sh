#!/bin/bash
# Round 6: per-kernel roofline of the CTR step (sync-free, batch 4096, tower 1024-512-256) from the same three
# PMC passes as the ResNet table (scripts/gpu_r06_measure.sh) -> scripts/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_ctr
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
for g in P1 P2 P3; do
  rm -rf gpurun_out/pmc_ctr/$g
  timeout -s KILL 150 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/pmc_ctr/$g -o run -- python3 -m kubedl_amd.workers.xdl_ctr --steps 40 --warmup 5 > gpurun_out/pmc_ctr/$g.log 2>&1
  rc=$?
  echo "$g rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_ctr/$g.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_ctr --kdl --top 25 --steps 45 > gpurun_out/pmc_ctr/summary.txt 2>&1
cat gpurun_out/pmc_ctr/summary.txt
