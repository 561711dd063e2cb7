#!/bin/bash
# Round 5: whole-step PMC passes over the bench step (one counter group per run, each
# under its own hard timeout; kernel-trace only, no trace domains), for scripts/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc5
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
for g in P1 P2 P3; do
  timeout -s KILL 150 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/pmc5/$g -o run -- python3 bench.py --direct --steps 2 --warmup 2 > gpurun_out/pmc5/$g.log 2>&1
  rc=$?
  echo "$g rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc5/$g.log; exit $rc; }
done
exit 0
