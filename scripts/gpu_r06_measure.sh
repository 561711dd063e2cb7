#!/bin/bash
# Round 6 measurements: (1) whole-step ResNet-50 PMC passes for scripts/pmc_summary.py (bytes / MFMA per
# kernel), (2) CTR fixed-exchange rehearsal vs sync-free (interleaved), (3) GBDT PMC on the histogram kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc6 gpurun_out/r06
export TMPDIR=/tmp
P1="FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
for g in P1 P2 P3; do
  timeout -s KILL 150 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/pmc6/$g -o run -- python3 bench.py --direct --steps 2 --warmup 2 > gpurun_out/pmc6/$g.log 2>&1
  rc=$?
  echo "$g rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc6/$g.log; exit $rc; }
done
for i in 1 2; do
  for ex in fixed auto; do
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r06/ctr_$ex$i.log 2>&1 || { tail -20 gpurun_out/r06/ctr_$ex$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctr_$ex$i.log') if l.startswith('{')][-1]);print('$ex', d.get('exchange'), round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,3),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'))"
  done
done
bash scripts/gpu_r06_gbdt_pmc.sh
