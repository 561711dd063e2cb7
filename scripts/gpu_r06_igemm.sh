#!/bin/bash
# Round 6: new LDS-DMA tile configs (5-7: 4 waves of 128-row wave tiles, accumulators in AGPRs):
# numerics vs fp32 torch, then the per-config probe on the stage 2-4 3x3 shapes with the
# hipBLASLt yardstick, then PMC on the standalone stage-3 shape (cfg 0 vs 5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_igemm_gpu.py tests/test_dgrad_s2_gpu.py > gpurun_out/r06/igemm_tests.log 2>&1 || { tail -30 gpurun_out/r06/igemm_tests.log; exit 1; }
tail -3 gpurun_out/r06/igemm_tests.log
timeout -k 10 300 python -u scripts/igemm_cfg_probe.py ${CFGS:-0,1,2,3,5,6,7} > gpurun_out/r06/igemm_cfg_probe.txt 2>&1 || { cat gpurun_out/r06/igemm_cfg_probe.txt; exit 1; }
cat gpurun_out/r06/igemm_cfg_probe.txt
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
for shape in "3x3 256 14 256 256 1 0" "3x3 256 14 256 256 1 5" "3x3 256 28 128 128 1 2" "3x3 256 28 128 128 1 6"; do
  tag=$(echo $shape | tr ' ' _)
  for g in G1 G2; do
    timeout -s KILL 60 rocprofv3 --pmc ${!g} --output-format csv -d gpurun_out/r06/pmc/${tag}_$g -o run -- python scripts/igemm_one.py $shape 3 > gpurun_out/r06/pmc_${tag}_$g.log 2>&1 || { echo "pmc $tag $g failed"; tail -5 gpurun_out/r06/pmc_${tag}_$g.log; exit 1; }
  done
done
echo done
