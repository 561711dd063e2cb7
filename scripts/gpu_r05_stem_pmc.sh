#!/bin/bash
# Round 5: the fused stem weight gradient alone -- time, then PMC passes (each its own run).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out/r05/stempmc && cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05/stempmc/t -o t -- python3 $R/scripts/one_stem.py 10 > $R/gpurun_out/r05/stempmc/t.log 2>&1 || { tail -5 $R/gpurun_out/r05/stempmc/t.log; exit 1; }
grep -h stem_wgrad $R/gpurun_out/r05/stempmc/t/t_kernel_stats.csv | cut -d, -f1-7
run() { local name=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/r05/stempmc/$name -o p -- python3 $R/scripts/one_stem.py 4 > $R/gpurun_out/r05/stempmc/$name.log 2>&1 || { echo "fail $name"; exit 1; }
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU || exit 1
run b FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
run c WRITE_SIZE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES || exit 1
echo pmc-done
