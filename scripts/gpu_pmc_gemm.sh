#!/bin/bash
# PMC passes over single fused-GEMM shapes (each pass its own run, kernel-trace only).
mkdir -p gpurun_out/pmc && cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() { # name counters...
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmc/$name -o p -- python3 $R/scripts/one_gemm.py $SHAPE > $R/gpurun_out/pmc/$name.log 2>&1 || { echo "fail $name"; exit 1; }
}
for SHAPE in "64 256 56 1" "64 256 56 0" "64 256 56 3"; do
  tag=$(echo $SHAPE | tr ' ' _)
  run ${tag}_a FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  run ${tag}_w WRITE_SIZE || exit 1
  run ${tag}_b SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit 1
done
echo pmc-done
