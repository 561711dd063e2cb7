#!/bin/bash
# PMC passes (one counter group per run, each under its own hard timeout) over
# single conv-GEMM configurations: where do the waves of the LDS-DMA GEMM wait?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|TA_[A-Z0-9_]*\|TCC_[A-Z0-9_]*" gpurun_out/pmc/counters.txt | sort -u > gpurun_out/pmc/names.txt || true
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
G3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max"
n=0
for shape in "3x3 256 56 64 64 1 3" "3x3 256 28 128 128 1 2" "3x3 256 14 256 256 1 0" "1x1 50176 256 1024 0" "1x1 12544 512 2048 2"; do
  n=$((n+1))
  for g in G1 G2 G3; do
    ctr="${!g}"
    # keep only counters this box knows
    use=""
    for c in $ctr; do base=${c%_sum}; base=${base%_avr}; base=${base%_max}; grep -qx "$base" gpurun_out/pmc/names.txt && use="$use $c"; done
    [ -z "$use" ] && continue
    timeout -s KILL 90 rocprofv3 --pmc $use --output-format csv -d gpurun_out/pmc/s${n}_$g -o run -- python scripts/igemm_one.py $shape 3 > gpurun_out/pmc/s${n}_$g.log 2>&1
    rc=$?
    echo "shape $n ($shape) $g rc=$rc counters:$use"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/s${n}_$g.log; exit $rc; }
  done
done
exit 0
