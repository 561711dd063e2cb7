#!/bin/bash
# Round 4: (1) which stream RCCL collectives run on; (2) whole-step PMC passes
# (one counter group per run, each under its own hard timeout) over the bench
# step: per-kernel HBM bytes, MFMA busy, LDS conflicts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc4
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/rccl_stream -o run -- python scripts/probe_rccl_stream.py > gpurun_out/rccl_stream.log 2>&1 || exit $?
tail -2 gpurun_out/rccl_stream.log
P1="FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc4/counters.txt 2>&1 || true
grep -o "[A-Z][A-Z0-9_]*" gpurun_out/pmc4/counters.txt | sort -u > gpurun_out/pmc4/names.txt || true
for g in P1 P2 P3; do
  use=""
  for c in ${!g}; do base=${c%_sum}; grep -qx "$base" gpurun_out/pmc4/names.txt && use="$use $c"; done
  echo "$g counters:$use"
  [ -z "$use" ] && continue
  timeout -s KILL 150 rocprofv3 --pmc $use --output-format csv -d gpurun_out/pmc4/$g -o run -- python bench.py --direct --steps 2 --warmup 2 > gpurun_out/pmc4/$g.log 2>&1
  rc=$?
  echo "$g rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc4/$g.log; exit $rc; }
done
exit 0
