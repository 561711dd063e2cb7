#!/bin/bash
# Round 5: the fixed-capacity (PS + worker) CTR exchange on HIP kernels -- its GPU
# tests, the world-1 rehearsal (exact capacity, and adaptive slack 1.5) vs the
# sync-free path (2,000 steps each, interleaved), and a kernel summary of the
# rehearsal step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu \
  -k "a2a or rehearsal or fixed_exchange or world1_step or fused_pull or segment_reduce or embed" > gpurun_out/r05/ctr_tests.log 2>&1 || { tail -30 gpurun_out/r05/ctr_tests.log; exit 1; }
tail -1 gpurun_out/r05/ctr_tests.log
for i in 1 2; do
  for ex in fixed slack auto; do
    a=$ex; s=0; [ $ex = slack ] && { a=fixed; s=1.5; }
    KDL_TUNE=ctr_a2a_slack=$s timeout -k 10 240 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $a > gpurun_out/r05/ctr_$ex$i.log 2>&1 || exit $?
    tail -1 gpurun_out/r05/ctr_$ex$i.log
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/ctr_fixed_prof -o run -- python -u -m kubedl_amd.workers.xdl_ctr --steps 50 --warmup 10 --exchange fixed > gpurun_out/r05/ctr_fixed_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r05/ctr_fixed_prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 60 > gpurun_out/r05/ctr_fixed_summary.txt; head -12 gpurun_out/r05/ctr_fixed_summary.txt
