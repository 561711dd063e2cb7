#!/bin/bash
# Round 6: host-side profile of the CTR step (fixed exchange rehearsal and sync-free), cProfile over 1000 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for ex in fixed auto; do
  timeout -k 10 300 python -u -m cProfile -o gpurun_out/r06/ctr_cprof_$ex.prof -m kubedl_amd.workers.xdl_ctr --steps 1000 --warmup 20 --exchange $ex > gpurun_out/r06/ctr_cprof_$ex.log 2>&1 || { tail -20 gpurun_out/r06/ctr_cprof_$ex.log; exit 1; }
  python3 -c "
import pstats
p = pstats.Stats('gpurun_out/r06/ctr_cprof_$ex.prof')
p.sort_stats('tottime').print_stats(30)
" > gpurun_out/r06/ctr_cprof_$ex.txt 2>&1
  echo "== $ex"; head -60 gpurun_out/r06/ctr_cprof_$ex.txt | tail -40
done
