#!/bin/bash
# Round 5: host-side profile (cProfile) of the CTR worker, fixed exchange vs sync-free.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for ex in fixed auto; do
  timeout -k 10 200 python3 -m cProfile -o gpurun_out/r05/ctr_cprof_$ex.prof -m kubedl_amd.workers.xdl_ctr --steps 500 --warmup 20 --exchange $ex > gpurun_out/r05/ctr_cprof_$ex.log 2>&1 || { tail -20 gpurun_out/r05/ctr_cprof_$ex.log; exit 1; }
  python3 -c "
import pstats
p = pstats.Stats('gpurun_out/r05/ctr_cprof_$ex.prof')
p.sort_stats('tottime').print_stats(30)
" > gpurun_out/r05/ctr_cprof_$ex.txt
done
