#!/bin/bash
# Round 5: where the fixed-exchange CTR step's host time goes (cProfile, 600 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 200 python -u -m cProfile -o gpurun_out/r05/ctr_fixed.pstats -m kubedl_amd.workers.xdl_ctr --steps 600 --warmup 20 --exchange fixed > gpurun_out/r05/ctr_hostprof.log 2>&1 || { tail -20 gpurun_out/r05/ctr_hostprof.log; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/r05/ctr_fixed.pstats')
p.sort_stats('tottime').print_stats(45)
" > gpurun_out/r05/ctr_hostprof_top.txt
head -80 gpurun_out/r05/ctr_hostprof_top.txt
