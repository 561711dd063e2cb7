#!/bin/bash
# Round 5: HIP runtime log (AMD_LOG_LEVEL=4) of a short bench run -- what the slow launches wait on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
AMD_LOG_LEVEL=4 AMD_LOG_LEVEL_FILE=/tmp/amdlog.txt timeout -k 10 240 python3 bench.py --direct --steps 2 --warmup 2 > gpurun_out/r05/amdlog_bench.log 2>&1 || exit $?
ls -la /tmp/amdlog.txt* 2>/dev/null
f=$(ls -S /tmp/amdlog.txt* | head -1)
wc -l $f
tail -c 30000000 $f | gzip > gpurun_out/r05/amdlog_tail.gz
ls -la gpurun_out/r05/amdlog_tail.gz
