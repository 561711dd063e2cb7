#!/bin/bash
# Round 4: is the first-communicator cost the comgr code-object cache?  Must be
# the FIRST GPU work of a gpurun call (a fresh box).  c1 cold, c2 warm, c3 warm
# with the comgr cache off, c4 with an empty cache directory; the cache
# directory listed before and after.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/comm5
export TMPDIR=/tmp
cdir="${XDG_CACHE_HOME:-$HOME/.cache}/comgr"
{ echo "cache dir $cdir before:"; ls -la "$cdir" 2>&1 | head -5; du -sh "$cdir" 2>&1; } > gpurun_out/comm5/cache.txt
timeout -k 10 120 python scripts/probe_comm_init.py > gpurun_out/comm5/c1.log 2>&1 || exit $?
{ echo "after c1:"; ls -la "$cdir" 2>&1 | head -8; du -sh "$cdir" 2>&1; } >> gpurun_out/comm5/cache.txt
timeout -k 10 120 python scripts/probe_comm_init.py > gpurun_out/comm5/c2.log 2>&1 || exit $?
AMD_COMGR_CACHE=0 timeout -k 10 120 python scripts/probe_comm_init.py > gpurun_out/comm5/c3.log 2>&1 || exit $?
mkdir -p /tmp/comgr_empty
AMD_COMGR_CACHE_DIR=/tmp/comgr_empty timeout -k 10 120 python scripts/probe_comm_init.py > gpurun_out/comm5/c4.log 2>&1 || exit $?
{ echo "after c4 (/tmp/comgr_empty):"; ls -la /tmp/comgr_empty 2>&1 | head -5; du -sh /tmp/comgr_empty 2>&1; } >> gpurun_out/comm5/cache.txt
for i in 1 2 3 4; do echo "c$i $(grep -h '^{' gpurun_out/comm5/c$i.log)"; done
cat gpurun_out/comm5/cache.txt
