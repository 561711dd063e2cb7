#!/bin/bash
# Round 4: where the first RCCL bootstrap on a fresh box spends ~3 s.  Must be
# the FIRST GPU work of a gpurun call.  c0: a GPU process that never touches
# RCCL; c1: the box's first communicator (RCCL's timestamped INFO log on
# stderr); c2: the same again, warm.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/comm4
export TMPDIR=/tmp
timeout -k 10 120 python scripts/probe_comm_init.py --no-rccl > gpurun_out/comm4/c0.log 2>&1 || exit $?
for i in 1 2; do
  NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=ALL NCCL_DEBUG_TIMESTAMP_LEVELS=ALL \
  NCCL_DEBUG_TIMESTAMP_FORMAT='[%T.%6f] ' \
    timeout -k 10 120 python scripts/probe_comm_init.py > gpurun_out/comm4/c$i.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/comm4/c0.log gpurun_out/comm4/c1.log gpurun_out/comm4/c2.log
