#!/bin/bash
# Round 5: host cost of a world-1 RCCL all-to-all call (scripts/a2a_call_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 120 python3 -u scripts/a2a_call_probe.py > gpurun_out/r05/a2a_call.log 2>&1 || { tail -20 gpurun_out/r05/a2a_call.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05/a2a_call.log
