#!/bin/bash
# Round 5: RCCL channel count vs the fixed CTR exchange's world-1 all-to-alls.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  for ch in def 16 32 64; do
    if [ $ch = def ]; then e="A=1"; else e="NCCL_MIN_NCHANNELS=$ch"; fi
    env $e timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange fixed > gpurun_out/r05/ctrch_$ch$i.log 2>&1 || { tail -20 gpurun_out/r05/ctrch_$ch$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/ctrch_$ch$i.log') if l.startswith('{')][-1]);print('ch=$ch', round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,2),'M/s')"
  done
done
