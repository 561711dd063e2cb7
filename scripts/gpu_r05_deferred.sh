#!/bin/bash
# Round 5: HIP_ENABLE_DEFERRED_LOADING vs default -- RCCL bootstrap and time to first step (job path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/defl
export TMPDIR=/tmp
for i in 1 2; do
  for m in def 1 0; do
    if [ $m = def ]; then e="A=1"; else e="HIP_ENABLE_DEFERRED_LOADING=$m"; fi
    env $e timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r05/defl/b_$m$i.json 2> gpurun_out/r05/defl/b_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/defl/b_$m$i.json').read().strip().splitlines()[-1]);print('deferred=$m', {k:d.get(k) for k in ('value','time_to_first_step_s','rank_ready_s','comm_init_s','first_step_s','startup')})"
  done
done
