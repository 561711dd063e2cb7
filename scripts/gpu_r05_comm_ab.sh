#!/bin/bash
# Round 5: RCCL bootstrap on a helper thread during the model build (comm_overlap=1)
# vs after it (0), interleaved, job path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
for i in 1 2; do
  for ov in 1 0; do
    KDL_TUNE=comm_overlap=$ov timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/comm_ab_$ov$i.json 2> gpurun_out/r05/comm_ab_$ov$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/comm_ab_$ov$i.json').read().strip().splitlines()[-1]);print('overlap=$ov', {k:d.get(k) for k in ('value','host_issue_ms_per_step','time_to_first_step_s','rank_ready_s','comm_init_s','first_step_s','startup')})"
  done
done
