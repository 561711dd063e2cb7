#!/bin/bash
# Round 5 (end): the full GPU test suite, the job-path bench twice, then smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05/final_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r05/final_suite.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/bench_final$i.json 2> gpurun_out/r05/bench_final$i.err || exit $?
  tail -1 gpurun_out/r05/bench_final$i.json | cut -c1-200
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/bench_final$i.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','time_to_first_step_s','rank_ready_s','comm_init_s','first_step_s')})"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke_final.log 2>&1 || { tail -20 gpurun_out/r05/smoke_final.log; exit 1; }
tail -1 gpurun_out/r05/smoke_final.log
