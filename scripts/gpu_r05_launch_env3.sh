#!/bin/bash
# Round 5: stream priority and the slow hipLaunchKernel path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/lenv
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/launch_probe.py > gpurun_out/r05/launch_probe2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05/launch_probe2.txt
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 180 python3 bench.py --direct --steps 30 --warmup 8 > gpurun_out/r05/lenv/$tag.json 2> gpurun_out/r05/lenv/$tag.err || { echo "$tag failed rc=$?"; tail -5 gpurun_out/r05/lenv/$tag.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/lenv/$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'))"
}
run base A=1 || exit 1
run prio0 KDL_TUNE=main_prio=0 || exit 1
run dedicated KDL_TUNE=streams=dedicated || exit 1
run prio0b KDL_TUNE=main_prio=0 || exit 1
run base2 A=1 || exit 1
