#!/bin/bash
# Round 5: is the fixed ~56 us hipLaunchKernel path caused by the process group's host threads?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/lenv
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 180 python3 bench.py --direct --steps 30 --warmup 8 > gpurun_out/r05/lenv/$tag.json 2> gpurun_out/r05/lenv/$tag.err || { echo "$tag failed rc=$?"; tail -5 gpurun_out/r05/lenv/$tag.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/lenv/$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'))"
}
run base A=1 || exit 1
run nopg KDL_TUNE=world1_pg=0 || exit 1
run noloss KDL_TUNE=loss_allreduce=0 || exit 1
run nomon TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 || exit 1
run base2 A=1 || exit 1
KDL_TUNE=world1_pg=0 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r05/hipt_nopg -o run -- python3 bench.py --direct --steps 6 --warmup 3 > gpurun_out/r05/hipt_nopg.log 2>&1 || exit $?
python3 - <<'PY'
import csv, statistics
v=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open('gpurun_out/r05/hipt_nopg/run_hip_api_trace.csv')) if r['Function']=='hipLaunchKernel']
v=v[len(v)//2:]
print('nopg launches', len(v), 'median', statistics.median(v), 'mean', sum(v)/len(v), 'frac>40us', sum(x>40 for x in v)/len(v))
PY
