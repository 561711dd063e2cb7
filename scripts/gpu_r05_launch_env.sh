#!/bin/bash
# Round 5: which HIP runtime setting removes the fixed ~56 us hipLaunchKernel path
# (host issue time per step, bench --direct).
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
run sigpool ROC_SIGNAL_POOL_SIZE=8192 || exit 1
run aql ROC_AQL_QUEUE_SIZE=65536 || exit 1
run batch DEBUG_CLR_MAX_BATCH_SIZE=1024 || exit 1
run cmdbuf GPU_MAX_COMMAND_BUFFERS=64 || exit 1
run await ROC_ACTIVE_WAIT_TIMEOUT=0 || exit 1
run cpusync DEBUG_CLR_BATCH_CPU_SYNC_SIZE=1024 || exit 1
run fgs ROC_USE_FGS_KERNARG=0 || exit 1
run skipcopy ROC_SKIP_KERNEL_ARG_COPY=1 || exit 1
run base2 A=1 || exit 1
