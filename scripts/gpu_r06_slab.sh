#!/bin/bash
# Round 6: weight-gradient slabs cacheable (_C_slabc.so, -DKDL_SLAB_NT=0) vs nontemporal, and the
# weight-gradient block target re-swept on the round-6 step; the driver's bench flags, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
KDL_C_PATH=$PWD/kubedl_amd/_C_slabc.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_dma_gpu.py tests/test_ctr.py -m gpu > gpurun_out/r06/slab_tests.log 2>&1 || { tail -20 gpurun_out/r06/slab_tests.log; exit 1; }
tail -1 gpurun_out/r06/slab_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/slab_$name.json 2> gpurun_out/r06/slab_$name.err || { tail -20 gpurun_out/r06/slab_$name.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/slab_$name.json') if l.startswith('{')][-1]);print('$name', d['value'], d['ms_per_step'], d['step_ms']['median'], d.get('time_to_first_step_s'), d.get('cold_first_pod_launch_delay_s'))"
}
for r in 1 2; do
  run base_$r X=1 || exit 1
  run slabc_$r KDL_C_PATH=$PWD/kubedl_amd/_C_slabc.so || exit 1
  run wb320_$r KDL_TUNE=wgrad_blocks=320 || exit 1
  run wb448_$r KDL_TUNE=wgrad_blocks=448 || exit 1
done
