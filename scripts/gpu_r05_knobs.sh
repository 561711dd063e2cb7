#!/bin/bash
# Round 5: launch / schedule knobs re-checked on the final step (bench --direct 40 steps,
# two interleaved passes; each line: tag, img/s, ms/step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/knobs
export TMPDIR=/tmp
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 180 python3 bench.py --direct --steps 40 --warmup 10 > gpurun_out/r05/knobs/$tag.json 2> gpurun_out/r05/knobs/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/r05/knobs/$tag.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/knobs/$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run base$i A=1 || exit 1
  run red1024_$i KDL_TUNE=wgrad_red_blocks=1024 || exit 1
  run red4096_$i KDL_TUNE=wgrad_red_blocks=4096 || exit 1
  run hwg384_$i KDL_TUNE=halo_wg_blocks=384 || exit 1
  run hwg192_$i KDL_TUNE=halo_wg_blocks=192 || exit 1
  run bnrows256_$i KDL_TUNE=bn_min_rows=256 || exit 1
  run sideprio_$i KDL_ENGINE=side_prio=-1 || exit 1
  run respro1024_$i KDL_ENGINE=res_pro_kmax=1024 || exit 1
done
