#!/bin/bash
# Round 5: focused A/B of the halo weight-gradient block target and the BN row threshold
# (bench --direct 60 steps, three interleaved passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/knobs2
export TMPDIR=/tmp
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 180 python3 bench.py --direct --steps 60 --warmup 10 > gpurun_out/r05/knobs2/$tag.json 2> gpurun_out/r05/knobs2/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/r05/knobs2/$tag.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/knobs2/$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'])"
}
for i in 1 2 3; do
  run base$i A=1 || exit 1
  run hwg192_$i KDL_TUNE=halo_wg_blocks=192 || exit 1
  run hwg128_$i KDL_TUNE=halo_wg_blocks=128 || exit 1
  run both_$i KDL_TUNE=halo_wg_blocks=192,bn_min_rows=256 || exit 1
done
