#!/bin/bash
# Round 5: side-stream block targets re-swept on the Gram-fold step (bench --direct, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/bsw
export TMPDIR=/tmp
run() {  # tag tune
  local tag=$1 t=$2
  KDL_TUNE=$t timeout -k 10 180 python3 bench.py --direct --steps 60 --warmup 10 > gpurun_out/r05/bsw/$tag.json 2> gpurun_out/r05/bsw/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/r05/bsw/$tag.err; return 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r05/bsw/$tag.json').read().strip().splitlines()[-1]);print('$tag', '$t', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run base$i "x=1" || exit 1
  run g256_$i "gram_blocks=256" || exit 1
  run g1024_$i "gram_blocks=1024" || exit 1
  run w320_$i "wgrad_blocks=320" || exit 1
  run w448_$i "wgrad_blocks=448" || exit 1
done
