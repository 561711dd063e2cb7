#!/bin/bash
# Round 6: A/B of the tile of the N = 256 implicit GEMMs (stage 3: KDL_TUNE igemm_n256 = 0 (256x256, default),
# 1 (256x128), 2 (128x128 two blocks/CU)) in the two-stream step, driver flags, interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2 3; do
  for c in 0 1 2; do
    KDL_TUNE=igemm_n256=$c timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/n256_${c}_$i.json 2> gpurun_out/r06/n256_${c}_$i.err || { tail -20 gpurun_out/r06/n256_${c}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r06/n256_${c}_$i.json').read().strip().splitlines()[-1]);print('n256=$c run $i', d['value'], d['ms_per_step'], d['step_ms']['median'])"
  done
done
