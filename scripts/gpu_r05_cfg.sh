#!/bin/bash
# Round 5: the 32-deep-K GEMM config for short-K statistics GEMMs re-checked after the LDS swizzle
# (KDL_TUNE gemm_cfg=0 forces the 64-deep 128x128 config there), bench --direct interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/cfg
export TMPDIR=/tmp
for i in 1 2 3; do
  for m in def 0; do
    if [ $m = def ]; then t="x=1"; else t="gemm_cfg=$m"; fi
    KDL_TUNE=$t timeout -k 10 240 python bench.py --direct --steps 40 --warmup 10 > gpurun_out/r05/cfg/b_$m$i.json 2> gpurun_out/r05/cfg/b_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/cfg/b_$m$i.json').read().strip().splitlines()[-1]);print('cfg=$m', d['value'], d['ms_per_step'])"
  done
done
