#!/bin/bash
# Round 5: the wave-specialised fused stem weight gradient (KDL_TUNE stem_ws=1) vs the
# 7-wave in-place kernel (0): stem + engine numerics, standalone kernel time, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/stem3
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_stem_gpu.py tests/test_resnet_engine.py -m gpu -k "not write_through and not gram" > gpurun_out/r05/stem3/tests.log 2>&1 || { tail -30 gpurun_out/r05/stem3/tests.log; exit 1; }
tail -1 gpurun_out/r05/stem3/tests.log
for m in 1 0; do
  KDL_TUNE=stem_ws=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/stem3/t$m -o t -- python3 scripts/one_stem.py 10 > gpurun_out/r05/stem3/t$m.log 2>&1 || { tail -5 gpurun_out/r05/stem3/t$m.log; exit 1; }
  grep -h "stem_wgrad" gpurun_out/r05/stem3/t$m/t_kernel_stats.csv | cut -d, -f1,2,4,6 | cut -c1-160
done
for i in 1 2 3; do
  for m in 1 0; do
    KDL_TUNE=stem_ws=$m timeout -k 10 240 python bench.py --direct --steps 40 --warmup 10 > gpurun_out/r05/stem3/b_$m$i.json 2> gpurun_out/r05/stem3/b_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/stem3/b_$m$i.json').read().strip().splitlines()[-1]);print('stem_ws=$m', d['value'], d['ms_per_step'])"
  done
done
