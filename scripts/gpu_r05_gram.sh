#!/bin/bash
# Round 5: Gram-fold conv3 weight gradient (KDL_ENGINE bn_bwd_fuse=3) -- numerics,
# then an interleaved bench A/B against the default (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_resnet_engine.py -m gpu -k "gram" > gpurun_out/r05/gram_tests.log 2>&1 || { tail -40 gpurun_out/r05/gram_tests.log; exit 1; }
tail -3 gpurun_out/r05/gram_tests.log
for i in 1 2; do
  for m in 3 1; do
    KDL_ENGINE=bn_bwd_fuse=$m timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/gram_ab_$m$i.json 2> gpurun_out/r05/gram_ab_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/gram_ab_$m$i.json').read().strip().splitlines()[-1]);print('fuse=$m', {k:d.get(k) for k in ('value','ms_per_step','host_issue_ms_per_step')})"
  done
done
