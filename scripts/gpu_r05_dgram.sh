#!/bin/bash
# Round 5: Gram fold for the stride-1 downsample conv's weight gradient -- engine GPU tests,
# then an interleaved bench A/B (KDL_TUNE down_gram=1 vs 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_resnet_engine.py -m gpu > gpurun_out/r05/dgram_tests.log 2>&1 || { tail -30 gpurun_out/r05/dgram_tests.log; exit 1; }
tail -2 gpurun_out/r05/dgram_tests.log
for i in 1 2 3; do
  for m in 1 0; do
    KDL_TUNE=down_gram=$m timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/dgram_$m$i.json 2> gpurun_out/r05/dgram_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/dgram_$m$i.json').read().strip().splitlines()[-1]);print('down_gram=$m', d['value'], d['ms_per_step'])"
  done
done
