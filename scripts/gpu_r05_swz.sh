#!/bin/bash
# Round 5: XOR-swizzled LDS rows in the register-staged 1x1 GEMM (KDL_TUNE gemm_swz=1 vs 0):
# GEMM + engine numerics, an interleaved bench A/B, and LDS-conflict PMC on the step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/swz
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv1x1_gpu.py tests/test_resnet_engine.py -m gpu -k "not write_through and not gram" > gpurun_out/r05/swz/tests.log 2>&1 || { tail -30 gpurun_out/r05/swz/tests.log; exit 1; }
tail -2 gpurun_out/r05/swz/tests.log
for i in 1 2 3; do
  for m in 1 0; do
    KDL_TUNE=gemm_swz=$m timeout -k 10 240 python bench.py --steps 40 --warmup 10 > gpurun_out/r05/swz/b_$m$i.json 2> gpurun_out/r05/swz/b_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/swz/b_$m$i.json').read().strip().splitlines()[-1]);print('gemm_swz=$m', d['value'], d['ms_per_step'])"
  done
done
for m in 1 0; do
  KDL_TUNE=gemm_swz=$m timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r05/swz/pmc$m -o run -- python3 bench.py --direct --steps 2 --warmup 2 > gpurun_out/r05/swz/pmc$m.log 2>&1 || { echo "pmc $m rc=$?"; exit 1; }
done
echo done
