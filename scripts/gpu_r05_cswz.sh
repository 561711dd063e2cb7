#!/bin/bash
# Round 5: epilogue C-tile half swap (KDL_CSWZ) -- numerics of every GEMM epilogue user, an
# interleaved bench A/B against the plain-layout build, LDS-conflict PMC for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05/cswz
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv1x1_gpu.py tests/test_igemm_gpu.py tests/test_halo3x3_gpu.py tests/test_stem_gpu.py tests/test_resnet_engine.py -m gpu -k "not write_through and not gram" > gpurun_out/r05/cswz/tests.log 2>&1 || { tail -30 gpurun_out/r05/cswz/tests.log; exit 1; }
tail -1 gpurun_out/r05/cswz/tests.log
ALT="KDL_C_PATH=$PWD/kubedl_amd/_C_cplain.so"
for i in 1 2 3; do
  for m in swz plain; do
    if [ $m = plain ]; then e=$ALT; else e="A=1"; fi
    env $e timeout -k 10 240 python bench.py --direct --steps 40 --warmup 10 > gpurun_out/r05/cswz/b_$m$i.json 2> gpurun_out/r05/cswz/b_$m$i.err || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/r05/cswz/b_$m$i.json').read().strip().splitlines()[-1]);print('$m', d['value'], d['ms_per_step'])"
  done
done
for m in swz plain; do
  if [ $m = plain ]; then e=$ALT; else e="A=1"; fi
  env $e timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r05/cswz/pmc_$m -o run -- python3 bench.py --direct --steps 2 --warmup 2 > gpurun_out/r05/cswz/pmc_$m.log 2>&1 || { echo "pmc $m failed"; exit 1; }
done
echo done
