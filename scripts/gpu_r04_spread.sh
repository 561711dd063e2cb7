#!/bin/bash
# Round 4 A/B: the implicit GEMM's next-K-step DMA spread over the MFMA sub-steps
# (csrc/igemm.hip KDL_IGEMM_SPREAD=1, built into kubedl_amd/_C_alt.so) vs issued
# in one burst after the barrier (_C.so): correctness on the alt build, the
# per-config kernel probe on both, then the step (bench --direct), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT="$PWD/kubedl_amd/_C_alt.so"
KDL_C_PATH=$ALT timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_conv3x3_gpu.py tests/test_dgrad_s2_gpu.py tests/test_igemm_gpu.py > gpurun_out/spread_tests.log 2>&1
rc=$?; tail -2 gpurun_out/spread_tests.log; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/igemm_cfg_probe.py > gpurun_out/spread_probe_base.log 2>&1 || exit $?
KDL_C_PATH=$ALT timeout -k 10 300 python scripts/igemm_cfg_probe.py > gpurun_out/spread_probe_alt.log 2>&1 || exit $?
paste -d' ' <(grep -o '"shape.*"cfg": [0-9]*' gpurun_out/spread_probe_base.log) <(grep -o '"us": [0-9.]*' gpurun_out/spread_probe_base.log) <(grep -o '"us": [0-9.]*' gpurun_out/spread_probe_alt.log)
for r in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export KDL_C_PATH=$ALT; else unset KDL_C_PATH; fi
    timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/spread_${v}_r$r.log 2>&1 || exit $?
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/spread_${v}_r$r.log)"
  done
done
