#!/bin/bash
# Round 4 A/B of implicit-GEMM main-loop variants, each an extension build of its
# own (kubedl_amd/ops/build.py out/defines, loaded with KDL_C_PATH):
#   base  _C.so       next K-step's DMA issued in one burst after the barrier
#   alt   _C_alt.so   KDL_IGEMM_SPREAD=1: the DMA spread over the four MFMA sub-steps
#   alt2  _C_alt2.so  KDL_IGEMM_FRAGPIPE=1: fragment reads one sub-step ahead (not 256x256)
# Correctness on each variant, the per-config kernel probe, then the step, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
so() { case $1 in base) echo "";; alt) echo "$PWD/kubedl_amd/_C_alt.so";; alt2) echo "$PWD/kubedl_amd/_C_alt2.so";; esac; }
for v in ${VARIANTS:-alt alt2}; do
  KDL_C_PATH=$(so $v) timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_conv3x3_gpu.py tests/test_dgrad_s2_gpu.py tests/test_igemm_gpu.py > gpurun_out/spread_tests_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/spread_tests_$v.log)"; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 300 python scripts/gemm1x1_core_probe.py > gpurun_out/gemm1x1_core_probe.log 2>&1 || exit $?
grep -o '"shape.*' gpurun_out/gemm1x1_core_probe.log
for v in base ${VARIANTS:-alt alt2}; do
  p=$(so $v)
  if [ -n "$p" ]; then export KDL_C_PATH=$p; else unset KDL_C_PATH; fi
  timeout -k 10 300 python scripts/igemm_cfg_probe.py > gpurun_out/spread_probe_$v.log 2>&1 || exit $?
done
unset KDL_C_PATH
for v in base ${VARIANTS:-alt alt2}; do echo "== $v"; grep -o '"shape.*' gpurun_out/spread_probe_$v.log; done
for r in 1 2; do
  for v in base ${VARIANTS:-alt alt2}; do
    p=$(so $v)
    if [ -n "$p" ]; then export KDL_C_PATH=$p; else unset KDL_C_PATH; fi
    timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/spread_${v}_r$r.log 2>&1 || exit $?
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/spread_${v}_r$r.log)"
  done
done
