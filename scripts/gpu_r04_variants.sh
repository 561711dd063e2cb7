#!/bin/bash
# Round 4 A/B of conv GEMM main-loop variants:
#   base      _C.so
#   pro       _C.so + KDL_TUNE=igemm_pro=1: BN+ReLU-prologue forward statistics GEMMs on the LDS-DMA loop
#   spread    _C_alt.so  (KDL_IGEMM_SPREAD=1): the next K-step's DMA spread over the MFMA sub-steps
#   fragpipe  _C_alt2.so (KDL_IGEMM_FRAGPIPE=1): fragment reads one sub-step ahead (not 256x256)
# Correctness first (each variant's tests), kernel probes, then the step, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
setv() {
  unset KDL_C_PATH KDL_TUNE
  case $1 in
    pro) export KDL_TUNE=igemm_pro=1;;
    spread) export KDL_C_PATH=$PWD/kubedl_amd/_C_alt.so;;
    fragpipe) export KDL_C_PATH=$PWD/kubedl_amd/_C_alt2.so;;
  esac
}
T="tests/test_conv3x3_gpu.py tests/test_dgrad_s2_gpu.py tests/test_igemm_gpu.py"
for v in base spread fragpipe; do
  setv $v
  extra=""; [ $v = base ] && extra=tests/test_igemm_pro_gpu.py
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $extra $T \
    > gpurun_out/var_tests_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/var_tests_$v.log)"; [ $rc -eq 0 ] || exit 1
done
setv base
timeout -k 10 300 python scripts/gemm1x1_core_probe.py > gpurun_out/gemm1x1_core_probe.log 2>&1 || exit $?
grep -o '"shape.*' gpurun_out/gemm1x1_core_probe.log
for v in base spread fragpipe; do
  setv $v
  timeout -k 10 300 python scripts/igemm_cfg_probe.py > gpurun_out/var_probe_$v.log 2>&1 || exit $?
  echo "== $v"; grep -o '"shape.*' gpurun_out/var_probe_$v.log
done
for r in 1 2; do
  for v in ${VARS:-base pro spread fragpipe}; do
    setv $v
    timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/var_${v}_r$r.log 2>&1 || exit $?
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/var_${v}_r$r.log)"
  done
done
