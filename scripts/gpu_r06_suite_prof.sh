#!/bin/bash
# Round 6: the full GPU suite on the interleaved-DMA main loop, then kernel traces of the step
# (new vs the round-5 loop in _C_base.so) for the two-stream critical-path view (scripts/timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r06/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
for arm in new base; do
  if [ $arm = base ]; then export KDL_C_PATH=$PWD/kubedl_amd/_C_base.so; else unset KDL_C_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06/prof_$arm -o run -- python3 bench.py --direct --steps 10 --warmup 4 > gpurun_out/r06/prof_$arm.log 2>&1 || exit $?
  f=$(find gpurun_out/r06/prof_$arm -name '*kernel_trace.csv' | head -1)
  python3 scripts/timeline.py "$f" --steps 4 > gpurun_out/r06/timeline_$arm.txt 2>&1 || exit $?
  cat gpurun_out/r06/timeline_$arm.txt
done
