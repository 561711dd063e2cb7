#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_dma_gpu.py tests/test_conv1x1_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wgrad_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/time_igemm.py wgrad > gpurun_out/time_wgrad.jsonl 2> gpurun_out/time_wgrad.err
rc=$?; python3 -c "
import json,sys
for l in open('gpurun_out/time_wgrad.jsonl'):
    d=json.loads(l); print(d['op'], {k:d[k] for k in d if k in ('M','N','K','H','Cin','Cout','stride')}, d['variant'], d['us'], d['tflops'])"
exit $rc
