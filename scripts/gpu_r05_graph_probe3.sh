#!/bin/bash
# Round 5: the dedup segment sizes cleared in dedup_insert_kernel (no memset
# node in a captured step).  CTR GPU tests (eager numerics of the change), the
# synced replay stages, then back-to-back replays at the worker's GPU shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu > gpurun_out/r05/graph3_ctr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05/graph3_ctr_tests.log; [ $rc -eq 0 ] || { echo "ctr tests exit $rc"; exit $rc; }
for st in dedup fused; do
  timeout -k 10 120 python3 -u scripts/ctr_graph_probe.py --stage $st > gpurun_out/r05/graph3_probe_$st.log 2>&1
  rc=$?; tail -2 gpurun_out/r05/graph3_probe_$st.log; [ $rc -eq 0 ] || { echo "stage $st exit $rc"; exit $rc; }
done
timeout -k 10 90 python3 -u scripts/ctr_graph_probe.py --stage time --steps 2000 --batch 4096 --fields 26 \
  --vocab 100000 --dim 64 --hidden 1024,512,256 > gpurun_out/r05/graph3_probe_time.log 2>&1
rc=$?; tail -5 gpurun_out/r05/graph3_probe_time.log; [ $rc -eq 0 ] || { echo "time exit $rc"; exit $rc; }
