#!/bin/bash
# Round 6: GBDT with position-indexed node ids (coalesced route / partition), then one driver-flag ResNet bench
# on this fresh lease (the round's final-bench series, profiles/r06_final_bench.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r06/gbdtp_tests.log 2>&1 || { tail -20 gpurun_out/r06/gbdtp_tests.log; exit 1; }
tail -1 gpurun_out/r06/gbdtp_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtp_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/gbdtp_$i.log') if l.startswith('{')][-1]);print('pos', {k:round(d[k],5) for k in ('rounds_per_sec','fit_rounds_per_sec','logloss','accuracy')})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/gbdtp_prof -o run -- python3 -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/r06/gbdtp_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r06/gbdtp_prof -name '*kernel_stats.csv' | head -1); head -6 "$f" | cut -c1-130
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final_bench_${FINAL_TAG:-a}.json 2> gpurun_out/r06/final_bench_${FINAL_TAG:-a}.err || { tail -20 gpurun_out/r06/final_bench_${FINAL_TAG:-a}.err; exit 1; }
tail -1 gpurun_out/r06/final_bench_${FINAL_TAG:-a}.json | cut -c1-300
