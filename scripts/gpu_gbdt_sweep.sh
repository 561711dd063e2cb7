#!/bin/bash
# GBDT 2M x 28 depth-6: boosting rounds/s and the histogram kernel's time per
# histogram chunk length (KDL_TUNE gbdt_rpb), each run under rocprofv3 --kernel-trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m kubedl_amd.ops.build > gpurun_out/build.log 2>&1 || true
for r in ${SWEEP:-512:8 1024:8 2048:8 1024:16 2048:16 1024:4}; do
  export KDL_TUNE=gbdt_rpb=${r%%:*} KDL_GBDT_UNROLL=${r##*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof_${r/:/_} -o run -- python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 > gpurun_out/gbdt_${r/:/_}.log 2>&1 || exit $?
  f=$(find gpurun_out/gprof_${r/:/_} -name "*kernel_stats.csv" | head -1)
  echo "rpb:unroll=$r $(grep '"rounds_per_sec"' gpurun_out/gbdt_${r/:/_}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rounds_per_sec"],1), round(d["boost_s"],3), d["logloss"])') hist_total_ms=$(python3 -c 'import csv,sys; print(round(sum(float(d["TotalDurationNs"]) for d in csv.DictReader(open(sys.argv[1])) if "hist_build" in d["Name"])/1e6,2))' "$f")"
done
