#!/bin/bash
# Bench A/B: env variants, interleaved rounds (bench.py --direct, one process per run).
# usage: gpu_bench_ab.sh "NAME1:ENV=V ENV=V" "NAME2:..." ...   (ROUNDS, STEPS env)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 180 python bench.py --direct --steps ${STEPS:-20} --warmup 5 > gpurun_out/ab_${name}_r$r.log 2>&1
    rc=$?
    echo "$name r$r rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_${name}_r$r.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
