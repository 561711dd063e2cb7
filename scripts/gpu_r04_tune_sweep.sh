#!/bin/bash
# Re-sweep of native knobs on the current step (job-path bench, interleaved):
#   scripts/gpu_r04_tune_sweep.sh "wgrad_blocks=256" "" "wgrad_blocks=384" ...
# ("" = defaults).  One line per run: <KDL_TUNE> <img/s> <ms/step>.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  k=0
  for t in "$@"; do
    k=$((k + 1))
    if [ -n "$t" ]; then export KDL_TUNE="$t"; else unset KDL_TUNE; fi
    timeout -k 10 300 python -u bench.py > gpurun_out/r04_tune_${k}_$rep.log 2>&1 || exit 1
    echo "${t:-default} $(tail -1 gpurun_out/r04_tune_${k}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
