#!/bin/bash
# Re-sweep of native knobs on the current step (job-path bench, interleaved):
#   scripts/gpu_r04_tune_sweep.sh "wgrad_blocks=256" "" "wgrad_blocks=384" ...
# ("" = defaults; "E:key=val,..." sets KDL_ENGINE instead of KDL_TUNE).
# One line per run: <setting> <img/s> <ms/step>.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  k=0
  for t in "$@"; do
    k=$((k + 1))
    unset KDL_TUNE KDL_ENGINE
    case "$t" in
      E:*) export KDL_ENGINE="${t#E:}" ;;
      "") ;;
      *) export KDL_TUNE="$t" ;;
    esac
    timeout -k 10 300 python -u bench.py > gpurun_out/r04_tune_${k}_$rep.log 2>&1 || exit 1
    echo "${t:-default} $(tail -1 gpurun_out/r04_tune_${k}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
