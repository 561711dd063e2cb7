#!/bin/bash
# Generic gpurun driver: runs the steps listed in a steps file, one per line,
#   <name> <timeout_s> <command...>
# each under its own `timeout -k 10`, output to gpurun_out/<name>.log; a fatal
# exit (timeout, signal, abort) ends the run so nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
steps_file=$1
while read -r name to cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  echo "[gpu_run] >>> $name" | tee -a gpurun_out/summary.txt
  t0=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_run] <<< $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/summary.txt
  tail -n 3 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; then
    echo "[gpu_run] step '$name' ended with fatal code $rc; stopping" | tee -a gpurun_out/summary.txt
    exit "$rc"
  fi
done < "$steps_file"
exit 0
