#!/bin/bash
# Round 5: kernel + HIP runtime trace of the bench step (host launch vs GPU start at main-stream gaps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r05/hipt -o run -- python3 bench.py --direct --steps 6 --warmup 3 > gpurun_out/r05/hipt.log 2>&1 || exit $?
ls -la gpurun_out/r05/hipt
