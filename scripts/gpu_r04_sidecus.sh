#!/bin/bash
# Round 4 A/B: the weight-gradient side stream on a partial CU mask
# (EngineOptions.side_cus; 0 = pool stream on all CUs, 256 = full-mask own queue).
# bench.py --direct, interleaved, two rounds.  (Historical: every mask lost ~29 %,
# profiles/r04_side_stream_cu_mask_ab.txt, and the option was removed again.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for c in ${CUS:-0 256 192 128 64}; do
    KDL_ENGINE="side_cus=$c" timeout -k 10 180 python bench.py --direct --steps 20 --warmup 6 > gpurun_out/cus_${c}_r$r.log 2>&1 || exit $?
    echo "side_cus=$c r$r $(grep -o '"value": [0-9.]*' gpurun_out/cus_${c}_r$r.log)"
  done
done
