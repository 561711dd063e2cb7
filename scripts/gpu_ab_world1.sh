#!/bin/bash
# Stream/HW-queue experiment: queue probe, then bench with a world-1 RCCL group and pool vs dedicated streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_queues.py > gpurun_out/probe_queues.log 2>&1 || exit $?
grep -E "before|after" gpurun_out/probe_queues.log
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --direct --steps 20 --warmup 5 > gpurun_out/ab_$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/ab_$name.log)"
}
for r in 1 2; do
run G_pg_ded_$r KDL_TUNE=world1_pg=1,streams=dedicated
run H_pg_pool_$r KDL_TUNE=world1_pg=1,streams=pool
run I_nopg_ded_$r KDL_TUNE=world1_pg=0,streams=dedicated
run J_pg_ded_noar_$r KDL_TUNE=world1_pg=1,streams=dedicated,loss_allreduce=0
done
