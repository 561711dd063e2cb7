#!/bin/bash
# GPU-box check run via gpurun: numerics tests, bench A/B, rocprofv3 kernel stats.
# Every GPU step has its own timeout; a crash/timeout (exit >= 124 or signal)
# ends the script so nothing else touches the GPU after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-all}"

fatal() {  # $1 = exit code, $2 = step name
  local rc=$1
  if [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; then
    echo "[gpu_check] step '$2' ended with fatal code $rc; stopping" | tee -a gpurun_out/summary.txt
    exit "$rc"
  fi
}

run_step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[gpu_check] >>> $name" | tee -a gpurun_out/summary.txt
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] <<< $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/summary.txt
  tail -n 5 "gpurun_out/$name.log"
  fatal $rc "$name"
  return 0
}

want() { [ "$STEPS" = "all" ] || [[ ",$STEPS," == *",$1,"* ]]; }

python -c "import kubedl_amd._C" 2>/dev/null || python -m kubedl_amd.ops.build > gpurun_out/build.log 2>&1

want smoke  && run_step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
want pytest && run_step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
want pytestsub && run_step pytest_sub 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread
want bench  && run_step bench_job 600 python bench.py --gpus 1 --steps 20 --warmup 5
want benchdirect && run_step bench_direct 600 python bench.py --direct --gpus 1 --steps 20 --warmup 5
want bench2 && run_step bench_job2 600 python bench.py --gpus 1 --steps 20 --warmup 5
want benchab && run_step bench_torch 600 python bench.py --direct --steps 20 --warmup 8 --bn-backend torch
want prof   && run_step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --direct --steps 5 --warmup 3
if want prof1s; then
  KDL_ENGINE=side=0 run_step prof_1stream 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1s -o run -- python bench.py --direct --steps 5 --warmup 3
fi
want benchfind && run_step bench_find 900 python bench.py --direct --steps 20 --warmup 8 --conv-benchmark 1
want launch && run_step bench_launch 600 python -m kubedl_amd.cli bench-launch --jobs 1 --gpus 1 --steps 20 --warmup 5
if want bnsweep; then
  for mr in ${SWEEP:-128 256 512 1024}; do
    KDL_TUNE=bn_min_rows=$mr run_step bench_minrows_$mr 600 python bench.py --steps 20 --warmup 8
  done
fi
if want envsweep; then  # SWEEPVAR=<env var> SWEEP="<values>": direct bench per value
  i=0
  for v in ${SWEEP}; do
    i=$((i+1))
    export "${SWEEPVAR}=$v"
    run_step "bench_${SWEEPVAR}_${v}_r$i" 600 python bench.py --direct --gpus 1 --steps 20 --warmup 5
    unset "${SWEEPVAR}"
  done
fi
want stem && run_step time_stem 300 python -u scripts/time_stem.py
want dgrads2 && run_step time_dgrad_s2 300 python -u scripts/time_dgrad_s2.py
want convgemm && run_step conv_vs_gemm 600 python scripts/conv_vs_gemm.py
want ctr && run_step ctr 300 python -u -m kubedl_amd.workers.xdl_ctr
want ctrprof && run_step ctr_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ctr_prof -o run -- python -u -m kubedl_amd.workers.xdl_ctr --steps 10 --warmup 3
want gbdt && run_step gbdt 300 python -u -m kubedl_amd.workers.xgboost_dist
want gbdt2m && run_step gbdt_2m 300 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100
want gbdtprof && run_step gbdt_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gbdt_prof -o run -- python -u -m kubedl_amd.workers.xgboost_dist
want benchimm && run_step bench_immediate 600 python bench.py --steps 20 --warmup 8 --conv-benchmark 0
# ship the MIOpen find-db / kernel cache back (merged into gpurun_out/)
if [ -d miopen_db ]; then mkdir -p gpurun_out/miopen_db && cp -r miopen_db/. gpurun_out/miopen_db/; du -sh gpurun_out/miopen_db; fi
exit 0
