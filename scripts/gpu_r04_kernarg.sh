#!/bin/bash
# A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the
# default, job-path bench and CTR worker, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in default devkernarg; do
    if [ $v = devkernarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 300 python -u bench.py > gpurun_out/r04_kernarg_bench_${v}_$i.log 2>&1 || exit 1
    echo "bench $v $i $(tail -1 gpurun_out/r04_kernarg_bench_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    timeout -k 10 240 python -u -m kubedl_amd.workers.xdl_ctr --steps 200 --warmup 10 > gpurun_out/r04_kernarg_ctr_${v}_$i.log 2>&1 || exit 1
    echo "ctr $v $i $(tail -1 gpurun_out/r04_kernarg_ctr_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["samples_per_sec"]/1e6,3))')"
  done
done
