#!/bin/bash
# A/B the fused GEMM: baseline tree (abl/base, built from an older commit) vs this tree.
mkdir -p gpurun_out
KDL_ROOT=$PWD/abl/base timeout -k 10 120 python -u scripts/time_gemm.py > gpurun_out/ab_base.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/time_gemm.py > gpurun_out/ab_new.log 2>&1 || exit $?
paste gpurun_out/ab_base.log gpurun_out/ab_new.log | grep -v amdgpu.ids
