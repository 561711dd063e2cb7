#!/bin/bash
# Tile-config sweep of the fused 1x1-conv GEMMs (KDL_TUNE gemm_cfg 0..3) on one MI355X.
mkdir -p gpurun_out
for c in ${CFGS:-0 1 2 3}; do
  KDL_TUNE=gemm_cfg=$c timeout -k 10 300 python -u scripts/bench_conv1x1.py > gpurun_out/gemm_cfg$c.log 2>&1 || exit $?
  tail -1 gpurun_out/gemm_cfg$c.log
done
