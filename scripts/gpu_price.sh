#!/bin/bash
# Price the A / B operand streams of the LDS-DMA conv GEMM (timing-only builds: dropped loads read zeros).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for price in none A B AB; do
  case $price in none) unset KDL_TUNE;; A) export KDL_TUNE=igemm_price=1;; B) export KDL_TUNE=igemm_price=2;; *) export KDL_TUNE=igemm_price=3;; esac
  timeout -k 10 200 python -u scripts/time_igemm.py ${1:-3x3} > gpurun_out/price_$price.jsonl 2>gpurun_out/price_$price.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/price_$price.err; exit $rc; }
done
exit 0
