#!/bin/bash
# Price the A / B operand streams of the LDS-DMA conv GEMM (timing-only builds: dropped loads read zeros).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for price in none A B AB; do
  if [ "$price" = none ]; then unset KDL_IGEMM_PRICE; else export KDL_IGEMM_PRICE=$price; fi
  timeout -k 10 200 python -u scripts/time_igemm.py ${1:-3x3} > gpurun_out/price_$price.jsonl 2>gpurun_out/price_$price.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/price_$price.err; exit $rc; }
done
exit 0
