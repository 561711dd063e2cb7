#!/bin/bash
# A/B of the GBDT histogram LDS stride (csrc/gbdt.hip KDL_HIST_PAD): base _C.so
# vs kubedl_amd/_C_hpad.so (-DKDL_HIST_PAD=1), interleaved, 2M rows x 100 rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base hpad; do
    if [ $v = hpad ]; then export KDL_C_PATH=kubedl_amd/_C_hpad.so; else unset KDL_C_PATH; fi
    timeout -k 10 240 python -u -m kubedl_amd.workers.xgboost_dist --rows 2000000 --n_estimators 100 \
      > gpurun_out/r04_gbdt_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(tail -1 gpurun_out/r04_gbdt_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rounds_per_sec"],1), round(d["boost_s"],4), d["logloss"])')"
  done
done
