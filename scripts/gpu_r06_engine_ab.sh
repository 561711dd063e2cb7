#!/bin/bash
# Round 6: engine schedule options re-swept on the round-6 kernels (KDL_ENGINE), bench.py driver flags, interleaved x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2; do
  for arm in "" "bn_bwd_fuse_bn1=1" "bn_bwd_fuse_kmax=2048" "res_pro_kmax=2048" "side_prio=-1"; do
    tag=$(echo "${arm:-default}" | tr '=,' '__')
    KDL_ENGINE="$arm" timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/eng_${tag}_$i.json 2> gpurun_out/r06/eng_${tag}_$i.err || { tail -20 gpurun_out/r06/eng_${tag}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r06/eng_${tag}_$i.json').read().strip().splitlines()[-1]);print('${tag} run $i', d['value'], d['ms_per_step'], d['step_ms']['median'])"
  done
done
