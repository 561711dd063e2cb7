#!/bin/bash
# Round 5: kSegFly 16 (rows in flight per segment) vs 8: CTR tests, both paths, kernel profile.
# CTR GPU tests (bitwise parity), both exchange paths twice, a kernel-time profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ctr.py -m gpu > gpurun_out/r05/segfly16_tests.log 2>&1 || { tail -30 gpurun_out/r05/segfly16_tests.log; exit 1; }
tail -1 gpurun_out/r05/segfly16_tests.log
for i in 1 2; do
  for ex in auto fixed; do
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r05/segfly16_$ex$i.log 2>&1 || { tail -20 gpurun_out/r05/segfly16_$ex$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r05/segfly16_$ex$i.log') if l.startswith('{')][-1]);print('$ex', d.get('exchange'), round(d['steps_per_sec'],1), round(d['samples_per_sec']/1e6,3),'M/s', 'host ms/step', d.get('host_issue_ms_per_step'), 'loss', d['loss_last'])"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/segfly16_prof -o run -- python3 -u -m kubedl_amd.workers.xdl_ctr --steps 60 --warmup 10 > gpurun_out/r05/segfly16_prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r05/segfly16_prof/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(f"{float(r['TotalDurationNs'])/1e3/70:8.2f} us/step  {float(r['AverageNs'])/1e3:7.2f} us avg  {r['Calls']:>5}  {r['Name'][:90]}")
PY
