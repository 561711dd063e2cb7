#!/bin/bash
# Round 6 end: the CTR step (sync-free and the fixed PS + worker rehearsal) with the round's defaults x2, then a kernel
# trace of the sync-free step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for i in 1 2; do
  for ex in auto fixed; do
    timeout -k 10 200 python -u -m kubedl_amd.workers.xdl_ctr --steps 2000 --warmup 20 --exchange $ex > gpurun_out/r06/ctre_${ex}_$i.log 2>&1 || { tail -20 gpurun_out/r06/ctre_${ex}_$i.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r06/ctre_${ex}_$i.log') if l.startswith('{')][-1]);print('$ex run $i:', round(d['steps_per_sec'],1),'steps/s', round(d['samples_per_sec']/1e6,3),'M samples/s  host', d.get('host_issue_ms_per_step'),'ms/step  loss_last', d.get('loss_last'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/ctre_prof -o run -- python3 -m kubedl_amd.workers.xdl_ctr --steps 200 --warmup 20 > gpurun_out/r06/ctre_prof.log 2>&1 || { tail -5 gpurun_out/r06/ctre_prof.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r06/ctre_prof/run_kernel_stats.csv')))
steps = 220
print('kernel time per step %.1f us over %d kernels' % (sum(int(r['TotalDurationNs']) for r in rows) / steps / 1e3, len(rows)))
for r in rows[:24]:
    print('%7.2f us/step %5.2f calls/step %7.2f us avg  %s' % (int(r['TotalDurationNs']) / steps / 1e3, int(r['Calls']) / steps, float(r['AverageNs']) / 1e3, r['Name'][:100]))
PY
