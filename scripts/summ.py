"""Summarise bench JSON lines of gpurun_out/<name>.log files: ms/step, img/s, extras."""
import json
import sys

for name in sys.argv[1:]:
    row = None
    try:
        for line in open(f"gpurun_out/{name}.log"):
            if line.startswith("{"):
                row = json.loads(line)
                break
    except OSError:
        pass
    if row is None:
        print(f"{name:12s} NO JSON")
        continue
    keys = ("ms_per_step", "value", "comm_init_s", "host_issue_ms_per_step", "final_loss",
            "first_pod_launch_delay_s", "cold_first_pod_launch_delay_s")
    print(f"{name:12s} " + " ".join(f"{k.split('_')[0]}={row.get(k)}" for k in keys))
