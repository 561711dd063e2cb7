"""``kdl``: the operator binary + kubectl-like client for the local MI355X runtime.

Server (``main.go`` flags kept by name)::

    python -m kubedl_amd.cli manager [--metrics-addr 8443] [--controller-metrics-addr :8080]
        [--enable-leader-election=true] [--gang-scheduler-name kdl-gang]
        [--max-reconciles N] [--workloads auto|*|TFJob,...] [--object-storage sqlite]
        [--event-storage jsonl] [--region R] [--api-addr 127.0.0.1:8098] [--gpus N]

Client (talks to ``--api-addr`` / ``$KDL_API``)::

    kdl apply -f job.yaml        kdl get pytorchjobs [NAME] [-o json|yaml]
    kdl describe tfjob NAME      kdl delete xdljob NAME
    kdl logs POD [-c CONTAINER]  kdl top

One-shot (in-process control plane, no daemon)::

    kdl run -f job.yaml [--timeout S] [--gang]   # submit, wait for Succeeded/Failed, print status
    kdl bench-launch [--jobs N] [--gpus-per-job G]  # launch-delay benchmark (BASELINE.md metric)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import urllib.error
import urllib.request
from typing import List, Optional

from kubedl_amd.api import codec
from kubedl_amd.api import common as c
from kubedl_amd.api import kinds as K

DEFAULT_API = os.environ.get("KDL_API", "127.0.0.1:8098")


# ---------------------------------------------------------------- client helpers
class Client:
    def __init__(self, addr: str = DEFAULT_API):
        self.base = "http://" + addr

    def _req(self, method: str, path: str, body=None):
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.base + path, data=data, method=method,
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=30) as r:
                raw = r.read().decode()
                ctype = r.headers.get("Content-Type", "")
        except urllib.error.HTTPError as e:
            msg = e.read().decode()
            try:
                msg = json.loads(msg).get("error", msg)
            except ValueError:
                pass
            raise SystemExit(f"error: {msg}")
        except urllib.error.URLError as e:
            raise SystemExit(f"error: cannot reach kdl manager at {self.base} ({e.reason}); "
                             "start one with `python -m kubedl_amd.cli manager`")
        return json.loads(raw) if ctype.startswith("application/json") else raw

    def apply(self, obj):
        return self._req("POST", "/api/apply", obj)

    def list(self, kind, ns=None):
        q = f"?namespace={ns}" if ns else ""
        return self._req("GET", f"/api/objects/{kind}{q}")["items"]

    def get(self, kind, ns, name):
        return self._req("GET", f"/api/objects/{kind}/{ns}/{name}")

    def delete(self, kind, ns, name):
        return self._req("DELETE", f"/api/objects/{kind}/{ns}/{name}")

    def events(self, ns=None, uid=None):
        q = "&".join(x for x in (f"namespace={ns}" if ns else "", f"uid={uid}" if uid else "") if x)
        return self._req("GET", "/api/events" + ("?" + q if q else ""))["items"]

    def logs(self, ns, pod, container=None, tail=None):
        q = "&".join(x for x in (f"container={container}" if container else "", f"tail={tail}" if tail else "") if x)
        return self._req("GET", f"/api/logs/{ns}/{pod}" + ("?" + q if q else ""))

    def node(self):
        return self._req("GET", "/api/node")


def _table(rows: List[dict], cols: List[str]) -> str:
    widths = {k: max([len(k)] + [len(str(r.get(k, ""))) for r in rows]) for k in cols}
    lines = ["   ".join(k.ljust(widths[k]) for k in cols)]
    for r in rows:
        lines.append("   ".join(str(r.get(k, "")).ljust(widths[k]) for k in cols))
    return "\n".join(lines)


def _is_job_kind(kind: str) -> bool:
    try:
        K.lookup(kind)
        return True
    except KeyError:
        return False


def print_objects(kind: str, objs: List[dict], fmt: Optional[str]) -> None:
    if fmt in ("json", "yaml"):
        print(codec.dumps(objs, fmt))
        return
    if _is_job_kind(kind):
        print(_table([K.print_columns(o) for o in objs], ["NAME", "STATE", "AGE", "FINISHED-TTL", "MAX-LIFETIME"]))
    elif kind.lower() in ("pod", "pods", "po"):
        rows = []
        for p in objs:
            st = p.get("status") or {}
            cs = st.get("containerStatuses") or []
            rows.append({"NAME": p["metadata"]["name"], "READY": f"{sum(1 for x in cs if x.get('ready'))}/{len(cs)}",
                         "STATUS": st.get("phase", ""), "RESTARTS": sum(int(x.get("restartCount", 0)) for x in cs),
                         "GPUS": (p["metadata"].get("annotations") or {}).get("kubedl.io/gpus", "")})
        print(_table(rows, ["NAME", "READY", "STATUS", "RESTARTS", "GPUS"]))
    else:
        print(_table([{"NAME": o["metadata"]["name"], "NAMESPACE": o["metadata"]["namespace"]} for o in objs],
                     ["NAME", "NAMESPACE"]))


def describe(job: dict, events: List[dict]) -> str:
    md = job["metadata"]
    st = job.get("status") or {}
    out = [f"Name:         {md['name']}", f"Namespace:    {md['namespace']}", f"Kind:         {job['kind']}",
           f"UID:          {md.get('uid', '')}", f"Created:      {md.get('creationTimestamp', '')}",
           f"Start Time:   {st.get('startTime', '')}", f"Completion:   {st.get('completionTime', '')}",
           "Replica Statuses:"]
    for rt, rs in (st.get("replicaStatuses") or {}).items():
        out.append(f"  {rt}: active={c.rs_get(rs, 'active')} succeeded={c.rs_get(rs, 'succeeded')} "
                   f"failed={c.rs_get(rs, 'failed')}")
    out.append("Conditions:")
    for cond in st.get("conditions") or []:
        out.append(f"  {cond['type']:<11} {cond['status']:<6} {cond.get('reason', ''):<15} {cond.get('message', '')}")
    out.append("Events:")
    for e in events:
        out.append(f"  {e.get('type', ''):<8} {e.get('reason', ''):<24} x{e.get('count', 1):<3} {e.get('message', '')}")
    return "\n".join(out)


# ---------------------------------------------------------------- commands
def cmd_manager(a) -> int:
    import logging
    import signal
    from kubedl_amd.cli.server import APIServer
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    from kubedl_amd.metrics import parse_addr
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    mhost, mport = parse_addr(a.metrics_addr)
    chost, cport = parse_addr(a.controller_metrics_addr)
    opts = ManagerOptions(home=a.home, durable=True, workloads=a.workloads,
                          gang_scheduler_name=a.gang_scheduler_name,
                          max_reconciles=a.max_reconciles if a.max_reconciles > 0 else 1,
                          metrics_port=mport, metrics_host=mhost, controller_metrics_port=cport,
                          controller_metrics_host=chost, leader_election=a.enable_leader_election,
                          gpus=a.gpus, object_storage=a.object_storage,
                          event_storage=a.event_storage, region=a.region or os.environ.get("REGION", ""))
    if a.enable_leader_election:
        print(f"kdl manager: waiting for leadership of {os.path.join(a.home, 'leader.lock')}", flush=True)
    mgr = Manager(opts).start()
    host, aport = a.api_addr.rsplit(":", 1)
    api = APIServer(mgr, int(aport), host or "127.0.0.1").start()
    print(f"kdl manager up: api http://{host or '127.0.0.1'}:{api.port}  "
          f"controllers={sorted(mgr.loops)}  gpus={mgr.allocator.inv.count if mgr.allocator else 0}  "
          f"gang={a.gang_scheduler_name or 'off'}  metrics=:{mport or 'off'}  controller-metrics=:{cport or 'off'}  "
          f"leader-election={'on' if a.enable_leader_election else 'off'}", flush=True)
    stop = []
    signal.signal(signal.SIGTERM, lambda *_: stop.append(1))
    signal.signal(signal.SIGINT, lambda *_: stop.append(1))
    while not stop:
        time.sleep(0.2)
    api.stop()
    mgr.stop()
    return 0


def cmd_apply(a) -> int:
    cl = Client(a.api)
    for obj in codec.load_file(a.filename):
        if a.namespace:
            obj.setdefault("metadata", {})["namespace"] = a.namespace
        out = cl.apply(obj)
        print(f"{out['kind'].lower()}.{out['apiVersion'].split('/')[0]}/{out['metadata']['name']} created")
    return 0


def cmd_get(a) -> int:
    cl = Client(a.api)
    if a.name:
        objs = [cl.get(a.kind, a.namespace or "default", a.name)]
    else:
        objs = cl.list(a.kind, a.namespace)
    print_objects(a.kind, objs, a.output)
    return 0


def cmd_describe(a) -> int:
    cl = Client(a.api)
    job = cl.get(a.kind, a.namespace or "default", a.name)
    print(describe(job, cl.events(job["metadata"]["namespace"], job["metadata"].get("uid"))))
    return 0


def cmd_delete(a) -> int:
    Client(a.api).delete(a.kind, a.namespace or "default", a.name)
    print(f"{a.kind}/{a.name} deleted")
    return 0


def cmd_logs(a) -> int:
    sys.stdout.write(Client(a.api).logs(a.namespace or "default", a.pod, a.container, a.tail))
    return 0


def cmd_top(a) -> int:
    n = Client(a.api).node()
    print(f"GPUs: {n['gpus']} x {n['hbm_gb']} GB HBM   free: {n['free']}")
    for owner, pods in n["allocations"].items():
        for pod, gpus in pods.items():
            print(f"  {owner:<40} {pod.rsplit('/', 1)[0]:<40} gpus={gpus}")
    return 0


def cmd_run(a) -> int:
    """In-process control plane: submit manifests, wait, print final status."""
    import tempfile
    from kubedl_amd.engine.manager import Manager, ManagerOptions
    home = a.home or tempfile.mkdtemp(prefix="kdl-run-")
    # an explicit --home may be a running `kdl manager`'s: take its leader lock
    # (refuse at once if held) so two node runtimes never drive one home
    try:
        mgr = Manager(ManagerOptions(home=home, gang_scheduler_name="kdl-gang" if a.gang else "",
                                     gpus=a.gpus, leader_election=bool(a.home), leader_wait_s=0.0)).start()
    except TimeoutError as e:
        print(f"kdl run: {e} (a kdl manager runs on this home: submit with `kdl apply` instead)", file=sys.stderr)
        return 1
    rc = 0
    try:
        jobs = []
        for obj in codec.load_file(a.filename):
            if a.namespace:
                obj.setdefault("metadata", {})["namespace"] = a.namespace
            out = mgr.apply(obj)
            if out["kind"] in K.BY_KIND:
                jobs.append(out)
        for j in jobs:
            md = j["metadata"]
            fin = mgr.wait_for_condition(j["kind"], md["namespace"], md["name"], ["Succeeded", "Failed"],
                                         timeout=a.timeout)
            st = fin["status"]
            print(json.dumps({"kind": j["kind"], "name": md["name"], "state": c.last_condition_type(st),
                              "startTime": st.get("startTime"), "completionTime": st.get("completionTime"),
                              "replicaStatuses": st.get("replicaStatuses"),
                              "first_pod_launch_delay_s": mgr.metrics.observed["first"].get(md["uid"]),
                              "all_pods_launch_delay_s": mgr.metrics.observed["all"].get(md["uid"]),
                              "logs": os.path.join(home, "node", "pods")}, indent=1))
            if c.is_failed(st):
                rc = 1
    finally:
        mgr.stop()
    return rc


def cmd_bench_launch(a) -> int:
    from kubedl_amd.cli.bench_launch import main as bl
    return bl(a)


def _flag_bool(v) -> bool:
    """Go flag.Bool syntax: --flag, --flag=true|false|1|0."""
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "t", "true", "yes", "on"):
        return True
    if s in ("0", "f", "false", "no", "off"):
        return False
    raise argparse.ArgumentTypeError(f"invalid boolean value {v!r}")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="kdl", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    m = sub.add_parser("manager", help="run the controller manager + node runtime + API server")
    m.add_argument("--controller-metrics-addr", default=":8080",
                   help="controller-runtime metrics (reconcile / workqueue) endpoint; 0 = off (main.go:54)")
    m.add_argument("--metrics-addr", default="8443",
                   help="kubedl_jobs_* Prometheus endpoint: port or [host]:port; 0 = off (main.go:55)")
    m.add_argument("--enable-leader-election", default=True, nargs="?", const=True, type=_flag_bool,
                   help="only one manager per --home acts; others wait as standby (main.go:56, default true)")
    m.add_argument("--gang-scheduler-name", default="", help="enable gang scheduling (kdl-gang | kube-batch)")
    m.add_argument("--max-reconciles", type=int, default=1)
    m.add_argument("--workloads", default="auto")
    m.add_argument("--region", default="")
    m.add_argument("--object-storage", default="", help="object backend: sqlite | mysql")
    m.add_argument("--event-storage", default="", help="event backend: jsonl | sqlite | aliyun-sls")
    m.add_argument("--api-addr", default=DEFAULT_API)
    m.add_argument("--home", default=os.environ.get("KDL_HOME", os.path.expanduser("~/.kubedl_amd")))
    m.add_argument("--gpus", type=int, default=None, help="override detected GPU count")
    m.set_defaults(fn=cmd_manager)

    def client(p):
        p.add_argument("--api", default=DEFAULT_API)
        p.add_argument("-n", "--namespace", default=None)

    p = sub.add_parser("apply", help="create jobs from a manifest")
    p.add_argument("-f", "--filename", required=True)
    client(p)
    p.set_defaults(fn=cmd_apply)
    p = sub.add_parser("get")
    p.add_argument("kind")
    p.add_argument("name", nargs="?")
    p.add_argument("-o", "--output", choices=["json", "yaml", "wide"], default=None)
    client(p)
    p.set_defaults(fn=cmd_get)
    p = sub.add_parser("describe")
    p.add_argument("kind")
    p.add_argument("name")
    client(p)
    p.set_defaults(fn=cmd_describe)
    p = sub.add_parser("delete")
    p.add_argument("kind")
    p.add_argument("name")
    client(p)
    p.set_defaults(fn=cmd_delete)
    p = sub.add_parser("logs")
    p.add_argument("pod")
    p.add_argument("-c", "--container", default=None)
    p.add_argument("--tail", type=int, default=None)
    client(p)
    p.set_defaults(fn=cmd_logs)
    p = sub.add_parser("top", help="GPU allocation of the node")
    client(p)
    p.set_defaults(fn=cmd_top)
    p = sub.add_parser("run", help="submit manifests to an in-process control plane and wait")
    p.add_argument("-f", "--filename", required=True)
    p.add_argument("-n", "--namespace", default=None)
    p.add_argument("--timeout", type=float, default=3600)
    p.add_argument("--gang", action="store_true")
    p.add_argument("--gpus", type=int, default=None)
    p.add_argument("--home", default=None)
    p.set_defaults(fn=cmd_run)
    p = sub.add_parser("bench-launch", help="job launch-delay benchmark through the full control plane")
    from kubedl_amd.cli.bench_launch import add_args
    add_args(p)
    p.set_defaults(fn=cmd_bench_launch)
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
