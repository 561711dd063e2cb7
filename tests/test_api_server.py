"""The manager's HTTP API (kubedl_amd/cli/server.py): apply/list/get, the job
summary and the HTML dashboard, metrics, 404s."""
import json
import os
import sys
import urllib.error
import urllib.request

import pytest

from kubedl_amd.cli.server import APIServer
from kubedl_amd.engine.manager import Manager, ManagerOptions

PY = sys.executable


@pytest.fixture()
def api(tmp_path):
    os.environ["KDL_RESTART_BACKOFF_BASE"] = "0.05"
    m = Manager(ManagerOptions(home=str(tmp_path), gpus=8, metrics_port=0)).start()
    srv = APIServer(m, 0).start()
    yield m, f"http://127.0.0.1:{srv.port}"
    srv.stop()
    m.stop()
    os.environ.pop("KDL_RESTART_BACKOFF_BASE", None)


def _get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.status, r.headers.get("Content-Type"), r.read().decode()


def test_apply_summary_dashboard_metrics(api):
    m, base = api
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "web", "namespace": "default"},
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": {"spec": {"containers": [
               {"name": "pytorch", "image": "x", "command": [PY, "-c", "import time; time.sleep(0.2)"]}]}}}}}}
    req = urllib.request.Request(base + "/api/apply", data=json.dumps(job).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=10) as r:
        assert r.status == 201
    m.wait_for_condition("PyTorchJob", "default", "web", ["Succeeded"], timeout=60)
    code, _, body = _get(base + "/api/objects/pytorchjobs")
    assert code == 200 and [j["metadata"]["name"] for j in json.loads(body)["items"]] == ["web"]
    code, _, body = _get(base + "/api/summary")
    rows = json.loads(body)["items"]
    assert rows[0]["name"] == "web" and rows[0]["state"] == "Succeeded"
    assert rows[0]["replicas"]["Master"] == {"succeeded": 1}
    assert rows[0]["first_pod_launch_delay_s"] is not None
    code, ctype, body = _get(base + "/dashboard")
    assert code == 200 and ctype.startswith("text/html") and "<td>web</td>" in body and "Succeeded" in body
    code, _, body = _get(base + "/metrics")
    assert 'kubedl_jobs_successful{kind="pytorchjob"} 1.0' in body
    with pytest.raises(urllib.error.HTTPError) as e:
        _get(base + "/api/objects/pytorchjobs/default/nope")
    assert e.value.code == 404
