"""World-1 RCCL all-reduce through the engine's direct-mode DDP on a real
MI355X (``KDL_TUNE ddp_world1=1``): a one-rank "nccl" (= RCCL) process group, the
gradient buckets launched from inside the fused backward and all-reduced by
RCCL exactly as on N GPUs -- the result must equal the step without DDP
(a one-rank sum is the identity, scale 1)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

_CHILD = r"""
import os, socket, sys
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["KDL_REPO"])
from kubedl_amd.parallel.dist import DistInfo
from kubedl_amd.workers.resnet50 import ResNetTrainer
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
info = DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl")
out = []
for world1 in ("1", "0"):
    os.environ["KDL_TUNE"] = f"ddp_world1={world1}"
    tr = ResNetTrainer(info, batch=8, image=64, num_classes=10, bn_backend="hip", engine="fused",
                       bucket_cap_mb=2.0, seed=0)
    assert tr.ddp.active == (world1 == "1") and (world1 == "0" or len(tr.ddp.buckets) > 1)
    losses = [float(tr.step()) for _ in range(2)]
    torch.cuda.synchronize()
    out.append((losses, tr.space.master.detach().clone()))
(l1, m1), (l0, m0) = out
# (BN sums use replica-spread fp32 atomics: run-to-run bits may differ slightly)
torch.testing.assert_close(torch.tensor(l1), torch.tensor(l0), atol=1e-3, rtol=1e-3)
# (the atomics' rounding is amplified by two SGD steps in a few of 23.5M weights;
# a dropped or double-counted bucket would move whole tensors by ~lr * grad)
torch.testing.assert_close(m1, m0, atol=5e-3, rtol=5e-2)
assert (m1 - m0).abs().mean().item() < 1e-5 * max(1.0, m0.abs().mean().item())
dist.destroy_process_group()
print("WORLD1_OK")
"""


def test_world1_rccl_allreduce_in_engine_step():
    env = dict(os.environ, KDL_REPO=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "WORLD1_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
