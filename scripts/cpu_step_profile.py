"""Host-side cost of one ResNet-50 training step (cProfile over K steps).
The GPU side is in the rocprofv3 summaries; this shows what the CPU spends
issuing the ~500 launches per step."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402  (sets the MIOpen db env)
import torch  # noqa: E402
from kubedl_amd.parallel.dist import DistInfo  # noqa: E402
from kubedl_amd.workers.resnet50 import ResNetTrainer  # noqa: E402

info = DistInfo(0, 1, 0, torch.device("cuda", 0), "nccl")
tr = ResNetTrainer(info, batch=256, image=224)
for _ in range(5):
    tr.step()
torch.cuda.synchronize()
K = 10
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    tr.step()
pr.disable()
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"host issue time {t_issue / K * 1e3:.2f} ms/step (profiled), wall {t_all / K * 1e3:.2f} ms/step")
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
