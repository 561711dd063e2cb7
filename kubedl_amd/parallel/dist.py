"""Process-group bootstrap for rank processes launched by the kubedl_amd runtime.

The launchers (``kubedl_amd.controllers.*``) export exactly the rendezvous
environment KubeDL injects into pods -- ``MASTER_ADDR``, ``MASTER_PORT``,
``WORLD_SIZE``, ``RANK`` (``controllers/pytorch/pytorchjob_controller.go:180-233``)
-- plus ``LOCAL_RANK`` and ``HIP_VISIBLE_DEVICES`` from the gang allocator.
One process drives one MI355X; the backend is ``nccl`` (= RCCL over xGMI on
ROCm) on GPU and ``gloo`` on CPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_master(self) -> bool:
        return self.rank == 0


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_from_env(device: str | None = None, timeout_s: float = 600.0) -> DistInfo:
    rank = env_int("RANK", 0)
    world = env_int("WORLD_SIZE", 1)
    local_rank = env_int("LOCAL_RANK", 0)
    use_gpu = device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(ndev, 1))
        torch.cuda.set_device(dev)
        # KDL_DIST_BACKEND=gloo: rehearse a multi-rank job on fewer GPUs than
        # ranks (gloo moves CUDA tensors through host memory; RCCL would
        # refuse two ranks on one device)
        backend = os.environ.get("KDL_DIST_BACKEND", "nccl")
    else:
        dev = torch.device("cpu")
        backend = "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "23456")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistInfo(rank, world, local_rank, dev, backend)


def barrier(info: DistInfo) -> None:
    if info.world_size > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def all_reduce_max(value: float, info: DistInfo) -> float:
    if info.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if info.world_size > 1 and dist.is_initialized():
        dist.destroy_process_group()
