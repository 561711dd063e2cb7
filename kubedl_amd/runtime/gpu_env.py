"""GPU visibility of a rank process (one place for the kubelet and the tests).

A Kubernetes pod sees only its own GPUs, so every rank of a reference job finds
its device at ``cuda:0`` (and ``LOCAL_RANK`` is 0 or unset).  A rank of a
gang-scheduled job here keeps exactly that contract -- its own GPU is the
FIRST entry of ``HIP_VISIBLE_DEVICES``, so ``cuda:0`` (a user image's default
``cuda`` device) and ``cuda:LOCAL_RANK`` with ``LOCAL_RANK=0`` are its own
device -- and additionally sees the rest of the gang's GPUs behind it
(ascending).  With every peer visible RCCL builds its P2P/IPC transport over
xGMI and ``hipIpcOpenMemHandle`` maps a peer's buffer for the custom
all-reduce (csrc/p2p.hip); a rank that saw only its own device would leave
both to topology guesses about devices it cannot open.  RCCL identifies
devices by PCI bus id, so the per-rank ordering of the visible set does not
matter to it.  ``LOCAL_WORLD_SIZE`` is the gang's size on this node (all
ranks on one node: parallel/p2p.py ``single_node``), and
``KDL_GANG_GPU_INDEX`` the rank's position in the ascending gang set.

Ranks of different jobs never share a visible set (the gang allocator is
all-or-nothing and exclusive).  A pod outside a gang (or with several GPUs of
its own) keeps exactly its own GPUs, ``LOCAL_RANK=0``.
"""
from __future__ import annotations

from typing import Dict, List, Optional


def rank_gpu_env(pod_gpus: List[str], gang_gpus: Optional[List[str]] = None) -> Dict[str, str]:
    pod_gpus = [str(g) for g in pod_gpus]
    if gang_gpus and len(pod_gpus) == 1 and pod_gpus[0] in [str(g) for g in gang_gpus]:
        gl = sorted({str(g) for g in gang_gpus}, key=int)
        own = pod_gpus[0]
        vis = [own] + [g for g in gl if g != own]
        return {"HIP_VISIBLE_DEVICES": ",".join(vis), "LOCAL_RANK": "0",
                "LOCAL_WORLD_SIZE": str(len(gl)), "KDL_GANG_GPU_INDEX": str(gl.index(own))}
    return {"HIP_VISIBLE_DEVICES": ",".join(pod_gpus) if pod_gpus else "-1", "LOCAL_RANK": "0",
            "LOCAL_WORLD_SIZE": "1"}
