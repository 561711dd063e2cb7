"""GPU visibility of a rank process (one place for the kubelet and the tests).

A rank of a gang-scheduled job sees the WHOLE gang's GPU set
(``HIP_VISIBLE_DEVICES`` = the gang's GPUs on this node, ascending) and picks
its own with ``LOCAL_RANK`` = the position of its GPU in that list, plus
``LOCAL_WORLD_SIZE`` -- the process shape of ``torch.distributed.run``.  With
every peer visible RCCL can build its P2P/IPC transport over xGMI and
``hipIpcOpenMemHandle`` maps a peer's buffer for the custom all-reduce
(csrc/p2p.hip); a rank that saw only its own device would leave both to
topology guesses about devices it cannot open.  Ranks of different jobs never
share a visible set (the gang allocator is all-or-nothing and exclusive).

A pod outside a gang (or with several GPUs of its own) keeps exactly its own
GPUs, ``LOCAL_RANK=0``.
"""
from __future__ import annotations

from typing import Dict, List, Optional


def rank_gpu_env(pod_gpus: List[str], gang_gpus: Optional[List[str]] = None) -> Dict[str, str]:
    pod_gpus = [str(g) for g in pod_gpus]
    if gang_gpus and len(pod_gpus) == 1 and pod_gpus[0] in [str(g) for g in gang_gpus]:
        gl = sorted({str(g) for g in gang_gpus}, key=int)
        return {"HIP_VISIBLE_DEVICES": ",".join(gl), "LOCAL_RANK": str(gl.index(pod_gpus[0])),
                "LOCAL_WORLD_SIZE": str(len(gl))}
    return {"HIP_VISIBLE_DEVICES": ",".join(pod_gpus) if pod_gpus else "-1", "LOCAL_RANK": "0",
            "LOCAL_WORLD_SIZE": "1"}
