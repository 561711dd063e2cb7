"""Worker-side checkpoint / resume (SURVEY.md §5 "Checkpoint / resume").

The reference has none (KubeDL restarts a failed pod from scratch).  Here a rank
process that is restarted under the ``ExitCode`` / ``OnFailure`` policies picks
up where the job left off:

- ``KDL_CKPT_DIR``   directory shared by the job's ranks (set by the job spec;
                     the local runtime keeps it across restarts);
- ``KDL_CKPT_EVERY`` save period in optimizer steps (default 0 = off).

Data-parallel replicas hold identical state, so rank 0 writes
``step-<n>.pt`` (tmp file + ``os.replace``: a crash never leaves a torn file)
and updates ``latest.json``; every rank loads the newest complete file with
``torch.load(weights_only=True)`` (tensors, numbers and strings only: nothing in
a checkpoint file is executed).  ``keep`` old files are retained.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional, Tuple

import torch


class Checkpointer:
    def __init__(self, directory: Optional[str], rank: int = 0, every: int = 0, keep: int = 2,
                 writer_rank: int = 0):
        self.dir = directory
        self.rank = rank
        self.every = int(every)
        self.keep = max(int(keep), 1)
        self.writer = rank == writer_rank
        if self.dir and self.writer:
            os.makedirs(self.dir, exist_ok=True)

    @classmethod
    def from_env(cls, rank: int) -> "Checkpointer":
        return cls(os.environ.get("KDL_CKPT_DIR") or None, rank, int(os.environ.get("KDL_CKPT_EVERY", "0") or 0))

    @property
    def enabled(self) -> bool:
        return bool(self.dir)

    def _path(self, step: int) -> str:
        return os.path.join(self.dir, f"step-{step:08d}.pt")

    def due(self, step: int) -> bool:
        """``step`` = number of completed optimizer steps."""
        return self.enabled and self.every > 0 and step > 0 and step % self.every == 0

    def save(self, step: int, state: Dict[str, Any]) -> Optional[str]:
        if not (self.enabled and self.writer):
            return None
        path = self._path(step)
        tmp = path + f".tmp{os.getpid()}"
        cpu = {k: (v.detach().to("cpu") if torch.is_tensor(v) else v) for k, v in state.items()}
        cpu["__step__"] = int(step)
        torch.save(cpu, tmp)
        os.replace(tmp, path)
        latest = os.path.join(self.dir, "latest.json")
        with open(latest + ".tmp", "w") as f:
            json.dump({"step": int(step), "file": os.path.basename(path)}, f)
        os.replace(latest + ".tmp", latest)
        self._prune()
        return path

    def _prune(self) -> None:
        files = sorted(f for f in os.listdir(self.dir) if f.startswith("step-") and f.endswith(".pt"))
        for f in files[:-self.keep]:
            try:
                os.remove(os.path.join(self.dir, f))
            except FileNotFoundError:
                pass

    def load_latest(self, map_location=None) -> Optional[Tuple[int, Dict[str, Any]]]:
        if not self.enabled or not os.path.isdir(self.dir):
            return None
        files = sorted(f for f in os.listdir(self.dir) if f.startswith("step-") and f.endswith(".pt"))
        for f in reversed(files):  # newest first; a file is only ever visible complete
            try:
                state = torch.load(os.path.join(self.dir, f), map_location=map_location, weights_only=True)
            except Exception:  # torn / foreign file: the unpickler's errors vary; fall back to older
                continue
            return int(state.pop("__step__")), state
        return None
