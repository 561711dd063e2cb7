"""All-or-nothing GPU allocator for one MI355X node (8 GPUs x 288 GB HBM3E).

Replaces kube-batch's PodGroup admission (``pkg/gang_schedule/batch_scheduler``):
a gang (all pods of a job, ``minMember = sum(replicas)``) is placed only when
EVERY member fits; otherwise nothing is reserved and the job stays
``Created`` (pending).

Placement policy (MI355X-first):

* GPUs are exclusive (``amd.com/gpu: N`` per container); pods asking for no
  GPU (TF PS, XDL Scheduler, CPU ranks) always fit.
* Each GPU is one xGMI peer of every other (fully connected, 7 links each),
  so any set is bandwidth-equivalent for RCCL rings; what still matters is
  host locality: GPUs 0-3 and 4-7 hang off different CPU sockets/NUMA
  nodes on an 8-GPU MI355X platform.  A gang that fits inside one half is
  kept there, choosing the half with the FEWEST free GPUs that still fits
  (best fit -> two 4-GPU jobs land on opposite halves, leaving whole halves
  free for later 4-GPU jobs).
* HBM: each GPU advertises 288 GB.  A pod asking for whole GPUs
  (``amd.com/gpu: N``) owns them; ``kubedl.io/hbm-gb`` on such a pod is its
  per-process cap and must fit one GPU.  A pod asking for ``kubedl.io/hbm-gb:
  X`` and NO whole GPU gets an HBM *slice*: it shares a GPU with other slices
  as long as their sum stays <= 288 GB (best fit: the fullest shared GPU that
  still has X GB left, a fresh GPU only when none has -- so whole GPUs stay
  available for exclusive gangs).  Exclusive and shared use never mix on one
  GPU.  The kubelet exports the slice as ``KDL_HBM_LIMIT_GB`` and the rank
  caps its caching allocator to it (``parallel.dist.apply_hbm_limit``), which
  is what makes the accounting real: many small jobs (CTR towers, GBDT, tests)
  pack onto one 288 GB device instead of idling seven eighths of it.

The inventory is discovered from the KFD topology (no GPU initialisation,
so the controller never touches the device), or forced with
``KDL_FAKE_GPUS=N`` for CPU tests.
"""
from __future__ import annotations

import glob
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

MI355X_HBM_GB = 288


@dataclass
class GPUInventory:
    count: int
    hbm_gb: float = MI355X_HBM_GB
    numa_groups: List[List[int]] = field(default_factory=list)

    def __post_init__(self):
        if not self.numa_groups:
            if self.count >= 8 and self.count % 2 == 0:
                h = self.count // 2
                self.numa_groups = [list(range(h)), list(range(h, self.count))]
            else:
                self.numa_groups = [list(range(self.count))]


def detect_gpus() -> GPUInventory:
    fake = os.environ.get("KDL_FAKE_GPUS")
    if fake not in (None, ""):
        return GPUInventory(int(fake))
    n = 0
    hbm = MI355X_HBM_GB
    for props in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            kv = dict(line.split() for line in open(props) if len(line.split()) == 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) > 0 and int(kv.get("gfx_target_version", "0")) > 0:
            n += 1
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        n = min(n, len([v for v in vis.split(",") if v.strip() != ""])) if n else len(vis.split(","))
    return GPUInventory(n, hbm)


def _native():
    from kubedl_amd.runtime import native
    return native.load()


@dataclass
class Allocation:
    owner: str
    pods: Dict[str, List[int]]  # pod key -> gpu ids
    slices: Dict[str, float] = field(default_factory=dict)  # pod key -> HBM GB of a shared-GPU slice

    @property
    def gpus(self) -> List[int]:
        """GPUs owned exclusively."""
        return sorted(g for k, v in self.pods.items() if k not in self.slices for g in v)


class GPUAllocator:
    def __init__(self, inventory: Optional[GPUInventory] = None):
        self.inv = inventory or detect_gpus()
        self._lock = threading.Lock()
        self._owner_of: Dict[int, str] = {}
        self._allocs: Dict[str, Allocation] = {}
        self._shared: Dict[int, Dict[tuple, float]] = {}  # gpu -> {(owner, pod key): GB} of HBM slices

    def _is_free(self, g: int) -> bool:
        return g not in self._owner_of and not self._shared.get(g)

    @property
    def free(self) -> List[int]:
        """GPUs with neither an owner nor a slice."""
        with self._lock:
            return [g for g in range(self.inv.count) if self._is_free(g)]

    def hbm_free(self) -> Dict[int, float]:
        """Unreserved HBM GB per GPU (0 on exclusively owned GPUs)."""
        with self._lock:
            return {g: (0.0 if g in self._owner_of else self.inv.hbm_gb - sum(self._shared.get(g, {}).values()))
                    for g in range(self.inv.count)}

    def hbm_used(self) -> float:
        with self._lock:
            return (len(self._owner_of) * self.inv.hbm_gb
                    + sum(v for d in self._shared.values() for v in d.values()))

    def allocation(self, owner: str) -> Optional[Allocation]:
        with self._lock:
            return self._allocs.get(owner)

    def allocate(self, owner: str, requests: Dict[str, int],
                 hbm_gb: Optional[Dict[str, float]] = None) -> Optional[Allocation]:
        """Place every pod of ``requests`` (pod key -> #GPUs) or nothing.

        Idempotent per owner: pods already placed keep their GPUs; only the
        missing ones are placed, still all-or-nothing across the missing set.
        """
        hbm_gb = hbm_gb or {}
        with self._lock:
            cur = self._allocs.get(owner)
            placed = dict(cur.pods) if cur else {}
            slices = dict(cur.slices) if cur else {}
            todo = {k: n for k, n in requests.items() if k not in placed}
            for k, n in todo.items():
                if n < 0:
                    raise ValueError("negative GPU request")
                need = float(hbm_gb.get(k, 0.0) or 0.0)
                if need < 0:
                    raise ValueError("negative HBM request")
                if need > self.inv.hbm_gb:
                    return None  # can never fit on this node
            whole = {k: n for k, n in todo.items() if n > 0}
            sliced = {k: float(hbm_gb[k]) for k, n in todo.items() if n == 0 and float(hbm_gb.get(k, 0) or 0) > 0}
            need_total = sum(whole.values())
            free = [g for g in range(self.inv.count) if self._is_free(g)]
            if need_total > len(free):
                return None
            chosen = self._choose(free, need_total)
            if chosen is None:
                return None
            # slices go on GPUs not taken by this gang's whole-GPU members
            slice_gpu = self._place_slices(sliced, set(chosen))
            if slice_gpu is None:
                return None
            it = iter(chosen)
            for k, n in sorted(whole.items()):
                placed[k] = [next(it) for _ in range(n)]
            for k in todo:
                if k not in placed:
                    placed[k] = [slice_gpu[k]] if k in slice_gpu else []
            for k, g in slice_gpu.items():
                slices[k] = sliced[k]
                self._shared.setdefault(g, {})[(owner, k)] = sliced[k]
            alloc = Allocation(owner, placed, slices)
            self._allocs[owner] = alloc
            for g in alloc.gpus:
                self._owner_of[g] = owner
            return alloc

    def _place_slices(self, sliced: Dict[str, float], taken: set) -> Optional[Dict[str, int]]:
        """Best-fit packing of HBM slices (largest first) onto shared or free
        GPUs; all-or-nothing (nothing is recorded here)."""
        room = {g: self.inv.hbm_gb - sum(self._shared.get(g, {}).values())
                for g in range(self.inv.count) if g not in self._owner_of and g not in taken}
        shared_now = {g for g, d in self._shared.items() if d}
        out: Dict[str, int] = {}
        for k, gb in sorted(sliced.items(), key=lambda kv: (-kv[1], kv[0])):
            cands = [g for g, r in room.items() if r + 1e-9 >= gb]
            if not cands:
                return None
            # a GPU that already carries slices first (the fullest that fits), a fresh one last
            used = shared_now | set(out.values())
            g = min(cands, key=lambda g: (g not in used, room[g], g))
            room[g] -= gb
            out[k] = g
        return out

    def _choose(self, free: Sequence[int], n: int) -> Optional[List[int]]:
        if n == 0:
            return []
        nat = _native()
        if nat is not None and self.inv.count <= 64:
            free_mask = 0
            for g in free:
                free_mask |= 1 << g
            groups = [sum(1 << g for g in grp) for grp in self.inv.numa_groups]
            m = nat.best_fit(free_mask, n, groups)
            if m < 0:
                return None
            return [g for g in range(64) if m >> g & 1]
        fits = []
        for grp in self.inv.numa_groups:
            avail = [g for g in grp if g in free]
            if len(avail) >= n:
                fits.append((len(avail), grp[0], avail))
        if fits:
            fits.sort()
            return fits[0][2][:n]
        return sorted(free)[:n] if len(free) >= n else None

    def release(self, owner: str, pod_key: Optional[str] = None) -> List[int]:
        with self._lock:
            alloc = self._allocs.get(owner)
            if alloc is None:
                return []
            keys = [pod_key] if pod_key is not None else list(alloc.pods)
            freed = []
            for k in keys:
                gpus = alloc.pods.pop(k, [])
                if alloc.slices.pop(k, None) is not None:
                    for g in gpus:
                        d = self._shared.get(g, {})
                        d.pop((owner, k), None)
                        if not d:
                            self._shared.pop(g, None)
                            freed.append(g)
                    continue
                for g in gpus:
                    self._owner_of.pop(g, None)
                    freed.append(g)
            if not alloc.pods:
                self._allocs.pop(owner, None)
            return freed

    def used(self) -> int:
        """GPUs in use (owned, or carrying at least one slice)."""
        with self._lock:
            return len(self._owner_of) + sum(1 for g, d in self._shared.items() if d)

    def snapshot(self) -> Dict[str, Dict[str, List[int]]]:
        with self._lock:
            return {o: {k: list(v) for k, v in a.pods.items()} for o, a in self._allocs.items()}
