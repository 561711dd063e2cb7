"""PyTorchJob worker: ResNet-50 data-parallel bf16 training on MI355X.

Run by the PyTorch launcher (``kubedl_amd.controllers.pytorch``) as one
process per rank with the KubeDL rendezvous env, or directly by ``bench.py``.

Per step (all on the rank's HIP stream):
  zero flat grad (one memset) -> forward (the explicit engine of
  models/resnet_engine.py: kdl MFMA conv kernels -- 1x1 GEMMs, implicit-GEMM and
  halo 3x3, the 7x7 stem -- with BN statistics in their epilogues and fused
  BN/ReLU HIP kernels) -> fp32 cross-entropy -> backward (kdl data- and
  weight-gradient kernels, bucketed RCCL all-reduce of bf16 gradient slices
  overlapped with backward) -> one fused SGD-momentum launch (fp32 master,
  writes bf16 weights).
"""
from __future__ import annotations

import argparse
import json
import os
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# shipped MIOpen find-db / kernel cache (as bench.py): no conv-kernel recompiles per job
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_ROOT, "miopen_db", "user"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_ROOT, "miopen_db", "cache"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kubedl_amd.models.resnet import resnet50, resnet_tiny  # noqa: E402
from kubedl_amd.ops.optim import FlatParamSpace, FusedSGD
from kubedl_amd.parallel import dist as kdist
from kubedl_amd.parallel.ddp import FlatDDP
from kubedl_amd.utils.checkpoint import Checkpointer
from kubedl_amd.utils.trace import StepLog, trace_range
from kubedl_amd.utils.tune import tune
from kubedl_amd.workers import common


_LOSS_ALLREDUCE = tune("loss_allreduce", True)


class ResNetTrainer:
    def __init__(self, info: kdist.DistInfo, batch: int = 256, image: int = 224,
                 num_classes: int = 1000, dtype: torch.dtype = torch.bfloat16, lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 5e-5, tiny: bool = False,
                 bn_backend: str = "auto", bucket_cap_mb: float = 12.0, seed: int = 0,
                 conv_benchmark: bool = False, engine: str = "auto", on_streams_ready=None,
                 before_collectives=None):
        """``engine``: "fused" runs the step through ``models.resnet_engine``
        (fused 1x1-conv GEMMs + staged BN, explicit backward); "autograd" runs
        the module under autograd; "auto" = fused on the GPU when the model's
        channel counts fit the GEMM tiles (multiples of 64), else autograd.

        ``before_collectives``: called right before the trainer's first
        collective (the DDP parameter broadcast at world > 1), after the model
        is built -- a caller that bootstraps the communicator on a helper
        thread joins it here, so every rank's collectives reach RCCL in one order.

        ``on_streams_ready``: called once the step's streams (compute + the
        engine's weight-gradient side stream) exist and have run a kernel, i.e.
        before the model is built -- the bench starts the RCCL communicator's
        bootstrap there, on a helper thread, so it overlaps the weight init,
        the workspaces and the first transposes instead of following them
        (after the stream touch: RCCL's own streams must not claim the
        hardware queues first, profiles/r03_stream_touch_ab.txt)."""
        self.info = info
        dev = info.device
        if engine == "auto":
            engine = "fused" if (dev.type == "cuda" and not tiny and bn_backend != "torch") else "autograd"
        # the step runs on a non-blocking stream of its own, never the null
        # stream: with an RCCL process group present the null stream loses the
        # engine's side-stream overlap (-9 %, ops/streams.py); the caller's
        # stream waits for it after each step
        # Hardware-queue order as the measured step had it: the null stream (the
        # weight init's) first, then the weight-gradient side stream, then the
        # compute stream, all before RCCL creates its own streams
        # (profiles/r03_stream_touch_ab.txt, profiles/r05_comm_overlap_ab.jsonl)
        from kubedl_amd.ops.streams import compute_stream, side_stream
        if dev.type == "cuda":
            torch.zeros(1, device=dev).add_(1)
        side = None
        eopts = None
        if dev.type == "cuda" and engine == "fused":
            from kubedl_amd.models.resnet_engine import EngineOptions
            eopts = EngineOptions.from_env()
            side = side_stream(dev, eopts.side_prio) if eopts.side else None
        self._side = side
        if side is not None:
            with torch.cuda.stream(side):
                torch.zeros(1, device=dev).add_(1)
        self.stream = compute_stream(dev)
        if dev.type == "cuda":
            self.touch_streams()
        if on_streams_ready is not None:
            on_streams_ready(self.stream)
        if dev.type == "cuda":
            # MIOpen find (benchmark) vs immediate-mode heuristics: A/B'd in profiles/
            torch.backends.cudnn.benchmark = bool(conv_benchmark)
        torch.manual_seed(seed)
        if dev.type == "cuda":
            torch.cuda.manual_seed(seed)
        # built directly on the rank's device: the weight init runs on the GPU
        # instead of ~0.5 s of CPU RNG + a host->device copy (launch delay)
        with torch.device(dev):
            model = resnet_tiny(num_classes) if tiny else resnet50(num_classes)
        model.set_bn_backend(bn_backend)
        model = model.to(dev)
        if dev.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        with torch.no_grad():
            for p in model.parameters():
                p.data = p.data.to(dtype)
        self.model = model
        self.dtype = dtype
        self.space = FlatParamSpace(model, dtype=dtype, device=dev)
        self.engine_kind = engine
        if before_collectives is not None:
            before_collectives()
        self.ddp = FlatDDP(self.space, info.world_size, bucket_cap_mb=bucket_cap_mb,
                           direct=(engine == "fused"))
        self.engine = None
        if engine == "fused":
            from kubedl_amd.models.resnet_engine import ResNetEngine
            self.engine = ResNetEngine(model, backend="hip" if dev.type == "cuda" else "torch",
                                       grad_view=self.space.grad_view, on_ready=self.ddp.ready, options=eopts,
                                       side=side)
            self.ddp.join_stream = self.engine.side
        self.opt = FusedSGD(self.space, lr=lr, momentum=momentum, weight_decay=weight_decay)
        self.opt.grad_scale = self.ddp.grad_scale
        # synthetic batch, generated where it is used (no 77 MB host->device copy)
        g = torch.Generator(device=dev).manual_seed(seed + 1000 + info.rank)
        if dev.type == "cuda":
            x = torch.randn(batch, image, image, 3, generator=g, device=dev, dtype=dtype).permute(0, 3, 1, 2)
        else:
            x = torch.randn(batch, 3, image, image, generator=g).to(dtype)
        self.x = x
        self.y = torch.randint(0, num_classes, (batch,), generator=g, device=dev)
        self.batch = batch
        self.last_loss = None
        self._loss_work = None
        # (world 1: the caller may build the communicator after the first step;
        # until then the loss "sum" over the one rank is the loss itself)
        self.defer_collectives = False
        self._loss_sum = None
        self._loss_div = 1

    def touch_streams(self) -> None:
        """One tiny kernel on each stream the step uses (compute, weight-gradient
        side stream), so they are live before anything else -- the RCCL
        communicator's own streams -- claims the GPU's hardware queues.  Measured
        at world 1 with the communicator built before the first step: 22.04 ms
        per step untouched vs 19.28-19.44 touched (19.41 with the communicator
        built lazily inside step 1; the side stream's overlap is what is lost),
        profiles/r03_stream_touch_ab.txt."""
        for s in (self.stream, getattr(self, "_side", None)):
            if s is not None:
                with torch.cuda.stream(s):
                    torch.zeros(1, device=self.info.device).add_(1)
        torch.cuda.synchronize(self.info.device)

    def step(self) -> torch.Tensor:
        if self.stream is None:
            return self._step()
        caller = torch.cuda.current_stream(self.info.device)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            loss = self._step()
        caller.wait_stream(self.stream)
        return loss

    def _step(self) -> torch.Tensor:
        return self._finish_loss(self._step_body())

    def _step_body(self) -> torch.Tensor:
        """The step's device work: returns the loss."""
        self.space.zero_grad()
        with trace_range("forward_backward"):
            if self.engine is not None:
                loss = self.engine.forward_backward(self.x, self.y)
                self.space.mark_packed()  # gradients were written into the flat buffer
            else:
                out = self.model(self.x)
                loss = F.cross_entropy(out.float(), self.y)
                loss.backward()
        with trace_range("allreduce_wait"):
            self.ddp.finish()
        with trace_range("optimizer"):
            self.opt.step()
        return loss.detach().float().reshape(1)

    def _finish_loss(self, loss: torch.Tensor) -> torch.Tensor:
        self.last_loss = loss  # this rank's loss (returned)
        self._loss_sum = loss
        self._loss_div = 1
        if dist.is_initialized() and _LOSS_ALLREDUCE and not self.defer_collectives:
            # the step's loss summed over ranks (reporting); at world 1 this is
            # the collective that keeps the RCCL path exercised in every step
            self._loss_sum = loss.clone()
            self._loss_div = dist.get_world_size()
            self._loss_work = dist.all_reduce(self._loss_sum, async_op=True)
        return loss

    def loss(self) -> torch.Tensor:
        """The last step's loss averaged over ranks (waits for its all-reduce);
        without the all-reduce (no process group, or KDL_TUNE loss_allreduce=0) this
        rank's own loss -- divided only when the sum actually ran."""
        if self._loss_work is not None:
            self._loss_work.wait()
            self._loss_work = None
        return self._loss_sum / self._loss_div if self._loss_div > 1 else self._loss_sum

    def check_transport(self) -> None:
        """Raise if a P2P all-reduce of any step so far timed out.  Call after
        a device synchronisation: the kernels report through host-mapped
        memory, so before a sync the bits of in-flight steps are not there yet."""
        if self.ddp.transport is not None:
            self.ddp.transport.check()

    # ------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        """Everything a restarted rank needs to continue bit-exactly: bf16 params,
        fp32 master weights, momentum, step count, BN running statistics."""
        st = {"param": self.space.param, "master": self.space.master, "momentum": self.opt.mom,
              "opt_steps": int(self.opt.step_count)}
        for name, buf in self.model.named_buffers():
            st["buf." + name] = buf
        return st

    @torch.no_grad()
    def load_state_dict(self, st: dict) -> None:
        self.space.param.copy_(st["param"])
        self.space.master.copy_(st["master"])
        self.opt.mom.copy_(st["momentum"])
        self.opt.step_count = int(st["opt_steps"])
        for name, buf in self.model.named_buffers():
            buf.copy_(st["buf." + name])


def sync(info: kdist.DistInfo) -> None:
    if info.device.type == "cuda":
        torch.cuda.synchronize(info.device)


def run(args) -> dict:
    t_start = time.time()
    info = kdist.init_from_env("cpu" if args.cpu else None, world1_group=True)
    common.signal_ready({"rank": info.rank})
    tr = ResNetTrainer(info, batch=args.batch, image=args.image, tiny=args.tiny,
                       bn_backend=args.bn_backend, engine=args.engine)
    ckpt = Checkpointer.from_env(info.rank)
    steplog = StepLog(rank=info.rank)
    done = 0  # optimizer steps completed by this job (across restarts)
    resumed = ckpt.load_latest(map_location=info.device)
    if resumed is not None:
        done, st = resumed
        tr.load_state_dict(st)
    total = args.warmup + args.steps

    def one(i):
        t = time.perf_counter()
        tr.step()
        if steplog.enabled:
            sync(info)
            steplog.write(i + 1, (time.perf_counter() - t) * 1e3, loss=float(tr.loss().item()))
        if ckpt.due(i + 1):
            sync(info)
            tr.check_transport()  # never persist weights of a timed-out all-reduce
            ckpt.save(i + 1, tr.state_dict())
            kdist.barrier(info)  # peers wait for the save instead of racing ahead into timeouts
        common.maybe_inject_fault(info.rank, i)

    for i in range(done, args.warmup):
        one(i)
    sync(info)
    kdist.barrier(info)
    sync(info)
    t0 = time.perf_counter()
    timed = range(max(done, args.warmup), total)
    for i in timed:
        one(i)
    sync(info)
    kdist.barrier(info)
    sync(info)
    dt = time.perf_counter() - t0
    tr.check_transport()
    dt = kdist.all_reduce_max(dt, info)
    nsteps = len(timed)
    loss = float(tr.loss().item()) if tr.last_loss is not None else float("nan")
    res = {
        "rank": info.rank, "world_size": info.world_size, "steps": nsteps,
        "seconds": dt, "ms_per_step": dt / max(nsteps, 1) * 1e3,
        "steps_per_sec": nsteps / dt if dt > 0 else 0.0,
        "images_per_sec": nsteps * args.batch * info.world_size / dt if dt > 0 else 0.0,
        "loss": loss, "startup_s": t0 - t_start, "resumed_from_step": done if resumed is not None else None,
        "total_steps": total,
    }
    steplog.close()
    common.report_progress(total, res["steps_per_sec"], final=True, loss=loss)
    kdist.shutdown(info)
    return res


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="ResNet-50 DP bf16 trainer (PyTorchJob worker)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--tiny", action="store_true", help="tiny ResNet (tests)")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--bn-backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "autograd"])
    return ap


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    res = run(args)
    if res["rank"] == 0:
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(kdist.run_rank(main))
