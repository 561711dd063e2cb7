"""Fused BatchNorm (+residual add) (+ReLU) for NHWC activations.

Two backends:

* ``torch`` -- eager composition ``relu(batch_norm(x) + residual)``; this is
  the fp32 numerics reference used by the tests and the CPU path.
* ``hip``   -- the hand-written CDNA4 kernels in ``csrc/bn_act.hip``:
  forward = per-channel Welford/Chan partial reduction (16-byte bf16 vector
  loads along C) + one fused normalise/add/ReLU pass; backward = one
  reduction pass producing (dgamma, dbeta) and one elementwise pass producing
  dx (and d(residual)), reading the saved bf16 output for the ReLU mask so no
  extra activation is kept alive.

``auto`` picks ``hip`` when the tensor lives on the GPU and the extension is
built; on a GPU box a missing extension is an error (never a silent fallback:
see ``kubedl_amd.ops._ext``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from kubedl_amd.ops import _ext


def _torch_bn_act(x, weight, bias, running_mean, running_var, residual, relu,
                  training, momentum, eps):
    if x.is_cuda:
        # what an eager PyTorch/AMP trainer does on GPU: mixed bf16-in / fp32-param BN
        # (MIOpen), then separate add and ReLU kernels -- the A/B baseline for the HIP path
        y = F.batch_norm(x, running_mean, running_var, weight.float(), bias.float(),
                         training=training, momentum=momentum, eps=eps)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
    # computed in fp32 (running stats are fp32); result cast back to x's dtype
    y = F.batch_norm(x.float(), running_mean, running_var, weight.float(), bias.float(),
                     training=training, momentum=momentum, eps=eps)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = F.relu(y)
    return y.to(x.dtype)


def workspace_for(channels: int, device) -> torch.Tensor:
    """Per-layer zeroed fp32 workspace (replicated stat accumulators + coefs).

    The kernels leave it zeroed after every use, so a layer allocates it once
    and keeps it (no per-call memset)."""
    n = _ext.load().bn_workspace_floats(int(channels))
    return torch.zeros(n, dtype=torch.float32, device=device)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, relu, training,
                momentum, eps, ws):
        ext = _ext.load()
        x = x.contiguous(memory_format=torch.channels_last) if x.dim() == 4 else x.contiguous()
        if residual is not None:
            residual = residual.contiguous(memory_format=torch.channels_last) if residual.dim() == 4 \
                else residual.contiguous()
        y, mean, invstd, mbits = ext.bn_act_fwd(x, weight, bias, running_mean, running_var,
                                                residual, bool(relu), bool(training),
                                                float(momentum), float(eps), ws, True)
        # relu+residual layers: keep the packed 1-bit ReLU mask, not y, for the backward
        ctx.save_for_backward(x, y if mbits is None else None, weight, bias, mean, invstd, mbits)
        ctx.ws = ws
        ctx.relu = relu
        ctx.has_residual = residual is not None
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load()
        x, y, weight, bias, mean, invstd, mbits = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
        dx, dgamma, dbeta, dres = ext.bn_act_bwd(dy, x, y, weight, bias, mean, invstd,
                                                 bool(ctx.relu), bool(ctx.has_residual),
                                                 bool(ctx.training), ctx.ws, mbits)
        return dx, dgamma, dbeta, None, None, (dres if ctx.has_residual else None), \
            None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean, running_var, residual=None, relu=True,
                   training=True, momentum=0.1, eps=1e-5, backend="auto", workspace=None):
    if backend == "auto":
        backend = "hip" if (x.is_cuda and _ext.available()) else "torch"
        if x.is_cuda and backend == "torch":
            _ext.require_on_gpu("batch_norm_act")
    if backend == "torch" or x.dtype == torch.float64:
        return _torch_bn_act(x, weight, bias, running_mean, running_var, residual, relu,
                             training, momentum, eps)
    return _BNActFn.apply(x, weight, bias, running_mean, running_var, residual, relu,
                          training, momentum, eps, workspace)


class _BNPoolFn(torch.autograd.Function):
    """Stem BN + ReLU + max-pool(3, 2, 1): the full-resolution BN output is
    never materialised (``bn_pool_forward`` / ``bn_pool_backward``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, ws):
        ext = _ext.load()
        x = x.contiguous(memory_format=torch.channels_last)
        y, mean, invstd, idx, _ = ext.bn_pool_fwd(x, weight, bias, running_mean, running_var, bool(training),
                                                  float(momentum), float(eps), ws, False, False)
        ctx.save_for_backward(x, idx, weight, bias, mean, invstd)
        ctx.ws = ws
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load()
        x, idx, weight, bias, mean, invstd = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx, dgamma, dbeta = ext.bn_pool_bwd(dy, idx, x, weight, bias, mean, invstd, bool(ctx.training), ctx.ws,
                                            True)
        return dx, dgamma, dbeta, None, None, None, None, None, None


def batch_norm_relu_maxpool(x, weight, bias, running_mean, running_var, training=True, momentum=0.1,
                            eps=1e-5, backend="auto", workspace=None):
    """maxpool3x3s2p1(relu(batch_norm(x))) -- one fused op on the HIP backend."""
    if backend == "auto":
        backend = "hip" if (x.is_cuda and _ext.available()) else "torch"
        if x.is_cuda and backend == "torch":
            _ext.require_on_gpu("batch_norm_relu_maxpool")
    if backend == "torch" or x.dtype != torch.bfloat16 or x.dim() != 4 or x.shape[1] % 8:
        y = _torch_bn_act(x, weight, bias, running_mean, running_var, None, True, training, momentum, eps)
        return F.max_pool2d(y, 3, 2, 1)
    return _BNPoolFn.apply(x, weight, bias, running_mean, running_var, training, momentum, eps, workspace)
