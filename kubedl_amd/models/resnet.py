"""ResNet-50 (v1.5) written for MI355X training: NHWC (channels_last) bf16.

This is the flagship workload that a ``PyTorchJob`` launches (BASELINE.json
config "PyTorchJob ResNet-50 DDP bf16").  The reference (KubeDL) contains no
model code at all -- it only launches user images (SURVEY.md §0.2,
``example/pytorch/pytorch_job_mnist_mpi.yaml:14``) -- so the architecture here
follows the canonical ResNet-50 v1.5 definition (stride on the 3x3 conv of each
bottleneck, 25,557,032 parameters).

MI355X-first design choices:

* activations are kept NHWC bf16 end to end so MIOpen/hipBLASLt pick their
  NHWC implicit-GEMM (MFMA) solvers and the elementwise work is contiguous
  along C (16-byte vector loads along the channel axis in our HIP kernels);
* every BatchNorm is fused with its consumer elementwise op (ReLU, or the
  residual add + ReLU at the end of a bottleneck) by ``kubedl_amd.ops.bn``:
  one stats pass + one apply pass forward, one reduce pass + one apply pass
  backward, instead of the 3-5 separate passes eager PyTorch issues;
* the model owns no optimizer state; the fused multi-tensor optimizer in
  ``kubedl_amd.ops.optim`` keeps fp32 master weights next to the bf16 params.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from kubedl_amd.ops import bn as bn_ops


class BNAct(nn.Module):
    """BatchNorm2d (+ optional residual add) (+ optional ReLU), NHWC.

    Parameters/buffers are fp32 (weight, bias, running_mean, running_var);
    activations may be bf16.  ``backend`` selects the fused HIP kernels
    ("hip") or the eager PyTorch composition ("torch"), which is also the
    numerics reference in the tests.
    """

    def __init__(self, channels: int, relu: bool = True, zero_init: bool = False,
                 eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.channels = channels
        self.relu = relu
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.zeros(channels) if zero_init else torch.ones(channels))
        self.bias = nn.Parameter(torch.zeros(channels))
        self.register_buffer("running_mean", torch.zeros(channels))
        self.register_buffer("running_var", torch.ones(channels))
        self.backend = "auto"
        self._ws = None

    def forward(self, x: torch.Tensor, residual: torch.Tensor | None = None) -> torch.Tensor:
        ws = None
        if x.is_cuda and self.backend != "torch":
            if self._ws is None or self._ws.device != x.device:
                self._ws = bn_ops.workspace_for(self.channels, x.device)
            ws = self._ws
        return bn_ops.batch_norm_act(
            x, self.weight, self.bias, self.running_mean, self.running_var,
            residual=residual, relu=self.relu, training=self.training,
            momentum=self.momentum, eps=self.eps, backend=self.backend, workspace=ws)

    def forward_maxpool(self, x: torch.Tensor) -> torch.Tensor:
        """maxpool(3, 2, 1)(self(x)) for the stem, fused on the HIP backend."""
        ws = None
        if x.is_cuda and self.backend != "torch":
            if self._ws is None or self._ws.device != x.device:
                self._ws = bn_ops.workspace_for(self.channels, x.device)
            ws = self._ws
        return bn_ops.batch_norm_relu_maxpool(
            x, self.weight, self.bias, self.running_mean, self.running_var, training=self.training,
            momentum=self.momentum, eps=self.eps, backend=self.backend, workspace=ws)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_ch: int, width: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        out_ch = width * self.expansion
        self.conv1 = nn.Conv2d(in_ch, width, 1, bias=False)
        self.bn1 = BNAct(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BNAct(width)
        self.conv3 = nn.Conv2d(width, out_ch, 1, bias=False)
        # zero-init of the last BN gamma (Goyal et al.) keeps early training stable
        self.bn3 = BNAct(out_ch, relu=True, zero_init=True)
        if downsample:
            self.down_conv = nn.Conv2d(in_ch, out_ch, 1, stride=stride, bias=False)
            self.down_bn = BNAct(out_ch, relu=False)
        else:
            self.down_conv = None
            self.down_bn = None

    def forward(self, x):
        identity = x
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        out = self.conv3(out)
        if self.down_conv is not None:
            identity = self.down_bn(self.down_conv(x))
        # bn3 + residual add + relu in one fused pass
        return self.bn3(out, residual=identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = BNAct(width)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        blocks = []
        in_ch = width
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            stride = 1 if i == 0 else 2
            for j in range(n):
                blocks.append(Bottleneck(in_ch, w, stride if j == 0 else 1, downsample=(j == 0)))
                in_ch = w * Bottleneck.expansion
        self.layers = nn.Sequential(*blocks)
        self.fc = nn.Linear(in_ch, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = self.bn1.forward_maxpool(self.conv1(x))  # == self.maxpool(self.bn1(conv1(x)))
        x = self.layers(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)

    def set_bn_backend(self, backend: str) -> None:
        for m in self.modules():
            if isinstance(m, BNAct):
                m.backend = backend



def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes=num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Small ResNet used by CPU tests and the smoke path (same code path)."""
    return ResNet((1, 1, 1, 1), num_classes=num_classes, width=8)


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
