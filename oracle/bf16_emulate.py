"""ORACLE (test infrastructure only): a bf16-storage emulation of the
torchvision restatement, used to DERIVE the tolerances of the bf16 GPU path.

The HIP engine keeps every activation and activation gradient in bf16 while
accumulating in fp32 (include/ssip.h conventions): each conv reads bf16
inputs and bf16 weights and stores a bf16 output; in the backward the
gradient reaching a conv's output and the data gradient it produces are
bf16 too.  ``emulate_bf16(model)`` applies exactly those roundings around
every nn.Conv2d of a (float64) torchvision model, so comparing the emulated
run with the plain float64 run gives the error a correct bf16 kernel set
is expected to show; a GPU test then bounds the HIP path's error by a small
multiple of it (tests/test_gpu_semi_step.py, tests/test_gpu_resnet.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _RoundBF16(torch.autograd.Function):
    """Round to bf16 (kept in the input dtype) forward AND backward."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def round_bf16(x: torch.Tensor) -> torch.Tensor:
    return _RoundBF16.apply(x)


def _conv_forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    w = self.weight.detach().to(torch.bfloat16).to(self.weight.dtype) + (self.weight - self.weight.detach())
    y = F.conv2d(round_bf16(x), w, self.bias, self.stride, self.padding, self.dilation, self.groups)
    return round_bf16(y)


def emulate_bf16(model: nn.Module) -> nn.Module:
    """Patch every Conv2d of ``model`` in place (instance-level forward)."""
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            m.forward = _conv_forward.__get__(m, nn.Conv2d)
    return model
