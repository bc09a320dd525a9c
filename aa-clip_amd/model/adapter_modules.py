"""SimpleAdapter / SimpleProj — same constructor, attributes and state-dict
keys as the reference (model/adapter_modules.py:6-26): `fc` is an
nn.Sequential(Linear(no bias), LeakyReLU) (keys `fc.0.weight`), or a bare
Linear for SimpleProj(relu=False) (key `fc.weight`).

The modules hold the weights; their forward runs the HIP GEMM with the
LeakyReLU fused in the epilogue (device tensors only — no CPU path)."""
from __future__ import annotations

import torch
from torch import nn

from aaclip import ops


def _linear_leaky(x: torch.Tensor, weight: torch.Tensor, leaky: bool) -> torch.Tensor:
    shape = x.shape
    x2 = x.reshape(-1, shape[-1]).to(torch.float32).contiguous()
    out = torch.empty(x2.shape[0], weight.shape[0], device=x.device, dtype=torch.float32)
    ops.gemm(x2, weight.detach().to(torch.float32).contiguous(), out, leaky=leaky)
    return out.reshape(*shape[:-1], weight.shape[0])


class SimpleAdapter(nn.Module):
    def __init__(self, c_in, c_out=768):
        super().__init__()
        self.fc = nn.Sequential(nn.Linear(c_in, c_out, bias=False), nn.LeakyReLU())

    def forward(self, x):
        return _linear_leaky(x, self.fc[0].weight, True)


class SimpleProj(nn.Module):
    def __init__(self, c_in, c_out=768, relu=True):
        super().__init__()
        self.relu = relu
        if relu:
            self.fc = nn.Sequential(nn.Linear(c_in, c_out, bias=False), nn.LeakyReLU())
        else:
            self.fc = nn.Linear(c_in, c_out, bias=False)

    @property
    def weight(self):
        return self.fc[0].weight if self.relu else self.fc.weight

    def forward(self, x):
        return _linear_leaky(x, self.weight, self.relu)
