"""Restatement of kornia 0.6.9 kornia.filters.gaussian_blur2d (separable form):
1-D kernel g(t) = exp(-t^2 / (2 sigma^2)) / sum, t = arange(k) - k//2 (+0.5 if k
even); x-pass then y-pass, each F.pad(mode=border) + depthwise conv2d
(correlation). Written for the golden-fixture script only."""
import torch
import torch.nn.functional as F


def _gauss1d(k, sigma, dtype, device):
    x = torch.arange(k, dtype=dtype, device=device) - k // 2
    if k % 2 == 0:
        x = x + 0.5
    g = torch.exp(-x.pow(2.0) / float(2 * sigma ** 2))
    return g / g.sum()


def gaussian_blur2d(input, kernel_size, sigma, border_type="reflect", separable=True):
    ky, kx = kernel_size
    sy, sx = sigma
    b, c, h, w = input.shape
    gx = _gauss1d(kx, sx, input.dtype, input.device)
    gy = _gauss1d(ky, sy, input.dtype, input.device)
    # x pass
    t = F.pad(input, [(kx - 1) // 2, kx // 2, 0, 0], mode=border_type)
    t = F.conv2d(t, gx.view(1, 1, 1, kx).expand(c, 1, 1, kx), groups=c)
    # y pass
    t = F.pad(t, [0, 0, (ky - 1) // 2, ky // 2], mode=border_type)
    return F.conv2d(t, gy.view(1, 1, ky, 1).expand(c, 1, ky, 1), groups=c)
