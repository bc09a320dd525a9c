"""CPU restatement (PyTorch-CPU, fp32) of AA-CLIP's anomaly-map inference path.

TEST INFRASTRUCTURE — an ORACLE, like oracle/aaclip_np.py. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only
as the checker or as the timed CPU baseline (`cpu_baseline.kind = "port"`).
The product path (`aa-clip_amd/`) never imports it.

Why a second restatement: bench.py times the CPU path on the GPU box's host,
where the reference itself cannot run. The numpy oracle does its attention as
numpy batched matmuls and its GELU through scipy, which on the same host is
slower than the reference's ATen kernels (tools/cpu_calibrate.py,
profiles/r03/cpu_calibration.json). This module runs the same arithmetic on
the same ATen CPU kernels the reference calls (addmm/bmm/softmax/layer_norm/
gelu/interpolate), so its images/sec stands in for the reference's; it is
pinned to the reference's golden vectors by tests/test_oracle_golden.py.

Op order (citations /root/reference-relative):
  * visual forward   — model/adapter.py:67-112 (conv1, cls, pos, ln_pre, 24 blocks,
                       adapters on blocks 0-5, level taps, ln_post, seg/det projections)
  * residual block   — model/transformer.py:239-258 with torch MHA math
                       (in-proj, q * 1/sqrt(64), softmax over keys, out-proj)
  * similarity map   — forward_utils.py:196-216 (test branch), test.py:86-93
  * image score      — test.py:83-85
The Gaussian blur restates kornia 0.6.9's gaussian_blur2d (absent; UNPINNED, as in
the numpy oracle): reflect padding, separable 1-D kernel, x pass then y pass.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

WIDTH, HEADS, LAYERS, PATCH = 1024, 16, 24, 14


def prepare(sd: dict, img_ad: dict, levels=(6, 12, 18, 24), image_adapt_until: int = 6,
            quick_gelu: bool = False) -> dict:
    """State dicts (numpy or torch, reference key names) -> fp32 CPU tensors.
    quick_gelu: the tower's MLP activation is QuickGELU (model.py:84, transformer.py:46-49)."""
    t = lambda a: torch.as_tensor(np.asarray(a) if not isinstance(a, torch.Tensor) else a).float().contiguous()  # noqa: E731
    w = {"conv": t(sd["visual.conv1.weight"]).reshape(WIDTH, -1), "cls": t(sd["visual.class_embedding"]),
         "pos": t(sd["visual.positional_embedding"]),
         "ln_pre": (t(sd["visual.ln_pre.weight"]), t(sd["visual.ln_pre.bias"])),
         "ln_post": (t(sd["visual.ln_post.weight"]), t(sd["visual.ln_post.bias"])),
         "levels": tuple(levels), "blocks": [], "quick": bool(quick_gelu)}
    for i in range(LAYERS):
        p = f"visual.transformer.resblocks.{i}."
        w["blocks"].append({k: t(sd[p + n]) for k, n in (
            ("ln1w", "ln_1.weight"), ("ln1b", "ln_1.bias"), ("ln2w", "ln_2.weight"), ("ln2b", "ln_2.bias"),
            ("wqkv", "attn.in_proj_weight"), ("bqkv", "attn.in_proj_bias"), ("wo", "attn.out_proj.weight"),
            ("bo", "attn.out_proj.bias"), ("wfc", "mlp.c_fc.weight"), ("bfc", "mlp.c_fc.bias"),
            ("wpr", "mlp.c_proj.weight"), ("bpr", "mlp.c_proj.bias"))})
    w["adapt"] = [t(img_ad[f"layer_adapters.{i}.fc.0.weight"]) for i in range(image_adapt_until)]

    def proj(prefix):
        if prefix + ".fc.0.weight" in img_ad:
            return t(img_ad[prefix + ".fc.0.weight"]), True
        return t(img_ad[prefix + ".fc.weight"]), False
    w["seg"] = [proj(f"seg_proj.{i}") for i in range(len(levels))]
    w["det"] = proj("det_proj")
    return w


def _act(h: torch.Tensor, quick: bool) -> torch.Tensor:
    return h * torch.sigmoid(1.702 * h) if quick else F.gelu(h)


def _block(x: torch.Tensor, b: dict, quick: bool = False) -> torch.Tensor:
    """ResidualAttentionBlock (transformer.py:239-258) on token-major [B, N, D]."""
    B, N, D = x.shape
    h = F.layer_norm(x, (D,), b["ln1w"], b["ln1b"], 1e-5)
    qkv = F.linear(h, b["wqkv"], b["bqkv"]).view(B, N, 3, HEADS, D // HEADS)
    q = qkv[:, :, 0].transpose(1, 2) * (D // HEADS) ** -0.5
    k, v = qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
    a = torch.softmax(q @ k.transpose(-1, -2), dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B, N, D)
    x = x + F.linear(o, b["wo"], b["bo"])
    h = F.layer_norm(x, (D,), b["ln2w"], b["ln2b"], 1e-5)
    return x + F.linear(_act(F.linear(h, b["wfc"], b["bfc"]), quick), b["wpr"], b["bpr"])


def visual_forward(w: dict, x: torch.Tensor, image_adapt_weight: float = 0.1):
    """AdaptedCLIP.forward (adapter.py:67-112) -> (list of [B,P,768] unit rows, det [B,768])."""
    x = torch.as_tensor(x).float()
    B, C, S, _ = x.shape
    g = S // PATCH
    cols = x.reshape(B, C, g, PATCH, g, PATCH).permute(0, 2, 4, 1, 3, 5).reshape(B, g * g, C * PATCH * PATCH)
    x = cols @ w["conv"].T
    x = torch.cat([w["cls"].expand(B, 1, -1), x], 1) + w["pos"]
    x = F.layer_norm(x, (WIDTH,), *w["ln_pre"], 1e-5)
    taps = []
    for i, b in enumerate(w["blocks"][:max(w["levels"])]):
        x = _block(x, b, w["quick"])
        if i < len(w["adapt"]):  # adapter.py:92-99
            u = F.leaky_relu(x @ w["adapt"][i].T, 0.01)
            u = u * x.norm(dim=-1, keepdim=True) / u.norm(dim=-1, keepdim=True)
            x = image_adapt_weight * u + (1 - image_adapt_weight) * x
        if i + 1 in w["levels"]:
            taps.append(x[:, 1:])
    taps = [F.layer_norm(t, (WIDTH,), *w["ln_post"], 1e-5) for t in taps]
    seg = []
    for t, (wt, relu) in zip(taps, w["seg"]):
        s = t @ wt.T
        seg.append(F.normalize(F.leaky_relu(s, 0.01) if relu else s, dim=-1))
    wt, relu = w["det"]
    d = taps[-1] @ wt.T
    det = F.normalize(F.leaky_relu(d, 0.01) if relu else d, dim=-1).mean(1)
    return seg, det


def _gauss1d(k: int, sigma: float) -> torch.Tensor:
    t = torch.arange(k, dtype=torch.float32) - k // 2
    if k % 2 == 0:
        t = t + 0.5
    g = torch.exp(-(t * t) / (2.0 * sigma * sigma))
    return g / g.sum()


def gaussian_blur2d(m: torch.Tensor, k: int, sigma: float) -> torch.Tensor:
    """kornia 0.6.9 gaussian_blur2d restated: reflect pad + depthwise x pass, then y pass. m [B,C,H,W]."""
    g = _gauss1d(k, sigma)
    C = m.shape[1]
    r = k // 2
    m = F.conv2d(F.pad(m, (r, r, 0, 0), mode="reflect"), g.view(1, 1, 1, k).expand(C, 1, 1, k), groups=C)
    return F.conv2d(F.pad(m, (0, 0, r, r), mode="reflect"), g.view(1, 1, k, 1).expand(C, 1, k, 1), groups=C)


def similarity_map(f: torch.Tensor, T: torch.Tensor, img_size: int, domain: str) -> torch.Tensor:
    """calculate_similarity_map test branch (forward_utils.py:196-213) -> [B, 1, S, S]."""
    A = 100.0 * (f @ T)
    B, P, _ = A.shape
    g = int(round(P ** 0.5))
    A = A.permute(0, 2, 1).reshape(B, 2, g, g)
    m = ((A[:, 1] + 1 - A[:, 0]) / 2)[:, None]
    k, s = (7, 1.0) if domain == "Industrial" else (9, 1.5)
    return F.interpolate(gaussian_blur2d(m, k, s), size=(img_size, img_size), mode="bilinear", align_corners=True)


def anomaly_map(seg, T, img_size: int, domain: str) -> torch.Tensor:
    """test.py:86-93: per-level maps, cat, sum -> [B, S, S]."""
    return torch.cat([similarity_map(f, T, img_size, domain) for f in seg], 1).sum(1)


def image_score(det: torch.Tensor, T: torch.Tensor) -> torch.Tensor:
    """test.py:83-84."""
    return ((det @ T)[:, 1] + 1) / 2
