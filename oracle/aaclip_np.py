"""CPU restatement (numpy, fp32) of AA-CLIP's anomaly-map inference path.

TEST INFRASTRUCTURE — this is the ORACLE. Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import it, and only as the checker (or as
the timed CPU baseline, `cpu_baseline.kind = "port"`). The product path
(`aa-clip_amd/`) never imports it.

Pinned against the real reference: tests/golden/make_golden.py imports the
reference from /root/reference (with import-only stubs) in the build
container, drives it with oracle/synth.py weights, and commits the outputs as
tests/golden/*.npz; tests/test_oracle_golden.py checks this module against
them. Exception: the Gaussian blur comes from kornia==0.6.9 (absent, not
vendored) and is restated from its published algorithm — parity at that
boundary is UNPINNED by any reference test.

Op order follows the reference line by line (citations are
/root/reference-relative):
  * visual forward   — model/adapter.py:67-112
  * residual block   — model/transformer.py:239-258 (+ torch MHA, need_weights)
  * text encoding    — model/adapter.py:114-145, model/model.py:190-201
  * text anchors     — forward_utils.py:138-162, :185-192
  * similarity map   — forward_utils.py:196-216
  * image score      — test.py:83-85
  * metrics          — forward_utils.py:233-280
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf as _erf

F32 = np.float32


# --------------------------------------------------------------------------- primitives
def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    """F.layer_norm over the last dim, biased variance (transformer.py:37-43)."""
    x = x.astype(F32, copy=False)
    mu = x.mean(-1, keepdims=True, dtype=F32)
    d = x - mu
    var = (d * d).mean(-1, keepdims=True, dtype=F32)
    return (d / np.sqrt(var + F32(eps)) * w + b).astype(F32)


def gelu_erf(x: np.ndarray) -> np.ndarray:
    """nn.GELU() exact erf form (model.py:84, quick_gelu False)."""
    return (F32(0.5) * x * (F32(1.0) + _erf(x * F32(1.0 / np.sqrt(2.0))).astype(F32))).astype(F32)


def quick_gelu(x: np.ndarray) -> np.ndarray:
    """QuickGELU x * sigmoid(1.702 x) (transformer.py:46-49; towers built with quick_gelu=True,
    model.py:84,129)."""
    x = x.astype(F32, copy=False)
    return (x * (F32(1.0) / (F32(1.0) + np.exp(F32(-1.702) * x)))).astype(F32)


def leaky_relu(x: np.ndarray, slope: float = 0.01) -> np.ndarray:
    """nn.LeakyReLU() default slope 0.01 (adapter_modules.py:9,20)."""
    return np.where(x >= 0, x, x * F32(slope)).astype(F32)


def l2_normalize(x: np.ndarray, eps: float = 1e-12) -> np.ndarray:
    """F.normalize(dim=-1): x / max(||x||, eps)."""
    n = np.sqrt((x.astype(F32) ** 2).sum(-1, keepdims=True, dtype=F32))
    return (x / np.maximum(n, F32(eps))).astype(F32)


def linear(x: np.ndarray, w: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    y = x @ w.T
    if b is not None:
        y = y + b
    return y.astype(F32, copy=False)


def softmax(x: np.ndarray, axis: int = -1) -> np.ndarray:
    m = x.max(axis, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis, keepdims=True)).astype(F32)


# --------------------------------------------------------------------------- transformer
def attention(h: np.ndarray, p: dict, prefix: str, heads: int, causal: bool) -> np.ndarray:
    """nn.MultiheadAttention(q=k=v=h) in its need_weights=True form
    (transformer.py:200, torch F.multi_head_attention_forward): packed in-proj
    [q|k|v], q scaled by 1/sqrt(head_dim), softmax over keys, out-proj.
    h: [B, N, D] (NLD; the reference's LND is a layout detail)."""
    B, N, D = h.shape
    hd = D // heads
    qkv = linear(h, p[prefix + ".in_proj_weight"], p[prefix + ".in_proj_bias"])  # [B,N,3D]
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    q = q.reshape(B, N, heads, hd).transpose(0, 2, 1, 3) * F32(hd ** -0.5)
    k = k.reshape(B, N, heads, hd).transpose(0, 2, 1, 3)
    v = v.reshape(B, N, heads, hd).transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2)  # [B,H,N,N]
    if causal:
        s = s + np.triu(np.full((N, N), -np.inf, F32), 1)  # transformer.py:629-635
    a = softmax(s, -1)
    o = (a @ v).transpose(0, 2, 1, 3).reshape(B, N, D)
    return linear(o, p[prefix + ".out_proj.weight"], p[prefix + ".out_proj.bias"])


def resblock(x: np.ndarray, p: dict, prefix: str, heads: int, causal: bool = False,
             quick: bool = False) -> np.ndarray:
    """ResidualAttentionBlock.forward (transformer.py:239-258); quick: QuickGELU MLP."""
    h = layer_norm(x, p[prefix + ".ln_1.weight"], p[prefix + ".ln_1.bias"])
    x = x + attention(h, p, prefix + ".attn", heads, causal)
    h = layer_norm(x, p[prefix + ".ln_2.weight"], p[prefix + ".ln_2.bias"])
    h = (quick_gelu if quick else gelu_erf)(linear(h, p[prefix + ".mlp.c_fc.weight"], p[prefix + ".mlp.c_fc.bias"]))
    x = x + linear(h, p[prefix + ".mlp.c_proj.weight"], p[prefix + ".mlp.c_proj.bias"])
    return x.astype(F32)


def adapter_blend(x: np.ndarray, w: np.ndarray, weight: float) -> np.ndarray:
    """Residual adapter (adapter.py:92-99 / :129-136): u = LeakyReLU(x W^T);
    u = u * ||x|| / ||u||; x = w*u + (1-w)*x."""
    u = leaky_relu(linear(x, w))
    xn = np.sqrt((x * x).sum(-1, keepdims=True, dtype=F32))
    un = np.sqrt((u * u).sum(-1, keepdims=True, dtype=F32))
    u = u * xn / un
    return (F32(weight) * u + F32(1.0 - weight) * x).astype(F32)


def _proj_weight(img_ad: dict, prefix: str) -> tuple[np.ndarray, bool]:
    if prefix + ".fc.0.weight" in img_ad:
        return img_ad[prefix + ".fc.0.weight"], True
    return img_ad[prefix + ".fc.weight"], False


def patch_embed(sd: dict, x: np.ndarray) -> np.ndarray:
    """conv1 (k=s=14, no bias) -> [B, g*g, width] (adapter.py:68-70)."""
    B, C, S, _ = x.shape
    P = 14
    g = S // P
    cols = x.reshape(B, C, g, P, g, P).transpose(0, 2, 4, 1, 3, 5).reshape(B, g * g, C * P * P)
    w = sd["visual.conv1.weight"].reshape(sd["visual.conv1.weight"].shape[0], -1)
    return (cols @ w.T).astype(F32)


def visual_forward(sd: dict, img_ad: dict, x: np.ndarray, levels=(6, 12, 18, 24),
                   image_adapt_until: int = 6, image_adapt_weight: float = 0.1,
                   return_trace: bool = False, quick: bool = False):
    """AdaptedCLIP.forward (adapter.py:67-112) -> (seg_tokens list [B,P,768] unit rows, det [B,768])."""
    x = patch_embed(sd, x.astype(F32))
    B = x.shape[0]
    cls = np.broadcast_to(sd["visual.class_embedding"], (B, 1, x.shape[-1]))
    x = np.concatenate([cls, x], axis=1) + sd["visual.positional_embedding"]
    x = layer_norm(x, sd["visual.ln_pre.weight"], sd["visual.ln_pre.bias"])
    tokens = []
    trace = []
    for i in range(24):
        x = resblock(x, sd, f"visual.transformer.resblocks.{i}", 16, quick=quick)
        if i < image_adapt_until:
            x = adapter_blend(x, img_ad[f"layer_adapters.{i}.fc.0.weight"], image_adapt_weight)
        if return_trace:
            trace.append(x.copy())
        if i + 1 in levels:
            tokens.append(x[:, 1:, :])
    tokens = [layer_norm(t, sd["visual.ln_post.weight"], sd["visual.ln_post.bias"]) for t in tokens]
    seg = []
    for i, t in enumerate(tokens):
        w, relu = _proj_weight(img_ad, f"seg_proj.{i}")
        s = linear(t, w)
        seg.append(l2_normalize(leaky_relu(s) if relu else s))
    w, relu = _proj_weight(img_ad, "det_proj")
    d = linear(tokens[-1], w)
    d = l2_normalize(leaky_relu(d) if relu else d).mean(1, dtype=F32)
    if return_trace:
        return seg, d, trace
    return seg, d


def encode_text(sd: dict, txt_ad: dict | None, tokens: np.ndarray, text_adapt_until: int = 3,
                text_adapt_weight: float = 0.1, quick: bool = False) -> np.ndarray:
    """AdaptedCLIP.encode_text (adapter.py:114-145) when txt_ad is given,
    else CLIP.encode_text (model.py:190-201)."""
    tokens = np.asarray(tokens).astype(np.int64)
    x = sd["token_embedding.weight"][tokens] + sd["positional_embedding"]
    for i in range(12):
        x = resblock(x, sd, f"transformer.resblocks.{i}", 12, causal=True, quick=quick)
        if txt_ad is not None and i < text_adapt_until:
            x = adapter_blend(x, txt_ad[f"{i}.fc.0.weight"], text_adapt_weight)
    x = layer_norm(x, sd["ln_final.weight"], sd["ln_final.bias"])
    x = x[np.arange(x.shape[0]), tokens.argmax(-1)]
    if txt_ad is not None:
        return leaky_relu(linear(x, txt_ad[f"{text_adapt_until}.fc.0.weight"]))
    return (x @ sd["text_projection"]).astype(F32)


def class_anchor(sd: dict, txt_ad: dict | None, tok_normal: np.ndarray, tok_abnormal: np.ndarray) -> np.ndarray:
    """get_adapted_single_class_text_embedding (forward_utils.py:138-162) given
    the two token tables -> T [768, 2] (normal, abnormal)."""
    cols = []
    for tok in (tok_normal, tok_abnormal):
        e = encode_text(sd, txt_ad, tok)
        e = e / np.sqrt((e * e).sum(-1, keepdims=True, dtype=F32))
        m = e.mean(0, dtype=F32)
        cols.append(m / np.sqrt((m * m).sum(dtype=F32)))
    return np.stack(cols, axis=1).astype(F32)


# --------------------------------------------------------------------------- anomaly map
def gaussian_kernel1d(ksize: int, sigma: float) -> np.ndarray:
    """kornia 0.6.9 get_gaussian_kernel1d: exp(-x^2/(2 s^2)) normalised,
    x = arange(k) - k//2 (+0.5 if k even). Restated (kornia absent): UNPINNED."""
    x = np.arange(ksize, dtype=F32) - F32(ksize // 2)
    if ksize % 2 == 0:
        x = x + F32(0.5)
    g = np.exp(-(x * x) / F32(2.0 * sigma * sigma)).astype(F32)
    return (g / g.sum(dtype=F32)).astype(F32)


def _reflect_index(i: int, n: int) -> int:
    if i < 0:
        return -i
    if i >= n:
        return 2 * (n - 1) - i
    return i


def gaussian_blur2d(x: np.ndarray, ksize: int, sigma: float) -> np.ndarray:
    """kornia.filters.gaussian_blur2d(x, (k,k), (s,s)), border 'reflect',
    separable: x-pass then y-pass. x: [..., H, W]."""
    g = gaussian_kernel1d(ksize, sigma)
    H, W = x.shape[-2:]
    r = ksize // 2
    ix = np.array([[_reflect_index(w + t - r, W) for t in range(ksize)] for w in range(W)])
    iy = np.array([[_reflect_index(h + t - r, H) for t in range(ksize)] for h in range(H)])
    tmp = (x[..., :, ix] * g).sum(-1, dtype=F32)          # [..., H, W]
    out = (np.moveaxis(tmp[..., iy, :], -2, -1) * g).sum(-1, dtype=F32)  # [..., H, W]
    return out.astype(F32)


def upsample_bilinear_ac(x: np.ndarray, size: int) -> np.ndarray:
    """F.interpolate(mode='bilinear', align_corners=True) in ATen's CPU float
    arithmetic: scale=(in-1)/(out-1) in fp32, src=scale*dst, lambdas in fp32."""
    H, W = x.shape[-2:]

    def coords(n_in):
        scale = F32(n_in - 1) / F32(size - 1) if size > 1 else F32(0)
        src = scale * np.arange(size, dtype=F32)
        i0 = np.floor(src).astype(np.int64)
        i0 = np.minimum(i0, n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        l1 = (src - i0.astype(F32)).astype(F32)
        l0 = (F32(1) - l1).astype(F32)
        return i0, i1, l0, l1

    y0, y1, hy0, hy1 = coords(H)
    x0, x1, wx0, wx1 = coords(W)
    top = x[..., y0, :]
    bot = x[..., y1, :]
    a = hy0[:, None] * (wx0 * top[..., :, x0] + wx1 * top[..., :, x1])
    b = hy1[:, None] * (wx0 * bot[..., :, x0] + wx1 * bot[..., :, x1])
    return (a + b).astype(F32)


DOMAIN_BLUR = {"Industrial": (7, 1.0), "Medical": (9, 1.5)}


def calculate_similarity_map(f: np.ndarray, T: np.ndarray, img_size: int, test: bool = False,
                             domain: str = "Medical") -> np.ndarray:
    """forward_utils.py:196-216 -> [B, 1, S, S] (test) or [B, C, S, S] softmax (train)."""
    A = F32(100.0) * (f @ T)  # [B, L, C]
    B, L, C = A.shape
    g = int(np.sqrt(L))
    pred = A.transpose(0, 2, 1).reshape(B, C, g, g)
    if test:
        assert C == 2
        k, s = (7, 1.0) if domain == "Industrial" else (9, 1.5)
        pred = ((pred[:, 1] + F32(1) - pred[:, 0]) / F32(2))[:, None]
        pred = gaussian_blur2d(pred, k, s)
    out = upsample_bilinear_ac(pred, img_size)
    if not test and C > 1:
        out = softmax(out, axis=1)
    return out.astype(F32)


def anomaly_map(seg: list, T: np.ndarray, img_size: int, domain: str) -> np.ndarray:
    """test.py:86-93: per-level map, cat, sum -> [B, S, S]."""
    return sum(calculate_similarity_map(f, T, img_size, True, domain)[:, 0] for f in seg).astype(F32)


def image_score(det: np.ndarray, T: np.ndarray) -> np.ndarray:
    """test.py:83-84: ((det @ T)[:,1] + 1) / 2."""
    p = det @ T
    return ((p[:, 1] + F32(1)) / F32(2)).astype(F32)


def metrics_eval(pixel_label, image_label, pixel_preds, image_preds, class_names, domain):
    """forward_utils.py:233-280 (sklearn AUROC/AP; the reference's own dependency)."""
    from sklearn.metrics import average_precision_score, roc_auc_score
    if pixel_preds.max() != 1:
        pixel_preds = (pixel_preds - pixel_preds.min()) / (pixel_preds.max() - pixel_preds.min())
    if image_preds.max() != 1:
        image_preds = (image_preds - image_preds.min()) / (image_preds.max() - image_preds.min())
    pmax = pixel_preds.max(axis=(1, 2))
    image_preds = pmax * 0.5 + image_preds * 0.5 if domain != "Medical" else pmax
    pl, pp = pixel_label.flatten(), pixel_preds.flatten()
    pauc, pap = roc_auc_score(pl, pp), average_precision_score(pl, pp)
    if image_label.max() != image_label.min():
        iauc = roc_auc_score(image_label.flatten(), image_preds.flatten())
        iap = average_precision_score(image_label.flatten(), image_preds.flatten())
    else:
        iauc = iap = 0
    return {"class name": class_names, "pixel AUC": round(pauc, 4) * 100, "pixel AP": round(pap, 4) * 100,
            "image AUC": round(iauc, 4) * 100, "image AP": round(iap, 4) * 100}
