"""Deterministic synthetic weights and inputs for AA-CLIP parity tests.

TEST INFRASTRUCTURE — part of the oracle. Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module.

The reference ships no weights (`model/ViT-L-14-336px.pt` is absent,
reference `model/clip.py:16`), so every parity case runs on synthetic weights.
They come from a counter-based generator (numpy Philox keyed by (seed, crc32
of the tensor name)), so the GPU box regenerates exactly the bytes that the
golden-fixture script fed into the real reference in the build container.
`state_checksum` pins the bytes.

Shapes follow the reference state dict:
  * CLIP visual tower  — `model/transformer.py:320-402` (conv1, class_embedding,
    positional_embedding, ln_pre, transformer.resblocks.*, ln_post, proj)
  * CLIP text tower    — `model/model.py:165-172` (transformer.*, token_embedding,
    positional_embedding, ln_final, text_projection)
  * AA-CLIP adapters   — `model/adapter.py:27-44` (image_adapter.*, text_adapter.*)

Distributions: weights ~ N(0, std) with std chosen so each residual block adds
an O(1) update (larger than open_clip's proj_std, which would hide block-level
bugs behind a residual stream dominated by the embeddings); LayerNorm gamma/beta
and biases are randomised (the default init 1/0 would hide bugs).
Linear/conv/MHA weights+biases and proj/text_projection are rounded through
fp16, reproducing the effective weights of the OpenAI load path
(reference `model/model.py:366`, `:265-286`).
"""
from __future__ import annotations

import hashlib
import zlib

import numpy as np

VISION_WIDTH = 1024
VISION_LAYERS = 24
VISION_HEADS = 16
PATCH = 14
EMBED_DIM = 768
TEXT_WIDTH = 768
TEXT_LAYERS = 12
TEXT_HEADS = 12
CONTEXT = 77
VOCAB = 49408


def _rng(seed: int, name: str) -> np.random.Generator:
    key = (int(seed) & 0xFFFFFFFF) << 32 | zlib.crc32(name.encode())
    return np.random.Generator(np.random.Philox(key=key))


def normal(seed: int, name: str, shape, std: float = 1.0, mean: float = 0.0) -> np.ndarray:
    x = _rng(seed, name).standard_normal(size=shape, dtype=np.float32)
    return (x * np.float32(std) + np.float32(mean)).astype(np.float32)


def uniform(seed: int, name: str, shape, bound: float) -> np.ndarray:
    x = _rng(seed, name).random(size=shape, dtype=np.float32)
    return ((x * 2.0 - 1.0) * np.float32(bound)).astype(np.float32)


def _fp16(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).astype(np.float32)


def _ln(sd, seed, prefix, width):
    sd[prefix + ".weight"] = normal(seed, prefix + ".weight", (width,), 0.1, 1.0)
    sd[prefix + ".bias"] = normal(seed, prefix + ".bias", (width,), 0.05)


def _block(sd, seed, prefix, width, n_layers_total):
    _ln(sd, seed, prefix + ".ln_1", width)
    _ln(sd, seed, prefix + ".ln_2", width)
    w = width
    sd[prefix + ".attn.in_proj_weight"] = _fp16(normal(seed, prefix + ".attn.in_proj_weight", (3 * w, w), w ** -0.5))
    sd[prefix + ".attn.in_proj_bias"] = _fp16(normal(seed, prefix + ".attn.in_proj_bias", (3 * w,), 0.02))
    sd[prefix + ".attn.out_proj.weight"] = _fp16(normal(seed, prefix + ".attn.out_proj.weight", (w, w), w ** -0.5))
    sd[prefix + ".attn.out_proj.bias"] = _fp16(normal(seed, prefix + ".attn.out_proj.bias", (w,), 0.02))
    sd[prefix + ".mlp.c_fc.weight"] = _fp16(normal(seed, prefix + ".mlp.c_fc.weight", (4 * w, w), (2 * w) ** -0.5))
    sd[prefix + ".mlp.c_fc.bias"] = _fp16(normal(seed, prefix + ".mlp.c_fc.bias", (4 * w,), 0.02))
    sd[prefix + ".mlp.c_proj.weight"] = _fp16(normal(seed, prefix + ".mlp.c_proj.weight", (w, 4 * w), (4 * w) ** -0.5))
    sd[prefix + ".mlp.c_proj.bias"] = _fp16(normal(seed, prefix + ".mlp.c_proj.bias", (w,), 0.02))


def clip_state_dict(seed: int = 111, img_size: int = 336) -> dict[str, np.ndarray]:
    """Full CLIP ViT-L/14-336 state dict (visual + text), reference key names."""
    sd: dict[str, np.ndarray] = {}
    g = img_size // PATCH
    w = VISION_WIDTH
    sd["visual.class_embedding"] = normal(seed, "visual.class_embedding", (w,), w ** -0.5)
    sd["visual.positional_embedding"] = normal(seed, "visual.positional_embedding", (g * g + 1, w), w ** -0.5)
    sd["visual.proj"] = _fp16(normal(seed, "visual.proj", (w, EMBED_DIM), w ** -0.5))
    sd["visual.conv1.weight"] = _fp16(normal(seed, "visual.conv1.weight", (w, 3, PATCH, PATCH), (3 * PATCH * PATCH) ** -0.5))
    _ln(sd, seed, "visual.ln_pre", w)
    for i in range(VISION_LAYERS):
        _block(sd, seed, f"visual.transformer.resblocks.{i}", w, VISION_LAYERS)
    _ln(sd, seed, "visual.ln_post", w)

    tw = TEXT_WIDTH
    sd["positional_embedding"] = normal(seed, "positional_embedding", (CONTEXT, tw), 0.01)
    sd["text_projection"] = _fp16(normal(seed, "text_projection", (tw, EMBED_DIM), tw ** -0.5))
    sd["logit_scale"] = np.array(np.log(1 / 0.07), dtype=np.float32)
    for i in range(TEXT_LAYERS):
        _block(sd, seed, f"transformer.resblocks.{i}", tw, TEXT_LAYERS)
    sd["token_embedding.weight"] = normal(seed, "token_embedding.weight", (VOCAB, tw), 0.02)
    _ln(sd, seed, "ln_final", tw)
    return sd


def _xavier(seed, name, fan_out, fan_in):
    return uniform(seed, name, (fan_out, fan_in), float(np.sqrt(6.0 / (fan_in + fan_out))))


def adapter_state_dicts(seed: int = 111, relu: bool = False, n_levels: int = 4,
                        image_adapt_until: int = 6, text_adapt_until: int = 3):
    """(image_adapter, text_adapter) state dicts with the keys of reference
    `model/adapter.py:27-44` (SimpleAdapter = `fc.0`, SimpleProj = `fc` or `fc.0`
    when relu, `model/adapter_modules.py:6-26`). xavier_uniform like
    `adapter.py:47-53`."""
    img: dict[str, np.ndarray] = {}
    for i in range(image_adapt_until):
        k = f"layer_adapters.{i}.fc.0.weight"
        img[k] = _xavier(seed, "image_adapter." + k, 1024, 1024)
    proj_key = "fc.0.weight" if relu else "fc.weight"
    for i in range(n_levels):
        k = f"seg_proj.{i}.{proj_key}"
        img[k] = _xavier(seed, f"image_adapter.seg_proj.{i}", 768, 1024)
    img[f"det_proj.{proj_key}"] = _xavier(seed, "image_adapter.det_proj", 768, 1024)
    txt: dict[str, np.ndarray] = {}
    for i in range(text_adapt_until):
        txt[f"{i}.fc.0.weight"] = _xavier(seed, f"text_adapter.{i}", 768, 768)
    txt[f"{text_adapt_until}.fc.0.weight"] = _xavier(seed, f"text_adapter.{text_adapt_until}", 768, 768)
    return img, txt


def images(seed: int, batch: int, img_size: int = 336) -> np.ndarray:
    """Synthetic post-normalisation images, N(0,1)."""
    return normal(seed, f"images.{batch}.{img_size}", (batch, 3, img_size, img_size), 1.0)


def masks(seed: int, batch: int, img_size: int) -> np.ndarray:
    """Seeded rectangles covering 1-10% of pixels in half the images."""
    rng = _rng(seed, f"masks.{batch}.{img_size}")
    m = np.zeros((batch, 1, img_size, img_size), np.float32)
    for b in range(batch):
        if b % 2 == 1:
            area = rng.uniform(0.01, 0.10) * img_size * img_size
            h = int(max(1, min(img_size, round(np.sqrt(area) * rng.uniform(0.6, 1.4)))))
            w = int(max(1, min(img_size, round(area / h))))
            y = int(rng.integers(0, img_size - h + 1))
            x = int(rng.integers(0, img_size - w + 1))
            m[b, 0, y:y + h, x:x + w] = 1.0
    return m


def state_checksum(sd: dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest()


_OPENAI_FP16 = ("conv1.weight", "in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias",
                "c_fc.weight", "c_fc.bias", "c_proj.weight", "c_proj.bias", "visual.proj", "text_projection")


def write_openai_checkpoint(path: str, seed: int = 111) -> None:
    """A synthetic checkpoint in the OpenAI ViT-L-14-336px.pt state-dict layout: the
    tensors OpenAI's convert_weights casts (reference model/model.py:265-286) stored as
    fp16, the rest fp32, plus the input_resolution/context_length/vocab_size entries the
    loaders drop (reference model/model.py:366). Plain torch.save (no pickled code)."""
    import torch
    sd = clip_state_dict(seed)
    out = {}
    for k, v in sd.items():
        t = torch.from_numpy(np.ascontiguousarray(v))
        out[k] = t.half() if k.endswith(_OPENAI_FP16) else t
    out["input_resolution"] = torch.tensor(336)
    out["context_length"] = torch.tensor(CONTEXT)
    out["vocab_size"] = torch.tensor(VOCAB)
    torch.save(out, path)


def _torchscript_holder(tensors: dict):
    """A module tree whose state_dict() keys are exactly `tensors`' dotted names (floating
    tensors as parameters, the rest as buffers), scriptable: the shape of the OpenAI
    release archive's module (reference model/openai.py:56-59 reads it with
    torch.jit.load(...).state_dict())."""
    import torch
    from torch import nn

    class Holder(nn.Module):
        def forward(self, x: torch.Tensor) -> torch.Tensor:
            return x

    root = Holder()
    for k, v in tensors.items():
        parts = k.split(".")
        m = root
        for p in parts[:-1]:
            if p not in m._modules:
                m.add_module(p, Holder())
            m = m._modules[p]
        if v.is_floating_point():
            m.register_parameter(parts[-1], nn.Parameter(v, requires_grad=False))
        else:
            m.register_buffer(parts[-1], v)
    return root


def write_openai_torchscript(path: str, seed: int = 111) -> None:
    """The same synthetic checkpoint as write_openai_checkpoint, in the OpenAI RELEASE
    format: a TorchScript archive (torch.jit.save of a scripted module holding the
    tensors; fp16 where OpenAI's convert_weights casts, metadata entries as buffers).
    The reference's loader takes its torch.jit.load branch on it (model/openai.py:56-59,
    then build_model_from_openai_state_dict(model.state_dict()))."""
    import torch
    sd = clip_state_dict(seed)
    tensors = {}
    for k, v in sd.items():
        t = torch.from_numpy(np.ascontiguousarray(v))
        tensors[k] = t.half() if k.endswith(_OPENAI_FP16) else t
    tensors["input_resolution"] = torch.tensor(336)
    tensors["context_length"] = torch.tensor(CONTEXT)
    tensors["vocab_size"] = torch.tensor(VOCAB)
    torch.jit.save(torch.jit.script(_torchscript_holder(tensors)), path)


def torch_state_checksum(sd) -> str:
    """SHA-256 over a torch state dict's floating tensors as float32 (sorted keys)."""
    h = hashlib.sha256()
    for k in sorted(sd):
        v = sd[k]
        if not v.is_floating_point():
            continue
        h.update(k.encode())
        h.update(v.detach().float().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()
