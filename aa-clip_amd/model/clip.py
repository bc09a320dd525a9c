"""create_model + the CLIP container (reference model/clip.py:84-202, model/model.py:149-212).

The container keeps the reference's module tree and parameter names
(`visual.conv1`, `visual.transformer.resblocks.{i}.attn.in_proj_weight`, ...,
`transformer.resblocks.{i}...`, `token_embedding`, `positional_embedding`,
`ln_final`, `text_projection`, `logit_scale`, buffer `attn_mask`), so the
reference's state dicts load with strict=True. The modules are weight holders:
compute runs on the HIP engines (aaclip.engine), never through their eager
forward.

Only the ViT-L/14-336 tower of the reference's config registry is on the path
(model/model_configs/ViT-L-14-336.json); it is restated below.
"""
from __future__ import annotations

import logging
import math
import os
from collections import OrderedDict
from typing import Optional, Tuple, Union

import torch
import torch.nn.functional as F
from torch import nn

MODEL_CONFIGS = {
    "ViT-L-14-336": {
        "embed_dim": 768,
        "vision_cfg": {"image_size": 336, "layers": 24, "width": 1024, "patch_size": 14},
        "text_cfg": {"context_length": 77, "vocab_size": 49408, "width": 768, "heads": 12, "layers": 12},
    }
}
_MODEL_CKPT_PATHS = {"ViT-L-14-336": os.path.join(os.path.dirname(os.path.abspath(__file__)), "ViT-L-14-336px.pt")}
OPENAI_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_STD = (0.26862954, 0.26130258, 0.27577711)


def get_model_config(model_name):
    cfg = MODEL_CONFIGS.get(model_name)
    return None if cfg is None else {k: (dict(v) if isinstance(v, dict) else v) for k, v in cfg.items()}


class QuickGELU(nn.Module):
    """x * sigmoid(1.702 x) (reference model/transformer.py:46-49). Marks a tower built
    with quick_gelu=True: the engines fuse it into the c_fc epilogue
    (AACLIP_EPI_QGELU); this eager forward is never on the HIP path."""

    def forward(self, x: torch.Tensor):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    """Parameter holder with the names of reference transformer.py:183-219."""

    def __init__(self, d_model: int, n_head: int, mlp_ratio: float = 4.0, act_layer=nn.GELU):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d_model)
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_2 = nn.LayerNorm(d_model)
        w = int(d_model * mlp_ratio)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d_model, w)), ("gelu", act_layer()),
                                              ("c_proj", nn.Linear(w, d_model))]))


class Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int, mlp_ratio: float = 4.0, act_layer=nn.GELU):
        super().__init__()
        self.width, self.layers = width, layers
        self.grad_checkpointing = False
        self.resblocks = nn.ModuleList([ResidualAttentionBlock(width, heads, mlp_ratio, act_layer)
                                        for _ in range(layers)])

    @property
    def quick_gelu(self) -> bool:
        """The MLP activation the engines fuse: QuickGELU (True) or nn.GELU."""
        return bool(self.resblocks) and isinstance(self.resblocks[0].mlp.gelu, QuickGELU)

    def get_cast_dtype(self) -> torch.dtype:
        return self.resblocks[0].mlp.c_fc.weight.dtype


class VisionTransformer(nn.Module):
    """Parameter holder with the names of reference transformer.py:320-402."""

    def __init__(self, image_size: int, patch_size: int, width: int, layers: int, heads: int,
                 output_dim: int, mlp_ratio: float = 4.0, act_layer=nn.GELU):
        super().__init__()
        self.image_size = (image_size, image_size)
        self.patch_size = (patch_size, patch_size)
        self.grid_size = (image_size // patch_size, image_size // patch_size)
        self.output_dim = output_dim
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn(self.grid_size[0] * self.grid_size[1] + 1, width))
        self.patch_dropout = nn.Identity()  # PatchDropout is the identity in eval (transformer.py:74-75)
        self.ln_pre = nn.LayerNorm(width)
        self.transformer = Transformer(width, layers, heads, mlp_ratio, act_layer)
        self.embed_dim, self.num_heads = width, heads
        self.ln_post = nn.LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))


class CLIP(nn.Module):
    def __init__(self, embed_dim: int, vision_cfg: dict, text_cfg: dict, quick_gelu: bool = False,
                 cast_dtype: Optional[torch.dtype] = None, output_dict: bool = False):
        super().__init__()
        # reference model/model.py:84,129: act_layer = QuickGELU if quick_gelu else nn.GELU
        act_layer = QuickGELU if quick_gelu else nn.GELU
        self.quick_gelu = bool(quick_gelu)
        self.output_dict = output_dict
        v = vision_cfg
        self.visual = VisionTransformer(v["image_size"], v["patch_size"], v["width"], v["layers"],
                                        v["width"] // v.get("head_width", 64), embed_dim, v.get("mlp_ratio", 4.0),
                                        act_layer)
        t = text_cfg
        self.transformer = Transformer(t["width"], t["layers"], t["heads"], act_layer=act_layer)
        self.vocab_size = t["vocab_size"]
        self.token_embedding = nn.Embedding(t["vocab_size"], t["width"])
        self.positional_embedding = nn.Parameter(torch.empty(t["context_length"], t["width"]))
        self.ln_final = nn.LayerNorm(t["width"])
        self.text_projection = nn.Parameter(torch.empty(t["width"], embed_dim))
        mask = torch.full((t["context_length"], t["context_length"]), float("-inf")).triu_(1)
        self.register_buffer("attn_mask", mask, persistent=False)
        self.logit_scale = nn.Parameter(torch.ones([]) * math.log(1 / 0.07))
        self._init_text()
        self._text_engine = None
        self._text_sig = None

    def _init_text(self):
        # reference TextTransformer.init_parameters (transformer.py:597-617)
        nn.init.normal_(self.token_embedding.weight, std=0.02)
        nn.init.normal_(self.positional_embedding, std=0.01)
        w, L = self.transformer.width, self.transformer.layers
        for blk in self.transformer.resblocks:
            nn.init.normal_(blk.attn.in_proj_weight, std=w ** -0.5)
            nn.init.normal_(blk.attn.out_proj.weight, std=(w ** -0.5) * ((2 * L) ** -0.5))
            nn.init.normal_(blk.mlp.c_fc.weight, std=(2 * w) ** -0.5)
            nn.init.normal_(blk.mlp.c_proj.weight, std=(w ** -0.5) * ((2 * L) ** -0.5))
        nn.init.normal_(self.text_projection, std=w ** -0.5)

    def text_params(self) -> dict:
        return {k: v for k, v in self.state_dict().items() if not k.startswith("visual.")}

    def text_engine(self, adapter_sd=None, adapt_until=3, adapt_weight=0.1):
        from aaclip.engine import TextEngine
        from .adapter import param_signature
        sig = (param_signature(self, prefix_excl="visual."), None if adapter_sd is None else
               tuple((k, v.data_ptr(), v._version) for k, v in adapter_sd.items()), adapt_until, adapt_weight)
        if self._text_engine is None or self._text_sig != sig:
            self._text_engine = TextEngine(self.text_params(), adapter_sd, text_adapt_until=adapt_until,
                                           text_adapt_weight=adapt_weight, dtype=torch.float32,
                                           quick_gelu=self.transformer.quick_gelu)
            self._text_sig = sig
        return self._text_engine

    def encode_text(self, text, normalize: bool = False):
        """CLIP.encode_text (reference model/model.py:190-201), on the HIP text engine."""
        x = self.text_engine().encode(text)
        if normalize:
            from aaclip import ops
            y = torch.empty_like(x)
            ops.l2_normalize(x, y)
            return y
        return x

    def encode_image(self, image, out_layers, normalize: bool = False):
        raise NotImplementedError("CLIP.encode_image (forward_original) is not on the AA-CLIP eval path; "
                                  "use AdaptedCLIP.forward")


def resize_pos_embed(state_dict, model, interpolation: str = "bicubic", antialias: bool = True):
    """Load-time grid resize of visual.positional_embedding (reference
    model/model.py:395-426): bicubic, antialias, align_corners=False; the CLS
    row is kept. Host-side, once per checkpoint load (not on the hot path)."""
    old = state_dict.get("visual.positional_embedding", None)
    if old is None:
        return
    gh, gw = model.visual.grid_size
    if gh * gw + 1 == old.shape[0]:
        return
    tok, img = old[:1], old[1:]
    og = int(math.sqrt(len(img)))
    logging.info("Resizing position embedding grid-size from %s to %s", (og, og), (gh, gw))
    img = img.reshape(1, og, og, -1).permute(0, 3, 1, 2).float()
    img = F.interpolate(img, size=(gh, gw), mode=interpolation, antialias=antialias, align_corners=False)
    img = img.permute(0, 2, 3, 1).reshape(gh * gw, -1)
    state_dict["visual.positional_embedding"] = torch.cat([tok.float(), img], 0)


def _fp16_round_openai(model: nn.Module, state_dict: dict) -> dict:
    """The OpenAI loader converts Linear/Conv/MHA weights+biases and
    proj/text_projection to fp16 before loading (model/model.py:265-286, :366),
    so the effective fp32 weights are fp16-rounded."""
    out = {}
    for k, v in state_dict.items():
        lp = (k.endswith(("in_proj_weight", "in_proj_bias")) or k.endswith(("proj", "text_projection"))
              or (".weight" in k and any(s in k for s in ("conv1", "c_fc", "c_proj", "out_proj")))
              or (".bias" in k and any(s in k for s in ("c_fc", "c_proj", "out_proj"))))
        out[k] = v.half().float() if (lp and v.is_floating_point()) else v.float() if v.is_floating_point() else v
    return out


def _is_torchscript(path: str) -> bool:
    import zipfile
    try:
        with zipfile.ZipFile(path) as z:
            names = z.namelist()
    except (zipfile.BadZipFile, OSError):
        return False
    return any(n.endswith("constants.pkl") for n in names) and any("/code/" in n or n.startswith("code/")
                                                                   for n in names)


def load_openai_state_dict(path: str) -> dict:
    """OpenAI ViT-L-14-336px.pt: a TorchScript archive (reference model/openai.py:56-65);
    read its tensors with torch.jit.load, or a plain state dict with weights_only."""
    if not os.path.exists(path):
        raise RuntimeError(f"Model {path} not found; available models = {list(_MODEL_CKPT_PATHS)}")
    try:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd:
            sd = sd["state_dict"]
    except Exception:
        # only a TorchScript archive (the OpenAI release format: code/ + constants.pkl)
        # goes to torch.jit.load; a corrupt / truncated / other file keeps its error
        if not _is_torchscript(path):
            raise
        sd = torch.jit.load(path, map_location="cpu").state_dict()
    for k in ("input_resolution", "context_length", "vocab_size"):
        sd.pop(k, None)
    return sd


def create_model(model_name: str, img_size: int, pretrained: Optional[str] = None, precision: str = "fp32",
                 device: Union[str, torch.device] = "cpu", jit: bool = False, force_quick_gelu: bool = False,
                 force_custom_text: bool = False, force_patch_dropout: Optional[float] = None,
                 force_image_size: Optional[Union[int, Tuple[int, int]]] = None, output_dict: Optional[bool] = None,
                 require_pretrained: bool = False, adapter=False):
    """Same signature and error behaviour as reference model/clip.py:84-202.

    jit=True: the reference scripts the model (torch.jit.script, clip.py:141,199); here
    the compiled form of the hot path is the engines' hipGraph (predict_cached captures
    the whole forward + map + score per shape), so the model is returned as built.
    force_quick_gelu: as in the reference, honoured on the non-OpenAI branch only
    (clip.py:151-153); the OpenAI branch builds from the config (nn.GELU)."""
    model_name = model_name.replace("/", "-")
    if isinstance(device, str):
        device = torch.device(device)
    if force_custom_text:
        raise NotImplementedError("custom-text CLIP variants are not on the AA-CLIP path")
    if jit:
        logging.info("jit=True: the HIP engines capture the forward in a hipGraph (predict_cached); "
                     "no TorchScript pass")
    model_cfg = get_model_config(model_name)
    if model_cfg is None:
        raise RuntimeError(f"Model config for {model_name} not found.")
    if pretrained and pretrained.lower() == "openai":
        logging.info(f"Loading pretrained {model_name} from OpenAI.")
        model_cfg["vision_cfg"]["image_size"] = img_size
        model = CLIP(**model_cfg)
        sd = _fp16_round_openai(model, load_openai_state_dict(str(_MODEL_CKPT_PATHS[model_name])))
        resize_pos_embed(sd, model)
        model.load_state_dict(sd, strict=True)
    else:
        if force_quick_gelu:
            model_cfg["quick_gelu"] = True
        if force_image_size is not None:
            model_cfg["vision_cfg"]["image_size"] = force_image_size
        model = CLIP(**model_cfg)
        if pretrained:
            raise RuntimeError(f"Pretrained weights ({pretrained}) not found for model {model_name}.")
        if require_pretrained:
            raise RuntimeError(f"Pretrained weights were required for (model: {model_name}, "
                               f"pretrained: {pretrained}) but not loaded.")
    model.to(device=device)
    if precision not in ("fp32", "amp", "pure_fp32"):
        logging.info("precision=%s: weights stay fp32; the engines choose the compute dtype", precision)
    model.visual.image_mean = OPENAI_MEAN
    model.visual.image_std = OPENAI_STD
    if output_dict:
        model.output_dict = True
    return model
