"""Drop-in for the reference forward_utils.py entry points of the eval path.

  get_adapted_single_class_text_embedding / get_adapted_text_embedding
      forward_utils.py:138-162, :185-192 — prompt ensemble -> T [768, 2]; the
      encoder runs on the HIP text engine, the normalise/mean/normalise
      reduction in the aaclip_anchor_reduce kernel.
  calculate_similarity_map   forward_utils.py:196-216 — aaclip_patch_scores +
      aaclip_blur_upsample (test: (A1+1-A0)/2 -> Gaussian -> bilinear;
      train: bilinear -> softmax over the two anchors).
  anomaly_map_multilevel     the fused form of test.py:86-93 (all levels in one
      stream kernel, level sum before blur+upsample).
  metrics_eval               forward_utils.py:233-280 — on device (aaclip_metrics_eval:
      min-max normalisation, score fusion, radix-sorted exact tie-aware AUROC / AP,
      identical to sklearn after the reference's 4-decimal rounding). numpy inputs
      are copied to the device; there is no CPU path (without a GPU it raises).
Training losses and visualize() (cv2) are out of scope.
"""
from __future__ import annotations

import numpy as np
import torch

from aaclip import ops
from aaclip.engine import _blur_for
from dataset.constants import CLASS_NAMES, PROMPTS, REAL_NAMES
from model.tokenizer import tokenize

prompt = PROMPTS
prompt_normal = prompt["prompt_normal"]
prompt_abnormal = prompt["prompt_abnormal"]
prompt_state = [prompt_normal, prompt_abnormal]
prompt_templates = prompt["prompt_templates"]


def _sentences(real_name):
    out = []
    for states in prompt_state:
        out.append([tpl.format(s.format(real_name)) for s in states for tpl in prompt_templates])
    return out


def get_adapted_single_class_text_embedding(model, dataset_name, class_name, device):
    if class_name == "object":
        real_name = class_name
    else:
        assert class_name in CLASS_NAMES[dataset_name], (
            f"class_name {class_name} not found; available class_names: {CLASS_NAMES[dataset_name]}")
        real_name = REAL_NAMES[dataset_name][class_name]
    device = torch.device(device)
    T = None
    for col, sentences in enumerate(_sentences(real_name)):
        emb = model.encode_text(tokenize(sentences).to(device)).to(torch.float32).contiguous()
        if T is None:
            T = torch.empty(emb.shape[1], 2, device=emb.device, dtype=torch.float32)
        ops.anchor_reduce(emb, T, col)
    return T.to(device)


def get_adapted_text_embedding(model, dataset_name, device):
    """forward_utils.py:185-192. Same result as one
    get_adapted_single_class_text_embedding per class, but every prompt of every
    class goes through the text tower in ONE encode call (MVTec: 240 sequences =
    18480 token rows, instead of 30 calls of 6-10 sequences that leave the GEMMs
    a few hundred rows): prompts are independent sequences and each one's
    encoding is bit-identical whatever batch it is in
    (tests/test_e2e_gpu.py::test_text_encode_sequence_invariance), so the
    anchors are unchanged."""
    device = torch.device(device)
    sentences, spans = [], []
    for c in CLASS_NAMES[dataset_name]:
        real_name = c if c == "object" else REAL_NAMES[dataset_name][c]
        for col, sents in enumerate(_sentences(real_name)):
            spans.append((c, col, len(sentences), len(sentences) + len(sents)))
            sentences.extend(sents)
    emb = model.encode_text(tokenize(sentences).to(device)).to(torch.float32).contiguous()
    out = {}
    for c, col, a, b in spans:
        if c not in out:
            out[c] = torch.empty(emb.shape[1], 2, device=emb.device, dtype=torch.float32)
        ops.anchor_reduce(emb[a:b], out[c], col)
    return {c: T.to(device) for c, T in out.items()}


def calculate_similarity_map(patch_features, epoch_text_feature, img_size, test=False, domain="Medical"):
    """[B, L, C] features x [C, 2] anchors -> [B, 1, S, S] (test) / [B, 2, S, S] (train)."""
    B, L, C = patch_features.shape
    H = int(np.sqrt(L))
    if H * H != L:
        raise ValueError("patch count must be a square")
    Cn = epoch_text_feature.shape[1]
    if test:
        assert Cn == 2
    elif not 1 <= Cn <= 8:  # checked before any launch: the train-branch upsample holds <= 8 channels per pixel
        raise ValueError(f"train-branch similarity map supports 1..8 anchors, got {Cn}")
    f = patch_features.reshape(B * L, C)
    if f.dtype not in (torch.float32, torch.bfloat16):
        f = f.float()
    f = f.contiguous()
    T = epoch_text_feature.to(f.device, torch.float32).contiguous()
    dev = f.device
    if test:
        grid = torch.empty(B, 1, H, H, device=dev, dtype=torch.float32)
        ops.patch_scores([f], T, grid, normalize=False, mode=0)
        k, s = _blur_for(domain)
        out = torch.empty(B, 1, img_size, img_size, device=dev, dtype=torch.float32)
        return ops.blur_upsample(grid, out, ksize=k, sigma=s)
    grid = torch.empty(B, Cn, H, H, device=dev, dtype=torch.float32)
    if Cn == 2:
        ops.patch_scores([f], T, grid, normalize=False, mode=1, group=L)
    else:  # any anchor count (reference forward_utils.py:199-215 handles every C)
        ops.patch_logits(f, T, grid, group=L)
    out = torch.empty(B, Cn, img_size, img_size, device=dev, dtype=torch.float32)
    return ops.blur_upsample(grid, out, ksize=0, sigma=0.0, softmax=Cn > 1)


def anomaly_map_multilevel(patch_features, epoch_text_feature, img_size, domain="Industrial", normalize=False):
    """sum_l calculate_similarity_map(f_l, T, S, test=True, domain) -> [B, S, S] in one pass."""
    B, L, C = patch_features[0].shape
    g = int(np.sqrt(L))
    lv = [f.reshape(B * L, C).contiguous() for f in patch_features]
    T = epoch_text_feature.to(lv[0].device, torch.float32).contiguous()
    out = torch.empty(B, img_size, img_size, device=lv[0].device, dtype=torch.float32)
    grid = torch.empty(B * L, device=lv[0].device, dtype=torch.float32)
    k, s = _blur_for(domain)
    return ops.anomaly_map(lv, T, out, grid, g=g, ksize=k, sigma=s, normalize=normalize)


def metrics_eval(pixel_label, image_label, pixel_preds, image_preds, class_names: str, domain: str):
    """forward_utils.py:233-280 on the device (aaclip_metrics_eval: class min-max, score
    fusion, exact tie-aware AUROC / AP). Tensors or numpy arrays; the rounding and the
    dict layout are the reference's. There is no CPU path: without a GPU this raises."""
    return metrics_eval_deferred(pixel_label, image_label, pixel_preds, image_preds, class_names, domain)()


def metrics_eval_deferred(pixel_label, image_label, pixel_preds, image_preds, class_names: str, domain: str):
    """metrics_eval enqueued on the device now, read later: returns a function that syncs
    and builds the reference's dict. The harness enqueues every class before reading any,
    so no class waits for the previous one's metrics on the host."""
    if not torch.cuda.is_available():
        raise RuntimeError("metrics_eval runs on the MI355X kernels (aaclip_metrics_eval); no GPU is visible "
                           "and there is no CPU path")
    dev = next((t.device for t in (pixel_preds, pixel_label) if isinstance(t, torch.Tensor) and t.is_cuda),
               torch.device("cuda", torch.cuda.current_device()))
    t = [x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))
         for x in (pixel_preds, pixel_label, image_preds, image_label)]
    t = [x.to(dev, non_blocking=True) for x in t]
    res = ops.metrics_eval_device(t[0], t[1], t[2], t[3], medical=(domain == "Medical"))

    def read():
        pauc, pap, iauc, iap = res.tolist()
        if pauc != pauc:  # NaN: one pixel class only, sklearn raises here
            raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
        return {"class name": class_names, "pixel AUC": round(pauc, 4) * 100, "pixel AP": round(pap, 4) * 100,
                "image AUC": round(iauc, 4) * 100, "image AP": round(iap, 4) * 100}
    return read


def visualize(pixel_label, pixel_preds, file_names, save_dir, dataset_name, class_name):
    raise NotImplementedError("visualize() writes cv2 overlays; cv2 is not in this image and it is not on the path")
