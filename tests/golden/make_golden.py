"""Generate the golden vectors under tests/golden/ by running the REAL reference.

Run in the build container only (needs /root/reference; the GPU box never runs
this):  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (wei-paul/AA-CLIP) is imported from /root/reference with the
import-only stubs in tests/golden/stubs (ipdb, cv2, torchvision, ftfy, kornia;
SURVEY §8(c)). Weights are oracle/synth.py's deterministic synthetic weights
loaded into the reference's own modules via load_state_dict(strict=True), so
every fixture here is "reference code on synthetic weights". Outputs:

  golden_e2e.npz    AdaptedCLIP.forward + calculate_similarity_map + image score,
                    B=2 at 336 px (model/adapter.py:67-112, forward_utils.py:196-216,
                    test.py:80-93)
  golden_text.npz   tokenize + encode_text (adapted/unadapted) + class anchors
                    (forward_utils.py:138-162, model/adapter.py:114-145)
  golden_ops.npz    per-op known-answer vectors (LayerNorm, residual blocks,
                    adapter blend, similarity map incl. train branch, metrics_eval)
  golden_c5.npz     config-C5 shapes: 448 px (1025 tokens), 6 levels [4..24],
                    relu=True projections, Medical-domain map, B=1
  golden_quick.npz  towers built with force_quick_gelu=True (clip.py:151-153 -> QuickGELU,
                    transformer.py:46-49): visual/text block KATs, text encoding, B=1
                    336 px grid/det/score/map (`python tests/golden/make_golden.py quick`)
  golden_518.npz    the reference's default test size (test.py:111, results/test.log:1-3):
                    518 px (37x37 grid, 1370 tokens), 4 levels, B=1, both domains
                    (`python tests/golden/make_golden.py 518` regenerates only this file)
  ../../aa-clip_amd/model/prompt_tokens.json   token ids of every prompt the
                    reference can build (tokenizer.py:150-185 over
                    dataset/constants.py:78-148)
  ../../aa-clip_amd/dataset/constants.json     the reference's dataset tables
                    (DATA_PATH, CLASS_NAMES, DOMAINS, REAL_NAMES, PROMPTS)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import torch  # noqa: E402

from oracle import synth  # noqa: E402

torch.set_num_threads(8)
SEED = 111


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def build_reference(relu=False, levels=(6, 12, 18, 24), img_size=336, quick_gelu=False):
    prev = os.getcwd()
    os.chdir(REF)  # the reference resolves ./dataset/metadata relative to cwd
    try:
        from model.clip import create_model
        from model.adapter import AdaptedCLIP
    finally:
        os.chdir(prev)
    # the random-init branch ignores img_size; force_image_size sets the grid (clip.py:159-161)
    clip = create_model("ViT-L-14-336", img_size, pretrained=None, device="cpu",
                        force_image_size=img_size if img_size != 336 else None, force_quick_gelu=quick_gelu)
    sd = synth.clip_state_dict(SEED, img_size=img_size)
    clip.load_state_dict({k: t(v) for k, v in sd.items()}, strict=True)
    clip.eval()
    model = AdaptedCLIP(clip, text_adapt_weight=0.1, image_adapt_weight=0.1, text_adapt_until=3,
                        image_adapt_until=6, levels=list(levels), relu=relu)
    img_ad, txt_ad = synth.adapter_state_dicts(SEED, relu=relu, n_levels=len(levels))
    model.image_adapter.load_state_dict({k: t(v) for k, v in img_ad.items()}, strict=True)
    model.text_adapter.load_state_dict({k: t(v) for k, v in txt_ad.items()}, strict=True)
    model.eval()
    return clip, model, sd, img_ad, txt_ad


def prompt_table():
    from dataset.constants import CLASS_NAMES, PROMPTS, REAL_NAMES
    from model.tokenizer import tokenize
    sentences = []
    for ds, classes in CLASS_NAMES.items():
        for cls in classes:
            names = [REAL_NAMES[ds][cls]] if ds in REAL_NAMES and cls in REAL_NAMES[ds] else []
            for real in names + ["object"]:
                for states in (PROMPTS["prompt_normal"], PROMPTS["prompt_abnormal"]):
                    for s in states:
                        for tpl in PROMPTS["prompt_templates"]:
                            sentences.append(tpl.format(s.format(real)))
    sentences = sorted(set(sentences))
    toks = tokenize(sentences).numpy()
    table = {}
    for s, row in zip(sentences, toks):
        n = int(np.nonzero(row)[0].max()) + 1
        table[s] = [int(v) for v in row[:n]]
    return table


def class_sentences(real_name):
    from dataset.constants import PROMPTS
    out = []
    for states in (PROMPTS["prompt_normal"], PROMPTS["prompt_abnormal"]):
        sent = []
        for s in states:
            for tpl in PROMPTS["prompt_templates"]:
                sent.append(tpl.format(s.format(real_name)))
        out.append(sent)
    return out


@torch.no_grad()
def main():
    clip, model, sd, img_ad, txt_ad = build_reference()
    import forward_utils as fu
    from model.tokenizer import tokenize
    from dataset.constants import REAL_NAMES

    meta = {
        "seed": SEED,
        "clip_sha256": synth.state_checksum(sd),
        "image_adapter_sha256": synth.state_checksum(img_ad),
        "text_adapter_sha256": synth.state_checksum(txt_ad),
        "reference": "wei-paul/AA-CLIP @ /root/reference (synthetic weights, stubs: tests/golden/stubs)",
        "torch": torch.__version__,
    }
    print(meta)

    # ---------------------------------------------------------------- prompt token table
    table = prompt_table()
    tok_path = os.path.join(REPO, "aa-clip_amd", "model", "prompt_tokens.json")
    with open(tok_path, "w") as f:
        json.dump({"generated_by": "tests/golden/make_golden.py (reference tokenizer.py:150-185)",
                   "sot": 49406, "eot": 49407, "context_length": 77, "tokens": table}, f, indent=0,
                  sort_keys=True)
    print("prompts:", len(table), "max len:", max(len(v) for v in table.values()))
    from dataset import constants as C
    with open(os.path.join(REPO, "aa-clip_amd", "dataset", "constants.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/make_golden.py (reference dataset/constants.py tables)",
                   "DATA_PATH": C.DATA_PATH, "CLASS_NAMES": C.CLASS_NAMES, "DOMAINS": C.DOMAINS,
                   "REAL_NAMES": C.REAL_NAMES, "PROMPTS": C.PROMPTS}, f, indent=1)

    # ---------------------------------------------------------------- text
    text = {}
    for tag, real in (("bottle", REAL_NAMES["MVTec"]["bottle"]), ("brain", REAL_NAMES["Brain"]["Brain"])):
        normal_s, abnormal_s = class_sentences(real)
        tn, ta = tokenize(normal_s), tokenize(abnormal_s)
        text[f"{tag}_tok_normal"] = tn.numpy()
        text[f"{tag}_tok_abnormal"] = ta.numpy()
        text[f"{tag}_T_adapted"] = fu.get_adapted_single_class_text_embedding(
            model, "MVTec" if tag == "bottle" else "Brain", "bottle" if tag == "bottle" else "Brain", "cpu").numpy()
        text[f"{tag}_T_clip"] = fu.get_adapted_single_class_text_embedding(
            clip, "MVTec" if tag == "bottle" else "Brain", "bottle" if tag == "bottle" else "Brain", "cpu").numpy()
    text["bottle_enc_abnormal_adapted"] = model.encode_text(t(text["bottle_tok_abnormal"])).numpy()
    text["bottle_enc_abnormal_clip"] = clip.encode_text(t(text["bottle_tok_abnormal"])).numpy()
    np.savez_compressed(os.path.join(HERE, "golden_text.npz"), meta=json.dumps(meta), **text)

    # ---------------------------------------------------------------- e2e visual
    B = 2
    x = synth.images(SEED, B, 336)
    T = t(text["bottle_T_adapted"])
    seg, det = model(t(x))
    grid = np.stack([(100.0 * (f @ T)).numpy() for f in seg], axis=1)  # [B,L,P,2]
    pred = det @ T
    score = ((pred[:, 1] + 1) / 2).numpy()
    maps = {}
    for dom in ("Industrial", "Medical"):
        m = torch.cat([fu.calculate_similarity_map(f, T, 336, test=True, domain=dom) for f in seg], 1).sum(1)
        maps[dom] = m.numpy()
    # residual-stream trace (first 4 tokens of image 0) via hooks on the same forward
    trace = {}
    hooks = []
    for i in (0, 5, 11, 23):
        def mk(i):
            def hook(mod, inp, out):
                trace[i] = out[0][:4, 0, :].detach().clone().numpy()  # LND
            return hook
        hooks.append(model.image_encoder.transformer.resblocks[i].register_forward_hook(mk(i)))
    model(t(x[:1]))
    for h in hooks:
        h.remove()
    e2e = dict(
        image_sha=np.array(synth.state_checksum({"x": x})),
        T=text["bottle_T_adapted"],
        grid_A=grid.astype(np.float32),
        det=det.numpy(),
        score=score,
        map_ind0=maps["Industrial"][0],
        map_ind_sub=maps["Industrial"][:, ::7, ::7],
        map_med_sub=maps["Medical"][:, ::7, ::7],
        seg_head=np.stack([f[:, :8].numpy() for f in seg], axis=1),
        trace_blocks=np.array([0, 5, 11, 23]),
        trace=np.stack([trace[i] for i in (0, 5, 11, 23)]),  # pre-adapter block outputs
    )
    np.savez_compressed(os.path.join(HERE, "golden_e2e.npz"), meta=json.dumps(meta), **e2e)

    # ---------------------------------------------------------------- per-op KATs
    ops = {}
    g = np.random.Generator(np.random.Philox(key=SEED))
    # LayerNorm (transformer.py:37-43)
    ln = model.image_encoder.ln_pre
    xr = (g.standard_normal((16, 1024), dtype=np.float32) * 3 + 0.5).astype(np.float32)
    ops["ln_x"], ops["ln_y"] = xr, ln(t(xr)).numpy()
    # visual residual block 3 on [N=17, B=2, 1024] LND (transformer.py:239-258)
    xv = g.standard_normal((17, 2, 1024), dtype=np.float32)
    ops["vblock_x"] = xv
    ops["vblock_y"] = model.image_encoder.transformer.resblocks[3](t(xv), attn_mask=None)[0].numpy()
    # text residual block 1 with the causal mask, [77, 2, 768]
    xt = (g.standard_normal((77, 1, 768), dtype=np.float32) * 0.5).astype(np.float32)
    ops["tblock_x"] = xt
    ops["tblock_y"] = clip.transformer.resblocks[1](t(xt), attn_mask=clip.attn_mask)[0].numpy()
    # image adapter blend (adapter.py:92-99), layer 2
    xa = g.standard_normal((33, 1024), dtype=np.float32)
    xa_t = t(xa)
    u = model.image_adapter["layer_adapters"][2](xa_t)
    u = u * xa_t.norm(dim=-1, keepdim=True) / u.norm(dim=-1, keepdim=True)
    ops["adapt_x"], ops["adapt_y"] = xa, (0.1 * u + 0.9 * xa_t).numpy()
    # similarity map on a small grid (forward_utils.py:196-216): test (both domains) and train
    f = g.standard_normal((2, 64, 32), dtype=np.float32)
    f = f / np.linalg.norm(f, axis=-1, keepdims=True)
    Tk = g.standard_normal((32, 2), dtype=np.float32)
    Tk = (Tk / np.linalg.norm(Tk, axis=0, keepdims=True)).astype(np.float32)
    ops["sim_f"], ops["sim_T"] = f.astype(np.float32), Tk
    for dom in ("Industrial", "Medical"):
        ops[f"sim_test_{dom}"] = fu.calculate_similarity_map(t(f.astype(np.float32)), t(Tk), 40, test=True,
                                                            domain=dom).numpy()
    ops["sim_train"] = fu.calculate_similarity_map(t(f.astype(np.float32)), t(Tk), 40, test=False).numpy()
    # metrics_eval (forward_utils.py:233-280) on synthetic masks / preds
    mk = synth.masks(SEED, 8, 32)
    pp = g.random((8, 32, 32), dtype=np.float32) + mk[:, 0] * 0.3
    ip = g.random((8,), dtype=np.float32)
    lab = (mk.reshape(8, -1).max(1) > 0).astype(np.int64)
    res = {}
    for dom in ("Industrial", "Medical"):
        r = fu.metrics_eval(mk, lab, pp.copy(), ip.copy(), "synthetic", dom)
        res[dom] = {k: (float(v) if not isinstance(v, str) else v) for k, v in r.items()}
    ops["met_masks"], ops["met_labels"], ops["met_pp"], ops["met_ip"] = mk, lab, pp, ip
    ops["met_result"] = np.array(json.dumps(res))
    np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), meta=json.dumps(meta), **ops)

    # ---------------------------------------------------------------- C5 shapes: 448 px, 6 levels, relu proj
    lv6 = (4, 8, 12, 16, 20, 24)
    _, model448, sd448, ia448, _ = build_reference(relu=True, levels=lv6, img_size=448)
    x448 = synth.images(SEED, 1, 448)
    seg, det = model448(t(x448))
    T = t(text["bottle_T_adapted"])
    c5 = dict(
        levels=np.array(lv6), image_sha=np.array(synth.state_checksum({"x": x448})),
        clip_sha=np.array(synth.state_checksum(sd448)), adapter_sha=np.array(synth.state_checksum(ia448)),
        grid_A=np.stack([(100.0 * (f @ T)).numpy() for f in seg], axis=1).astype(np.float32),
        det=det.numpy(), score=((det @ T)[:, 1].numpy() + 1) / 2,
        map_med_sub=torch.cat([fu.calculate_similarity_map(f, T, 448, test=True, domain="Medical") for f in seg],
                              1).sum(1).numpy()[:, ::8, ::8],
    )
    np.savez_compressed(os.path.join(HERE, "golden_c5.npz"), meta=json.dumps(meta), **c5)
    for fn in ("golden_e2e.npz", "golden_text.npz", "golden_ops.npz", "golden_c5.npz"):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


@torch.no_grad()
def main_518():
    """518 px: 37x37 patch grid (1369 patches + CLS = 1370 tokens), the size of every
    published number; maps are not a multiple of 4 wide (518 % 4 = 2)."""
    _, model, sd, img_ad, _ = build_reference(img_size=518)
    import forward_utils as fu
    text = np.load(os.path.join(HERE, "golden_text.npz"))
    T = t(text["bottle_T_adapted"])
    x = synth.images(SEED, 1, 518)
    seg, det = model(t(x))
    out = dict(image_sha=np.array(synth.state_checksum({"x": x})), clip_sha=np.array(synth.state_checksum(sd)),
               T=text["bottle_T_adapted"],
               grid_A=np.stack([(100.0 * (f @ T)).numpy() for f in seg], axis=1).astype(np.float32),
               det=det.numpy(), score=((det @ T)[:, 1].numpy() + 1) / 2)
    for dom in ("Industrial", "Medical"):
        m = torch.cat([fu.calculate_similarity_map(f, T, 518, test=True, domain=dom) for f in seg], 1).sum(1).numpy()
        out[f"map_{dom}_sub"] = m[:, ::7, ::7]      # every column residue mod 4 and 7
        out[f"map_{dom}_rows"] = m[:, [0, 1, 258, 517], :]  # whole rows incl. the last columns
    np.savez_compressed(os.path.join(HERE, "golden_518.npz"), **out)
    print("golden_518.npz", os.path.getsize(os.path.join(HERE, "golden_518.npz")))


@torch.no_grad()
def main_quick():
    """force_quick_gelu=True (the reference honours it on the non-OpenAI branch,
    model/clip.py:151-153): every MLP runs QuickGELU (transformer.py:46-49)."""
    clip, model, sd, img_ad, txt_ad = build_reference(quick_gelu=True)
    assert type(clip.transformer.resblocks[0].mlp.gelu).__name__ == "QuickGELU"
    import forward_utils as fu
    text = np.load(os.path.join(HERE, "golden_text.npz"))
    g = np.random.Generator(np.random.Philox(key=SEED + 7))
    xv = g.standard_normal((17, 2, 1024), dtype=np.float32)
    xt = (g.standard_normal((77, 1, 768), dtype=np.float32) * 0.5).astype(np.float32)
    # inputs are regenerated by the test from the same Philox key; outputs thinned to keep the file small
    out = dict(clip_sha=np.array(synth.state_checksum(sd)),
               vblock_y=model.image_encoder.transformer.resblocks[3](t(xv), attn_mask=None)[0].numpy()[::2],
               tblock_y=clip.transformer.resblocks[1](t(xt), attn_mask=clip.attn_mask)[0].numpy()[::4],
               tok_abnormal=text["bottle_tok_abnormal"],
               enc_abnormal_adapted=model.encode_text(t(text["bottle_tok_abnormal"])).numpy(),
               enc_abnormal_clip=clip.encode_text(t(text["bottle_tok_abnormal"])).numpy())
    T = t(text["bottle_T_adapted"])
    x = synth.images(SEED, 1, 336)
    seg, det = model(t(x))
    m = torch.cat([fu.calculate_similarity_map(f, T, 336, test=True, domain="Industrial") for f in seg], 1).sum(1)
    out.update(image_sha=np.array(synth.state_checksum({"x": x})), T=text["bottle_T_adapted"],
               grid_A=np.stack([(100.0 * (f @ T)).numpy() for f in seg], axis=1).astype(np.float32),
               det=det.numpy(), score=((det @ T)[:, 1].numpy() + 1) / 2, map_ind_sub=m.numpy()[:, ::7, ::7])
    np.savez_compressed(os.path.join(HERE, "golden_quick.npz"), **out)
    print("golden_quick.npz", os.path.getsize(os.path.join(HERE, "golden_quick.npz")))


if __name__ == "__main__":
    if sys.argv[1:] == ["518"]:
        main_518()
    elif sys.argv[1:] == ["quick"]:
        main_quick()
    else:
        main()
        main_518()
        main_quick()
