"""Golden for the weight-load path: a synthetic checkpoint in the
OpenAI state-dict layout (oracle/synth.py:write_openai_checkpoint) loaded by the REAL
reference create_model(..., pretrained='openai') (model/clip.py:84-142 ->
model/openai.py:17-83 -> build_model_from_openai_state_dict + fp16 convert_weights,
model/model.py:265-286, :311-368; resize_pos_embed bicubic+antialias, model.py:395-426)
at 336 px (no resize), 448 px (24 -> 32 grid) and 518 px (24 -> 37, the reference's default), from
both checkpoint formats: a plain state dict and the OpenAI release format, a TorchScript
archive (oracle/synth.py:write_openai_torchscript; the reference's torch.jit.load branch,
model/openai.py:56-59). Records SHA-256 of the loaded fp32
state dicts and the resized positional embedding's first rows.
Build container only: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_load_golden.py"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "stubs"))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

import torch  # noqa: E402

from oracle import synth  # noqa: E402


def main():
    prev = os.getcwd()
    os.chdir("/root/reference")
    try:
        import model.clip as rclip
    finally:
        os.chdir(prev)
    out = {"generated_by": "tests/golden/make_load_golden.py (reference create_model pretrained='openai')"}
    import torch
    jit_load = torch.jit.load
    took = []

    def recording_jit_load(*a, **k):  # which branch of openai.py:56-65 ran
        try:
            m = jit_load(*a, **k)
        except RuntimeError:
            took.append(False)
            raise
        took.append(True)
        return m
    torch.jit.load = recording_jit_load
    with tempfile.TemporaryDirectory() as d:
        # both checkpoint formats: a plain state dict (the reference's torch.load fallback)
        # and the OpenAI release format, a TorchScript archive (its torch.jit.load branch,
        # model/openai.py:56-59); the tag records which branch the reference took
        for fmt, writer in (("state_dict", synth.write_openai_checkpoint),
                            ("torchscript", synth.write_openai_torchscript)):
            ck = os.path.join(d, f"{fmt}.pt")
            writer(ck, 111)
            rclip._MODEL_CKPT_PATHS["ViT-L-14-336"] = ck
            for size in (336, 448, 518):
                took.clear()
                m = rclip.create_model("ViT-L-14-336", size, pretrained="openai")
                took_jit = took == [True]
                assert took_jit == (fmt == "torchscript"), (fmt, took)
                sd = m.state_dict()
                key = str(size) if fmt == "state_dict" else f"torchscript_{size}"
                out[key] = {"sha256": synth.torch_state_checksum(sd),
                            "n_keys": len(sd), "reference_branch": "torch.jit.load" if took_jit else "torch.load",
                            "pos_rows": sd["visual.positional_embedding"][:3, :8].tolist(),
                            "pos_shape": list(sd["visual.positional_embedding"].shape)}
                print(fmt, size, out[key]["sha256"], out[key]["pos_shape"], out[key]["reference_branch"])
    torch.jit.load = jit_load
    with open(os.path.join(HERE, "golden_load.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
