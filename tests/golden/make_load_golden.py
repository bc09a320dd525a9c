"""Golden for the weight-load path: a synthetic checkpoint in the
OpenAI state-dict layout (oracle/synth.py:write_openai_checkpoint) loaded by the REAL
reference create_model(..., pretrained='openai') (model/clip.py:84-142 ->
model/openai.py:17-83 -> build_model_from_openai_state_dict + fp16 convert_weights,
model/model.py:265-286, :311-368; resize_pos_embed bicubic+antialias, model.py:395-426)
at 336 px (no resize), 448 px (24 -> 32 grid) and 518 px (24 -> 37, the reference's default). Records SHA-256 of the loaded fp32
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
    with tempfile.TemporaryDirectory() as d:
        ck = os.path.join(d, "ViT-L-14-336px.pt")
        synth.write_openai_checkpoint(ck, 111)
        rclip._MODEL_CKPT_PATHS["ViT-L-14-336"] = ck
        for size in (336, 448, 518):
            m = rclip.create_model("ViT-L-14-336", size, pretrained="openai")
            sd = m.state_dict()
            out[str(size)] = {"sha256": synth.torch_state_checksum(sd),
                              "n_keys": len(sd),
                              "pos_rows": sd["visual.positional_embedding"][:3, :8].tolist(),
                              "pos_shape": list(sd["visual.positional_embedding"].shape)}
            print(size, out[str(size)]["sha256"], out[str(size)]["pos_shape"])
    with open(os.path.join(HERE, "golden_load.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
