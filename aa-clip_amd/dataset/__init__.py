"""get_dataset — drop-in for reference dataset/__init__.py:175-232 (test stage).

Test transform (reference :127-143): PIL bicubic resize to (S, S) -> [0,1]
tensor -> CLIP mean/std normalise; masks: nearest resize -> (mask != 0).
Implemented with PIL + numpy (torchvision is not in this image). Metadata is the
reference's jsonl layout, `./dataset/metadata/<dataset>/full-shot.jsonl`
relative to the working directory (or under $AACLIP_METADATA_ROOT, e.g. the
reference checkout's dataset/metadata — the lists are not shipped here), images
under DATA_PATH[dataset].

Extra: dataset name "synthetic" (no files needed) yields seeded N(0,1)
post-normalisation images and rectangle masks.
Training datasets/augmentation are out of scope.

raw=True (build extension): items carry the decoded uint8
image [H, W, 3] and mask [H, W] instead of the transformed tensors; batch them
with `collate_raw` and transform on the GPU with aaclip.preprocess.Preprocessor,
which is bit-exact with the Pillow transform above (tests/test_preprocess.py).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch
from torch.utils.data import Dataset

from .constants import CLASS_NAMES, DATA_PATH, DOMAINS, PROMPTS, REAL_NAMES  # noqa: F401

MEAN = np.array((0.48145466, 0.4578275, 0.40821073), np.float32)[:, None, None]
STD = np.array((0.26862954, 0.26130258, 0.27577711), np.float32)[:, None, None]


class BaseSingleClassDataset(Dataset):
    def __init__(self, data_path: str, meta_path: str, img_size: int, class_name: str, logger=None,
                 raw: bool = False):
        assert class_name is not None, "class_name should be provided"
        self.data_path, self.img_size, self.raw = data_path, img_size, raw
        self.meta = []
        with open(meta_path) as f:
            for line in f:
                m = json.loads(line.strip())
                if m["class_name"] == class_name:
                    self.meta.append(m)
        if logger:
            logger.info(f"Class name: {class_name}")
            logger.info(f"Sample number: {len(self.meta)}")
            logger.info("=====================================")

    def __len__(self):
        return len(self.meta)

    def _image(self, path):
        from PIL import Image
        img = Image.open(path).convert("RGB").resize((self.img_size, self.img_size), Image.BICUBIC)
        a = np.asarray(img, dtype=np.float32).transpose(2, 0, 1) / 255.0
        return torch.from_numpy((a - MEAN) / STD)

    def _mask(self, path):
        from PIL import Image
        m = Image.open(path).convert("L").resize((self.img_size, self.img_size), Image.NEAREST)
        return torch.from_numpy((np.asarray(m) != 0).astype(np.float32))[None]

    def _raw_item(self, meta):
        from PIL import Image
        img = np.asarray(Image.open(os.path.join(self.data_path, meta["image_path"])).convert("RGB"))
        if meta["label"]:
            m = np.asarray(Image.open(os.path.join(self.data_path, meta["mask_path"])).convert("L"))
        else:
            m = np.zeros(img.shape[:2], np.uint8)
        return {"image_u8": torch.from_numpy(img.copy()), "mask_u8": torch.from_numpy(m.copy()),
                "label": meta["label"], "file_name": meta["image_path"], "class_name": meta["class_name"]}

    def __getitem__(self, idx):
        meta = self.meta[idx]
        if self.raw:
            return self._raw_item(meta)
        img = self._image(os.path.join(self.data_path, meta["image_path"]))
        if meta["label"]:
            mask = self._mask(os.path.join(self.data_path, meta["mask_path"]))
        else:
            mask = torch.zeros([1, self.img_size, self.img_size])
        return {"image": img, "mask": mask, "label": meta["label"], "file_name": meta["image_path"],
                "class_name": meta["class_name"]}


class SyntheticSingleClassDataset(Dataset):
    """Seeded synthetic test set: N(0,1) images (already in normalised space) and
    rectangles covering 1-10% of pixels in every other image (label = mask non-empty)."""

    def __init__(self, n: int, img_size: int, class_name: str = "bottle", seed: int = 111):
        self.n, self.img_size, self.class_name, self.seed = n, img_size, class_name, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        rng = np.random.Generator(np.random.Philox(key=(self.seed << 20) + idx))
        S = self.img_size
        img = rng.standard_normal((3, S, S), dtype=np.float32)
        mask = np.zeros((1, S, S), np.float32)
        if idx % 2 == 1:
            area = rng.uniform(0.01, 0.10) * S * S
            h = int(max(1, min(S, round(np.sqrt(area) * rng.uniform(0.6, 1.4)))))
            w = int(max(1, min(S, round(area / h))))
            y, x = int(rng.integers(0, S - h + 1)), int(rng.integers(0, S - w + 1))
            mask[0, y:y + h, x:x + w] = 1.0
        return {"image": torch.from_numpy(img), "mask": torch.from_numpy(mask), "label": int(mask.max() > 0),
                "file_name": f"synthetic/{idx:05d}.png", "class_name": self.class_name}


def collate_raw(items):
    """Batch raw items: uint8 images/masks stacked when the sizes agree (one
    preprocessing launch), else kept as lists (one launch per size)."""
    out = {k: [it[k] for it in items] for k in items[0]}
    for k in ("image_u8", "mask_u8"):
        if len({tuple(t.shape) for t in out[k]}) == 1:
            out[k] = torch.stack(out[k])
    return out


def metadata_root() -> str:
    """Where the per-dataset jsonl test lists live. The reference reads
    ./dataset/metadata relative to the working directory (dataset/__init__.py:204);
    the same relative path is used here when it exists, else $AACLIP_METADATA_ROOT
    (e.g. <reference checkout>/dataset/metadata: the lists ship with the reference,
    not with this build)."""
    local = "./dataset/metadata"
    if os.path.isdir(local) or "AACLIP_METADATA_ROOT" not in os.environ:
        return local
    return os.environ["AACLIP_METADATA_ROOT"]


def get_dataset(dataset_name: str, img_size: int, training_mode: str, shot: int = -1, stage: str = "train",
                logger=None, synthetic_n: int = 16, raw: bool = False):
    if dataset_name in ("synthetic", "synthetic_mvtec"):
        if stage not in ("test", "visualize"):
            raise ValueError("the synthetic dataset only has a test stage")
        if dataset_name == "synthetic":
            return {"bottle": SyntheticSingleClassDataset(synthetic_n, img_size)}
        # config C4's shape: every MVTec class, its own seed
        return {c: SyntheticSingleClassDataset(synthetic_n, img_size, class_name=c, seed=111 + i)
                for i, c in enumerate(CLASS_NAMES["synthetic_mvtec"])}
    if "Med" not in dataset_name:
        assert dataset_name in DATA_PATH, (
            f"Dataset {dataset_name} not found; available datasets: {list(DATA_PATH.keys())}")
    if stage == "train":
        raise NotImplementedError("training datasets are out of scope (inference path only)")
    if stage in ("test", "visualize"):
        meta_path = os.path.join(metadata_root(), dataset_name, "full-shot.jsonl")
        return {c: BaseSingleClassDataset(DATA_PATH[dataset_name], meta_path, img_size, c,
                                          logger=logger if stage == "test" else None, raw=raw)
                for c in CLASS_NAMES[dataset_name]}
    raise ValueError(f"stage {stage} not found; available stages: train, test")
