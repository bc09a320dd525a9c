"""Dataset tables of the reference (dataset/constants.py:1-148): DATA_PATH,
CLASS_NAMES, DOMAINS, REAL_NAMES, PROMPTS — loaded from constants.json, which
tests/golden/make_golden.py dumps from the reference module."""
import json
import os

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "constants.json")) as _f:
    _T = json.load(_f)

BASE_PATH = "./data"
DATA_PATH = _T["DATA_PATH"]
CLASS_NAMES = _T["CLASS_NAMES"]
DOMAINS = _T["DOMAINS"]
REAL_NAMES = _T["REAL_NAMES"]
PROMPTS = _T["PROMPTS"]

# Build-only entry: the synthetic test set (config C1) reuses MVTec "bottle" prompts.
CLASS_NAMES["synthetic"] = ["bottle"]
REAL_NAMES["synthetic"] = {"bottle": REAL_NAMES["MVTec"]["bottle"]}
DOMAINS["synthetic"] = "Industrial"
# Build-only entry: config C4's flow (MVTec-AD's 15 classes and their ensemble
# prompts, Industrial blur) on seeded synthetic images and masks.
CLASS_NAMES["synthetic_mvtec"] = list(CLASS_NAMES["MVTec"])
REAL_NAMES["synthetic_mvtec"] = dict(REAL_NAMES["MVTec"])
DOMAINS["synthetic_mvtec"] = "Industrial"
