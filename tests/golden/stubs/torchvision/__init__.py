"""Import-only stub: torchvision is used by the reference's dataset/augmentation
code only; nothing on the golden-vector path calls it."""
from . import transforms  # noqa: F401
