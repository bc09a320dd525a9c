"""kornia stub: only kornia.filters.gaussian_blur2d is on the path
(forward_utils.py:8, :208-210); it is RESTATED from kornia==0.6.9's published
algorithm in filters.py (kornia is absent: parity at this boundary is unpinned)."""
from . import filters  # noqa: F401
