"""aaclip — MI355X-native (gfx950) runtime for AA-CLIP's anomaly-map inference path.

    _lib    ctypes binding of libaaclip_hip.so (include/aaclip.h)
    ops     tensor-level wrappers (host-side shape checks, current HIP stream)
    engine  VisualEngine / TextEngine: the device-resident forward passes
"""
from . import _lib, ops  # noqa: F401
from .engine import TextEngine, VisualEngine  # noqa: F401
