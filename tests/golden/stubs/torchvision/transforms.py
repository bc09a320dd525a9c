"""Import-only stub for torchvision.transforms."""
class _Unavailable:
    def __init__(self, *a, **k):
        pass
    def __call__(self, *a, **k):
        raise RuntimeError("torchvision stub")
def __getattr__(name):
    return _Unavailable
