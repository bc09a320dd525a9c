"""Import-only stub (the reference imports ipdb but never calls it on the eval path)."""
def set_trace(*a, **k):
    raise RuntimeError("ipdb stub")
