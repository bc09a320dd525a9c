"""Import-only stub: cv2 is used only by forward_utils.visualize (out of scope)."""
def __getattr__(name):
    raise AttributeError(f"cv2 stub has no {name}")
