"""torch_geometric.debug (PyG 1.4.3): a global flag that turns on the extra
argument checks of the layers (pattern: /root/reference/gmm_conv.py:106-129)."""
__debug_flag__ = {"enabled": False}


def is_debug_enabled():
    return __debug_flag__["enabled"]


def set_debug_enabled(mode):
    __debug_flag__["enabled"] = bool(mode)


class debug(object):
    """Context manager enabling debug mode."""

    def __init__(self):
        self.prev = is_debug_enabled()

    def __enter__(self):
        set_debug_enabled(True)

    def __exit__(self, *args):
        set_debug_enabled(self.prev)
        return False


class set_debug(object):
    """Sets debug mode on or off (usable as a function or a context manager)."""

    def __init__(self, mode):
        self.prev = is_debug_enabled()
        set_debug_enabled(mode)

    def __enter__(self):
        pass

    def __exit__(self, *args):
        set_debug_enabled(self.prev)
        return False
