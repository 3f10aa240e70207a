"""Loader for the in-tree native HIP extension ``epfl_megatron_amd._C``.

GPU tensors ALWAYS take the hand-written gfx950 kernels; there is no silent
fallback: if the extension is missing on a GPU run we raise.  CPU tensors
(the gloo plumbing path and test oracles) use plain PyTorch reference math.
"""
import importlib

_EXT = None
_ERR = None


def ext():
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    try:
        _EXT = importlib.import_module("epfl_megatron_amd._C")
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        _ERR = e
        raise RuntimeError(
            "epfl_megatron_amd native HIP extension (_C) is not built or failed to load: "
            f"{e}. Build it with `python -m epfl_megatron_amd.build` (hipcc, gfx950).") from e
    return _EXT


def available():
    try:
        ext()
        return True
    except RuntimeError:
        return False


def use_native(t):
    """True when ``t`` lives on the GPU (=> the HIP kernel must run)."""
    return t.is_cuda
