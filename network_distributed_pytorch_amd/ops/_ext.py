"""Loader for the in-tree gfx950 extension (``network_distributed_pytorch_amd._C``).

Policy: device (HIP) tensors ALWAYS go through the native kernels; if the extension is
missing on a GPU box every op raises instead of silently falling back to eager PyTorch.
CPU tensors (gloo unit tests, no GPU in the build container) take the pure-torch branches
written next to each op (``ops/__init__.py``, ``ops/conv.py``, ...; ``parallel/powersgd.py``
``_step_torch`` / ``_reduce_torch``).
"""
from __future__ import annotations

import importlib
import os

_EXT = None
_ERR: Exception | None = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return
    try:
        _EXT = importlib.import_module("network_distributed_pytorch_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def native_available() -> bool:
    _load()
    return _EXT is not None


def ext():
    """Return the extension module or raise a loud, actionable error."""
    _load()
    if _EXT is None:
        raise RuntimeError(
            "network_distributed_pytorch_amd native extension is not built "
            f"({_ERR!r}). Build it in-tree with `python setup.py build_ext --inplace` "
            "(PYTORCH_ROCM_ARCH=gfx950). Device tensors never fall back to eager PyTorch."
        )
    return _EXT


def extension_path() -> str | None:
    _load()
    return os.path.abspath(_EXT.__file__) if _EXT is not None else None
