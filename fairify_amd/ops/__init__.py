"""Op dispatch: hand-written HIP kernels on the GPU, PyTorch reference on the CPU.

On a ROCm device every hot op runs the in-tree HIP extension (``fairify_amd/_C*.so``, built
by ``python setup.py build_ext --inplace`` or ``__graft_entry__.build()``).  If the extension
is missing on a GPU run this module raises instead of silently falling back, so a GPU run
that reports numbers always ran the native kernels.  CPU tensors use ``ops.reference``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import reference as ref

_EXT = None
_EXT_ERR: Optional[BaseException] = None


def ext():
    """The compiled HIP extension module (raises with the build hint if absent)."""
    global _EXT, _EXT_ERR
    if _EXT is not None:
        return _EXT
    try:
        from .. import _C  # type: ignore  # noqa: F401

        _EXT = _C
        return _EXT
    except BaseException as e:  # pragma: no cover - depends on build state
        _EXT_ERR = e
        raise RuntimeError(
            "fairify_amd HIP extension (_C) is not built/importable: run "
            "`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950). "
            f"Import error: {e!r}") from e


def ext_available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


def use_hip(t: torch.Tensor) -> bool:
    """True when the tensor lives on a GPU: then the HIP path is mandatory."""
    if t.device.type != "cuda":
        return False
    if os.environ.get("FAIRIFY_FORCE_REFERENCE") == "1":
        return False
    ext()  # loud failure if missing
    return True
