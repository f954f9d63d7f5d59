"""Loader for the in-tree gfx950 kernel library (``_kfamd_ops.so``).

Policy (no silent fallbacks): on a machine with a visible GPU the HIP library MUST load;
if it is missing or stale it is (re)built in-tree, and if that fails the import raises.
CPU tensors are served by the explicit fp32 reference implementations in
``ops.reference`` -- those exist for CPU-only tests and numerics checks, never as a
substitute for a GPU kernel.
"""
from __future__ import annotations

import os
import threading

import torch

from . import _build

_lock = threading.Lock()
_loaded = False


def lib_path() -> str:
    return str(_build.LIB_PATH)


def load(build_if_missing: bool = True) -> bool:
    """Load the kernel library once. Returns True when ``torch.ops.kfamd`` is available."""
    global _loaded
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        path = _build.LIB_PATH
        if build_if_missing and os.environ.get("KFAMD_NO_BUILD") != "1":
            # incremental: a no-op when the stamp matches the sources.  A failed rebuild
            # raises -- loading the previous .so would silently run stale kernels.  Loading a
            # prebuilt library whose stamp may not match is only done on explicit request
            # (KFAMD_NO_BUILD=1).
            _build.build()
        if not path.exists():
            return False
        torch.ops.load_library(str(path))
        _loaded = True
        return True


def ops():
    """Return the ``torch.ops.kfamd`` namespace, loading (or failing loudly) first."""
    if not load():
        raise RuntimeError(f"kfamd HIP kernel library not found at {lib_path()}; run "
                           "`python -m service_account_auth_improvements_amd.ops._build`")
    return torch.ops.kfamd


def loaded() -> bool:
    return _loaded
