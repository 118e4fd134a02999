"""Loader for the in-tree native extension ``bcfl/_C*.so`` (HIP/CDNA4 kernels + bindings).

Policy: a CUDA(HIP) tensor reaching a bcfl op REQUIRES the native extension — there is no
silent eager fallback on the GPU path. CPU tensors use the PyTorch reference implementations in
:mod:`bcfl.ops.ref` (the same math; used by the CPU test-suite and as numerics oracles).
``BCFL_FORCE_TORCH=1`` routes GPU tensors to the reference path too (A/B benchmarking only).
"""
from __future__ import annotations

import glob
import importlib
import os
import sys

_C = None
_ERR = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    pkg_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cands = glob.glob(os.path.join(pkg_dir, "_C*.so"))
    if not cands:
        _ERR = "bcfl/_C*.so not found (build it: python -m bcfl.csrc.build)"
        return None
    try:
        import torch  # noqa: F401  (loads libtorch / libamdhip64 first)
        _C = importlib.import_module("bcfl._C")
    except Exception as e:  # pragma: no cover - depends on the build
        _ERR = f"failed to import bcfl._C: {e!r}"
        _C = None
    return _C


_SC = None   # bcfl.utils.streamcheck, bound on first use (import cycle: utils imports ops)


def native():
    """Return the extension module or raise (GPU path must never silently fall back)."""
    global _SC
    m = _C if _C is not None else _load()
    if m is None:
        raise RuntimeError("bcfl native extension unavailable on a GPU code path: " + str(_ERR))
    sc = _SC
    if sc is None:
        from ..utils import streamcheck as sc
        _SC = sc
    if "det" in sc._STATE:   # BCFL_DEBUG_STREAMS: every kernel call reported to the checker
        return sc.wrap_native(m)
    return m


def available() -> bool:
    return _load() is not None


# The routing switches are read once per process (every op consults them: an os.environ lookup
# per call was ~0.5 ms of host time per BERT-base step); code that changes them at run time
# (tests, A/B drivers) calls refresh_env() afterwards.
_FORCE = False
_TORCH_OPS: frozenset = frozenset()


def refresh_env() -> None:
    global _FORCE, _TORCH_OPS
    _FORCE = os.environ.get("BCFL_FORCE_TORCH", "0") == "1"
    _TORCH_OPS = frozenset(filter(None, os.environ.get("BCFL_TORCH_OPS", "").split(",")))


refresh_env()


def force_torch() -> bool:
    return _FORCE


def _torch_ops():
    return _TORCH_OPS


def use_native(t, op: str = "") -> bool:
    """True when tensor ``t`` must go through the HIP kernels. ``BCFL_TORCH_OPS=attn,rope,...``
    routes the named ops to the reference path on GPU (bisection / A-B benchmarking only)."""
    if _FORCE or not getattr(t, "is_cuda", False):
        return False
    return not (op and op in _TORCH_OPS)


def load_error():
    _load()
    return _ERR
