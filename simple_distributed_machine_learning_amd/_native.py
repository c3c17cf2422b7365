"""Loader for the in-tree native extensions (_runtime: C++ host runtime, _kernels: gfx950 HIP).

Policy: the C++ runtime is always required (it is built on CPU by ``__graft_entry__.build``).
The HIP kernel module is required whenever a CUDA (ROCm) device is used: GPU code paths call
:func:`kernels` which raises loudly instead of silently falling back to PyTorch ops.  The CPU
path (Gloo multi-process tests) uses PyTorch reference ops by design.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_rt = None
_k = None
_k_err = None


def _auto_build(what: str):
    if os.environ.get("SDML_NO_AUTOBUILD") == "1":
        return
    from . import _build

    if what == "runtime":
        _build.build_runtime(verbose=False)
    else:
        _build.build_kernels(verbose=False)


def runtime():
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            try:
                _rt = importlib.import_module(f"{__package__}._runtime")
            except ImportError:
                _auto_build("runtime")
                importlib.invalidate_caches()
                _rt = importlib.import_module(f"{__package__}._runtime")
    return _rt


def kernels():
    """Return the HIP kernel extension; raise if it cannot be loaded."""
    global _k, _k_err
    if _k is not None:
        return _k
    with _lock:
        if _k is None:
            try:
                _k = importlib.import_module(f"{__package__}._kernels")
            except ImportError as e:  # try an in-tree build once (CPU container / dev box)
                try:
                    _auto_build("kernels")
                    importlib.invalidate_caches()
                    _k = importlib.import_module(f"{__package__}._kernels")
                except Exception as e2:  # noqa: BLE001
                    _k_err = e2
                    raise RuntimeError(
                        "sdml: HIP kernel extension '_kernels' is not available "
                        f"({e}; build attempt: {e2}). Run `python -m "
                        f"{__package__}._build kernels`.") from e2
    return _k


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def use_hip(t) -> bool:
    """True when tensor ``t`` lives on a ROCm device -> the HIP kernels must be used."""
    return getattr(t, "is_cuda", False)


def apply_knobs_from_env(var: str = "SDML_KNOBS") -> dict:
    """Set kernel-variant switches (csrc/kernels/knobs.h) from ``NAME=V,NAME=V`` in the environment: the A/B
    runs of tools/ and bench.py use it; production code never reads it per launch. Returns what was set."""
    import os

    spec = os.environ.get(var, "").strip()
    out = {}
    if not spec:
        return out
    k = kernels()
    for item in spec.split(","):
        name, _, val = item.partition("=")
        k.set_knob(name.strip(), int(val))
        out[name.strip()] = int(val)
    return out
