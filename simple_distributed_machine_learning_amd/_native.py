"""Loader for the in-tree native extensions (_runtime: C++ host runtime, _kernels: gfx950 HIP).

Policy: the C++ runtime is always required (it is built on CPU by ``__graft_entry__.build``).
The HIP kernel module is required whenever a CUDA (ROCm) device is used: GPU code paths call
:func:`kernels` which raises loudly instead of silently falling back to PyTorch ops.  The CPU
path (Gloo multi-process tests) uses PyTorch reference ops by design.

Stale binaries: every module carries the content-hash build key it was linked from
(``_build.source_key``). Before a module is imported its key is compared with the key the tree's
current sources call for; a mismatch (a ``.so`` built from other sources, e.g. pushed from another
checkout) triggers one in-tree rebuild, or, under ``SDML_NO_AUTOBUILD=1``, an error. The key of the
loaded module is ``loaded_key(what)``; ``smoke()`` prints it.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_rt = None
_k = None
_k_err = None


_loaded_keys = {}


class StaleModuleError(RuntimeError):
    """A built module whose embedded build key does not match the current sources."""


def check_key(so_path, want: str):
    """Raise :class:`StaleModuleError` unless the module file at ``so_path`` carries ``want``."""
    from . import _build

    got = _build.embedded_key(so_path)
    if got != want:
        raise StaleModuleError(f"sdml: {so_path} was built from other sources (build key {got}, the tree wants "
                               f"{want}); rebuild with `python -m {__package__}._build`")
    return got


def _fresh(what: str):
    """Make sure the module file for ``what`` matches the tree (rebuild once if allowed), return its key."""
    from . import _build

    want = _build.source_key(what)
    path = _build.module_path(what)
    try:
        return check_key(path, want)
    except StaleModuleError:
        if os.environ.get("SDML_NO_AUTOBUILD") == "1":
            raise
    _auto_build(what)
    return check_key(path, want)


def loaded_key(what: str):
    return _loaded_keys.get(what)


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
            _loaded_keys["runtime"] = _fresh("runtime")
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
            try:  # the module must match the tree's sources: rebuild once (CPU container / dev box) or refuse
                _loaded_keys["kernels"] = _fresh("kernels")
                importlib.invalidate_caches()
                _k = importlib.import_module(f"{__package__}._kernels")
            except Exception as e:  # noqa: BLE001
                _k_err = e
                raise RuntimeError(
                    "sdml: HIP kernel extension '_kernels' is not available "
                    f"({type(e).__name__}: {e}). Run `python -m {__package__}._build kernels`.") from e
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
