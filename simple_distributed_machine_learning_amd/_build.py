"""Native build driver: compiles the C++ runtime and the gfx950 HIP kernels in-tree.

No hipify, no setuptools/BuildExtension magic: every object is compiled by an explicit
``hipcc --offload-arch=gfx950`` (kernels, torch bindings) or ``g++`` (host runtime) command,
cached by a content hash of the source + flags + included headers, and linked into two
CPython extension modules that live next to this file:

* ``_runtime``  — pure C++ (pybind11): pipeline schedule generator + deadlock validator,
  counter-based synthetic-data generator (host side of the same hash the HIP kernel uses).
* ``_kernels``  — HIP/CDNA4 kernels (MFMA GEMMs with fused epilogues, fused softmax-CE,
  fused SGD, ...) plus a thin torch binding unit.  Kernel translation units do not include
  torch headers, so they compile in seconds; only ``torch_bindings.cpp`` pays the torch
  header cost, once.

The reference has no native code of its own; these modules replace the native PyTorch
subsystems it leans on (TensorPipe RPC + distributed autograd + ATen CPU kernels, see
SURVEY.md §2c).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR.parent / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
OFFLOAD_ARCH = os.environ.get("SDML_OFFLOAD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CXX = shutil.which("g++") or "g++"


def _python_include() -> str:
    return sysconfig.get_paths()["include"]


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    return [str(p) for p in inc], str(lib)


def _headers_hash(src: Path, include_dirs) -> str:
    """Hash local (quoted) includes transitively so header edits trigger rebuilds."""
    h = hashlib.sha256()
    seen = set()
    stack = [src]
    while stack:
        p = stack.pop()
        if p in seen or not p.exists():
            continue
        seen.add(p)
        text = p.read_bytes()
        h.update(_rel(str(p)).encode())
        h.update(text)
        for m in re.finditer(rb'#include\s+"([^"]+)"', text):
            name = m.group(1).decode()
            for d in [p.parent] + [Path(x) for x in include_dirs]:
                cand = d / name
                if cand.exists():
                    stack.append(cand)
                    break
    return h.hexdigest()


def _rel(text: str) -> str:
    """Make cache keys independent of where the repo is checked out (GPU boxes use another path)."""
    return text.replace(str(PKG_DIR.parent), "<root>")


def _compile(cmd_base, src: Path, include_dirs, tag: str) -> Path:
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    obj = _obj_path(cmd_base, src, include_dirs, tag)
    if obj.exists():
        return obj
    cmd = list(cmd_base) + ["-c", str(src), "-o", str(obj) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def _link(cmd, out: Path):
    tmp = out.with_name(out.name + ".tmp")
    r = subprocess.run(cmd + ["-o", str(tmp)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


def _obj_path(cmd_base, src: Path, include_dirs, tag: str) -> Path:
    key = hashlib.sha256((_rel(" ".join(cmd_base)) + _headers_hash(src, include_dirs)).encode()).hexdigest()[:16]
    return BUILD_DIR / f"{tag}_{src.stem}_{key}.o"


# ---- build key: a content hash of every object a module links, embedded in the module at link time ----------------
# The key is the hash of the sorted object names; each name already carries the hash of its compile command and of its
# source with every quoted include (``_obj_path``), so the key changes with any source, header or flag edit.
# ``_native`` computes the key the current tree WANTS (no compiler needed) and compares it with the marker string in
# the .so file before importing it, so a module built from other sources is refused (or rebuilt) instead of loaded.
KEY_MARKER = b"SDML_BUILD_KEY="


def _plan(what: str):
    """(compile command, source, include dirs, tag) of every object the module ``what`` links."""
    if what == "runtime":
        srcs = sorted((CSRC / "runtime").glob("*.cpp"))
        incs = [str(CSRC / "runtime"), str(CSRC / "common"), _pybind_include(), _python_include()]
        base = [CXX, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
        base += [f"-I{d}" for d in incs]
        return [(base, s, incs, "rt") for s in srcs]
    tinc, _ = _torch_paths()
    kdir = CSRC / "kernels"
    common = [str(kdir), str(CSRC / "common")]
    kflags = [HIPCC, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}",
              "-munsafe-fp-atomics", "-Wno-unused-result"] + [f"-I{d}" for d in common]
    # SDML_KERNEL_EXPERIMENTS=1: timing-probe switches live, env-settable knobs (csrc/kernels/knobs.h).
    # Never the build that ships: build() / the driver compile without it.
    exp = ["-DSDML_KERNEL_EXPERIMENTS"] if os.environ.get("SDML_KERNEL_EXPERIMENTS") == "1" else []
    kflags += exp
    bflags = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              "-DTORCH_EXTENSION_NAME=_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-Wno-unused-result", "-Wno-deprecated-declarations"] + exp
    binc = common + tinc + [_python_include(), "/opt/rocm/include"]
    bflags += [f"-I{d}" for d in binc]
    return ([(kflags, s, common, "k") for s in sorted(kdir.glob("*.hip"))]
            + [(bflags, s, binc, "b") for s in sorted(kdir.glob("*.cpp"))])


def source_key(what: str) -> str:
    """The build key the current sources and flags call for (``what`` = "runtime" | "kernels")."""
    names = sorted(_obj_path(*job).name for job in _plan(what))
    return hashlib.sha256("\n".join(names).encode()).hexdigest()[:24]


def embedded_key(so_path) -> str | None:
    """The key a built module carries (None: no marker, i.e. built before keys existed)."""
    try:
        data = Path(so_path).read_bytes()
    except OSError:
        return None
    i = data.find(KEY_MARKER)
    if i < 0:
        return None
    return data[i + len(KEY_MARKER):i + len(KEY_MARKER) + 24].decode("ascii", "replace")


def _key_object(what: str, key: str) -> Path:
    """A one-symbol object holding the marker string; linked into the module."""
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    obj = BUILD_DIR / f"key_{what}_{key}.o"
    if obj.exists():
        return obj
    src = BUILD_DIR / f"key_{what}_{key}.c"
    src.write_text('__attribute__((used, visibility("default"))) const char sdml_build_key[] = "'
                   + KEY_MARKER.decode() + key + '";\n')
    r = subprocess.run(["gcc", "-fPIC", "-c", str(src), "-o", str(obj) + ".tmp"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: build key object\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def module_path(what: str) -> Path:
    return PKG_DIR / f"_{what}{EXT_SUFFIX}"


def build_runtime(verbose: bool = False) -> Path:
    jobs = _plan("runtime")
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(lambda j: _compile(*j), jobs))
    objs.append(_key_object("runtime", source_key("runtime")))
    out = module_path("runtime")
    if _needs_link(out, objs):
        _link([CXX, "-shared", "-fPIC"] + [str(o) for o in objs], out)
        _write_stamp(out, objs)
        if verbose:
            print(f"[sdml build] linked {out.name}")
    return out


def build_kernels(verbose: bool = False) -> Path:
    _, tlib = _torch_paths()
    jobs = _plan("kernels")
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(lambda j: _compile(*j), jobs))
    objs.append(_key_object("kernels", source_key("kernels")))
    out = module_path("kernels")
    if _needs_link(out, objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}"] + [str(o) for o in objs]
        link += [f"-L{tlib}", f"-Wl,-rpath,{tlib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
                 "-lc10_hip", "-ltorch_hip", "-L/opt/rocm/lib", "-lamdhip64"]
        _link(link, out)
        _write_stamp(out, objs)
        if verbose:
            print(f"[sdml build] linked {out.name}")
    return out


def _needs_link(out: Path, objs) -> bool:
    stamp = out.with_name(out.name + ".objs")
    want = "\n".join(sorted(o.name for o in objs))
    return not (out.exists() and stamp.exists() and stamp.read_text() == want)


def _write_stamp(out: Path, objs):
    out.with_name(out.name + ".objs").write_text("\n".join(sorted(o.name for o in objs)))


def build_all(verbose: bool = True):
    rt = build_runtime(verbose)
    k = build_kernels(verbose)
    return rt, k


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "runtime"):
        print(build_runtime(True))
    if what in ("all", "kernels"):
        print(build_kernels(True))
