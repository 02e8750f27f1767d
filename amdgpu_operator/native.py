"""Loader for the in-tree native artefacts (``amdgpu_operator/_native``).

The native pieces are built by ``native/Makefile`` (driven by
``__graft_entry__.build()`` or ``python -m amdgpu_operator.native``).  They are
loaded with :mod:`ctypes` (plain C ABI, no torch headers), so the same shared
objects serve the Python control plane and the standalone C++ binaries that go
into the operand images.

Loading is strict: if a library is missing or fails to load this module raises
:class:`NativeUnavailable` - callers never silently fall back to a pure-Python
path on a GPU box.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import sys
import threading
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
NATIVE_DIR = PKG_DIR / "_native"
REPO_ROOT = PKG_DIR.parent
NATIVE_SRC = REPO_ROOT / "native"

_lock = threading.Lock()
_libs: dict[str, ctypes.CDLL] = {}


class NativeUnavailable(RuntimeError):
    """A required native artefact is missing or could not be loaded."""


def artefact(name: str) -> Path:
    return NATIVE_DIR / name


def binary(name: str) -> Path:
    """Path of a native executable; raises if it has not been built."""
    p = artefact(name)
    if not p.is_file() or not os.access(p, os.X_OK):
        raise NativeUnavailable(f"native binary {p} not built (run `make -C native`)")
    return p


def build(targets: list[str] | None = None, jobs: int = 8) -> None:
    """Compile the native tree in place (hipcc for gfx950, g++ for host tools)."""
    cmd = ["make", "-C", str(NATIVE_SRC), f"-j{jobs}"] + (targets or ["all"])
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeUnavailable(f"native build failed:\n{res.stdout[-4000:]}\n{res.stderr[-4000:]}")


def load(libname: str) -> ctypes.CDLL:
    """Load ``_native/<libname>`` once and cache it."""
    with _lock:
        lib = _libs.get(libname)
        if lib is not None:
            return lib
        path = artefact(libname)
        if not path.is_file():
            raise NativeUnavailable(f"native library {path} not built (run `make -C native`)")
        try:
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"failed to load {path}: {e}") from e
        _libs[libname] = lib
        return lib


def loaded_native_paths() -> list[str]:
    """In-tree .so files mapped into this process (for smoke/bench evidence)."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if str(NATIVE_DIR) in line and line.rstrip().endswith(".so"):
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out


if __name__ == "__main__":  # python -m amdgpu_operator.native [targets...]
    build(sys.argv[1:] or None)
    print("built:", sorted(p.name for p in NATIVE_DIR.iterdir() if not p.name.startswith(".")))
