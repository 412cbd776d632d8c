"""Loader for the in-tree native core (``_dbfs_native*.so``).

The extension is built in-tree by ``make`` (see ``__graft_entry__.build``) and
is never silently replaced by a Python fallback: importing this module raises
if the shared object is missing or fails to load.
"""
from __future__ import annotations

import glob
import importlib
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_PKG_DIR)


def native_path() -> str | None:
    hits = sorted(glob.glob(os.path.join(_PKG_DIR, "_dbfs_native*.so")))
    return hits[0] if hits else None


def build(jobs: int = 8, quiet: bool = True) -> None:
    """Compile the HIP/C++ core for gfx950 in-tree (bin/bfs + the Python module)."""
    import subprocess

    cmd = ["make", "-C", _REPO, f"-j{jobs}"]
    out = subprocess.run(cmd, capture_output=quiet, text=True)
    if out.returncode != 0:
        raise RuntimeError("native build failed:\n" + (out.stdout or "") + (out.stderr or ""))


def load():
    if native_path() is None:
        raise ImportError(
            "distributed_cuda_bfs_amd native core is not built: run `make -j8` in "
            f"{_REPO} (or __graft_entry__.build())")
    return importlib.import_module("distributed_cuda_bfs_amd._dbfs_native")


N = load()
