"""In-tree build of lib/liblgcnhs.so with hipcc for gfx950 (csrc/Makefile)."""
from __future__ import annotations

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB = os.path.join(PKG_DIR, "lib", "liblgcnhs.so")


def build_native(jobs: int = 8, verbose: bool = False) -> str:
    """Run ``make`` in csrc/ (incremental); returns the library path, raises on failure."""
    r = subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], capture_output=True, text=True)
    if verbose or r.returncode != 0:
        print(r.stdout[-4000:])
        print(r.stderr[-4000:])
    if r.returncode != 0:
        raise RuntimeError("hipcc build of liblgcnhs.so failed (see output above)")
    return LIB
