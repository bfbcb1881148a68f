"""Content hash of the HIP sources libvdiff_hip.so is built from (no torch import).

build_ext.py compiles it into the library (vd_build_hash()); vdiff._lib recomputes it
from the tree at load time and refuses a library built from other sources, so a stale
or foreign .so can never stand in for the tracked kernels.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]          # video-diffusion-experiments_amd/
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"


def source_files():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")))


def source_hash(flags=()) -> str:
    """sha256 over (file name, bytes) of every source and header, plus the compile flags;
    the first 16 hex digits."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    h.update("\0".join(flags).encode())
    return h.hexdigest()[:16]
