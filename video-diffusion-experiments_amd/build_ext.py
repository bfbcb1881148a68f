"""Build libvdiff_hip.so in-tree for gfx950: hipcc per .hip source, then link.

Used by __graft_entry__.build() and `python build_ext.py`.  Incremental: a
source is recompiled only when it (or a header) is newer than its object.
The .so links against libamdhip64.so.7 / librccl.so.1 by SONAME, so inside a
process that imported torch first it binds to torch's bundled HIP runtime
(one runtime, shared streams).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG / "build"
LIB = PKG / "vdiff" / "libvdiff_hip.so"
ARCH = os.environ.get("VDIFF_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-mcode-object-version=5",
    "-Wno-unused-result",
    f"-I{INCLUDE}",
]


def _headers():
    return list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))


def _needs(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, verbose: bool) -> Path:
    obj = BUILD / (src.stem + ".o")
    if _needs(obj, [src, *_headers()]):
        cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
        if verbose:
            print("[vdiff build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return obj


def build(verbose: bool = True, jobs: int = 8) -> Path:
    BUILD.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    if _needs(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs),
               "-L/opt/rocm/lib", "-lrccl"]
        if verbose:
            print("[vdiff build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
    sys.exit(0)
