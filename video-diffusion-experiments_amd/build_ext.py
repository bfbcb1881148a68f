"""Build libvdiff_hip.so in-tree for gfx950: hipcc per .hip source, then link.

Used by __graft_entry__.build() (always a clean compile) and `python build_ext.py`
(`--clean` forces one; otherwise the library is rebuilt whenever the content hash of the
sources + flags differs from the one it was built with).  The hash is compiled into the
library (vd_build_hash()) and vdiff._lib checks it against the tree at load time, so a
pushed or stale .so is never used in place of the tracked sources.
The .so links against libamdhip64.so.7 / librccl.so.1 by SONAME, so inside a process that
imported torch first it binds to torch's bundled HIP runtime (one runtime, shared streams).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
sys.path.insert(0, str(PKG))
from vdiff._srchash import CSRC, INCLUDE, source_hash  # noqa: E402

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
# the flags that enter the content hash: no absolute paths (the tree moves between machines)
# and no --offload-arch (a library built for another arch is the same sources; the arch is
# compiled in separately as vd_build_arch(), so a loader without VDIFF_ARCH set still accepts it)
HASH_FLAGS = [f for f in CFLAGS if not f.startswith("-I") and not f.startswith("--offload-arch")]


def _compile(src: Path, defs, verbose: bool) -> Path:
    obj = BUILD / (src.stem + ".o")
    cmd = [HIPCC, *CFLAGS, *defs, "-c", str(src), "-o", str(obj)]
    if verbose:
        print("[vdiff build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(verbose: bool = True, jobs: int = 8, clean: bool = False) -> Path:
    h = source_hash(HASH_FLAGS)
    stamp = BUILD / "src.hash"
    # the stamp carries the arch too: a VDIFF_ARCH change rebuilds even though the content
    # hash (arch-free, see HASH_FLAGS) is unchanged
    want = f"{h} {ARCH}"
    if not clean and LIB.exists() and stamp.exists() and stamp.read_text().strip() == want:
        if verbose:
            print(f"[vdiff build] {LIB.name} is current (source hash {h})", flush=True)
        return LIB
    shutil.rmtree(BUILD, ignore_errors=True)
    BUILD.mkdir()
    defs = [f'-DVD_BUILD_HASH="{h}"', f'-DVD_BUILD_ARCH="{ARCH}"']
    srcs = sorted(CSRC.glob("*.hip"))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, defs, verbose), srcs))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
           "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print("[vdiff build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    stamp.write_text(want + "\n")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, clean="--clean" in sys.argv[1:]))
    sys.exit(0)
