"""The C-ABI boundary (CPU): include/vdiff.h <-> libvdiff_hip.so <-> ctypes."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest
import torch

import vdiff._lib as L
from vdiff import ops

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "vdiff.h"


def header_functions():
    txt = HEADER.read_text()
    return set(re.findall(r"^\s*(?:const\s+char\s*\*|int|int64_t)\s+(vd_\w+)\s*\(", txt, re.M))


def test_header_declares_exactly_the_bound_symbols():
    assert header_functions() == set(L.SIGNATURES)


def test_library_loads_and_exports_every_symbol():
    h = L.lib()
    for name in header_functions():
        assert hasattr(h, name), name
    assert h.vd_version() == 6
    from vdiff._srchash import source_hash
    import build_ext
    assert h.vd_build_hash().decode() == source_hash(build_ext.HASH_FLAGS)  # a build of THIS tree
    assert h.vd_build_arch().decode() == build_ext.ARCH
    assert not any(f.startswith("--offload-arch") for f in build_ext.HASH_FLAGS)  # arch-independent hash
    assert h.vd_strerror(1000).decode().startswith("vdiff: invalid argument")
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (vd_\w+)", out))
    assert header_functions() <= exported


def test_argument_counts_match_header():
    txt = HEADER.read_text()
    for name, (argt, _) in L.SIGNATURES.items():
        m = re.search(rf"{name}\s*\(([^;]*?)\);", txt, re.S)
        assert m, name
        params = m.group(1).strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert n == len(argt), (name, n, len(argt))


def test_gemm_desc_layout_matches_c(tmp_path):
    fields = [f for f, _ in L.GemmDesc._fields_]
    src = tmp_path / "probe.c"
    body = "".join(f'printf("{f} %zu\\n", offsetof(vd_gemm_desc, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "vdiff.h"\n'
                   f'int main(void){{ {body} printf("size %zu\\n", sizeof(vd_gemm_desc)); return 0; }}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n") if line)
    for f in fields:
        assert int(got[f]) == getattr(L.GemmDesc, f).offset, f
    assert int(got["size"]) == ctypes.sizeof(L.GemmDesc)


def test_ops_refuse_cpu_tensors():
    a = torch.zeros(16, 64, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.gemm(a, w)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.layer_norm(a, torch.ones(64), torch.zeros(64))


def test_error_path_raises_with_message():
    with pytest.raises(L.VdiffError, match="invalid argument"):
        L.check(1000, "probe")


def test_gemm_workspace_policy():
    """Split-K is requested only when the output tiles cannot fill the chip."""
    big = L.GemmDesc(M=131072, N=320, K=2880, k0=2880, lda0=2880, ldw=2880, a_mode=0)
    assert L.lib().vd_gemm_ws_bytes(ctypes.byref(big)) == 0
    small = L.GemmDesc(M=2048, N=1280, K=11520, k0=11520, lda0=11520, ldw=11520, a_mode=0)
    nbytes = L.lib().vd_gemm_ws_bytes(ctypes.byref(small))
    assert nbytes > 0 and nbytes % (2048 * 1280 * 4) == 0


def test_dit_entry_points_validate_before_launch():
    """The DiT / fp8 entry points (§8f rank 3) reject bad arguments with VD_EINVAL before any
    launch (null operands, unsupported head width, unaligned shapes) — no GPU needed."""
    h = L.lib()
    assert h.vd_patchify(None, 1, 4, 4, 16, 16, 2, 1, 1.0, None, 16, None) == 1000
    assert h.vd_unpatchify(None, 16, 4, 16, 16, 2, 4, None, None) == 1000
    assert h.vd_rope_qk(None, 384, 64, 256, 64, 0, 4, 8, 8, 10000.0, None) == 1000
    assert h.vd_res_ln_mod(None, 128, None, 0, None, None, None, 0, 64, None, 0, None, 128, 64, 128, 1e-6,
                           None) == 1000
    assert h.vd_attention_fp8(None, None, 64, None, None, None, None, None, 64, 1, 1, 64, 64, 64, 0.125,
                              None) == 1000
    buf = ctypes.create_string_buffer(64)
    p = ctypes.addressof(buf)
    # d = 80 is not an fp8 kernel variant; skv must be a multiple of 64
    assert h.vd_attention_fp8(p, p, 64, p, p, p, p, p, 64, 1, 1, 64, 64, 80, 0.1, None) == 1000
    assert h.vd_attention_fp8_quant(p, 64, p, 64, p, 64, 1, 1, 64, 70, 64, p, p, 64, p, p, p, p, 1.0, None) == 1000
    # fused temporal RoPE: 17..32 frames and d = 64 only
    assert h.vd_temporal_attention_rope(p, p, p, 192, p, 192, 1, 16, 4, 3, 64, 0.125, 10000.0, None) == 1000
    assert h.vd_temporal_attention_rope(p, p, p, 120, p, 120, 1, 32, 4, 3, 40, 0.125, 10000.0, None) == 1000
    # fused RoPE quantization: s must equal Hp*Wp; null operands
    assert h.vd_attention_fp8_quant_rope(p, 64, p, 64, p, 64, 1, 1, 64, 64, 8, 9, 10000.0, p, p, 64, p, p, p, p,
                                         1.0, None) == 1000
    assert h.vd_attention_fp8_quant_rope(None, 64, None, 64, None, 64, 1, 1, 64, 64, 8, 8, 10000.0, None, None,
                                         64, None, None, None, None, 1.0, None) == 1000


def test_dit_ops_refuse_cpu_tensors():
    x = torch.zeros(64, 128, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.res_ln_mod(x)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.patchify(torch.zeros(1, 4, 2, 8, 8), 2, 16)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.attention_fp8(x, x, x, 1, 2, 64, 64)


def test_loader_refuses_a_library_built_from_other_sources(monkeypatch):
    """a pushed/stale .so must not stand in for the tracked sources."""
    import vdiff._srchash as sh
    h = L.lib()
    monkeypatch.setattr(sh, "source_hash", lambda flags=(): "0000000000000000")
    with pytest.raises(L.VdiffError, match="built from other sources"):
        L._check_build_hash(h)


def test_loader_refuses_a_library_built_for_another_arch(monkeypatch):
    """the content hash is arch-free, so the arch is checked on its own — a VDIFF_ARCH
    that differs from the library's vd_build_arch() raises at load, and build() rebuilds when the
    arch in its stamp changes."""
    import build_ext
    h = L.lib()
    monkeypatch.setenv("VDIFF_ARCH", "gfx942")
    with pytest.raises(L.VdiffError, match="built for gfx950"):
        L._check_build_hash(h)
    monkeypatch.setenv("VDIFF_ARCH", "gfx950")
    L._check_build_hash(h)
    if (build_ext.BUILD / "src.hash").exists():  # the build directory is not shipped to GPU boxes
        assert (build_ext.BUILD / "src.hash").read_text().split()[1] == build_ext.ARCH


def test_product_library_has_no_selector_state():
    """VERDICT r3 #6 / SURVEY §8b "stateless and reentrant": the product library exports no
    mutable selector — no vd_*select* / *force* entry points, no exported data symbols beyond
    the HIP runtime's per-module ids — and every variant choice a test needs is a per-call
    argument (vd_gemm_desc.path / plan_m, vd_attention_ex's kernel, vd_temporal_attention_valu)."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], capture_output=True, text=True).stdout
    syms = [line.split() for line in out.splitlines() if len(line.split()) == 3]
    exported_fns = {name for _, kind, name in syms if kind == "T" and name.startswith("vd_")}
    assert exported_fns == header_functions()
    assert not any(("select" in n or "force" in n or "stamps" in n) for n in exported_fns)
    data = [name for _, kind, name in syms if kind in "BDGRSV" and not name.startswith("__hip_cuid_")]
    assert data == [], data
    fields = [f for f, _ in L.GemmDesc._fields_]
    assert fields[-7:] == ["path", "plan_m", "rmap_n1", "rmap_n2", "rmap_inner", "ln_fold_s", "ln_fold_eps"]
