"""ctypes binding of libvdiff_hip.so (the C ABI declared in include/vdiff.h).

The library must be loaded AFTER `import torch` so its libamdhip64.so.7 /
librccl.so.1 dependencies resolve (by SONAME) to the runtime torch already
loaded — one HIP runtime, so torch's hipStream_t handles are valid here.
There is no fallback: if the library is missing every op raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

LIB_PATH = Path(__file__).resolve().parent / "libvdiff_hip.so"

c_i64, c_i32, c_f32, c_vp = C.c_int64, C.c_int32, C.c_float, C.c_void_p
VD_OK, VD_EINVAL, VD_EUNSUPPORTED, VD_ERCCL = 0, 1000, 1001, 1002  # enum vd_status

# Every exported symbol and its argtypes: the single source of truth used by the
# loader and by tests/test_abi.py (which checks it against include/vdiff.h).
SIGNATURES = {
    "vd_strerror": ([c_i32], C.c_char_p),
    "vd_version": ([], c_i32),
    "vd_build_hash": ([], C.c_char_p),
    "vd_build_arch": ([], C.c_char_p),
    "vd_gemm": ([c_vp, c_vp], c_i32),
    "vd_gemm_ws_bytes": ([c_vp], c_i64),
    "vd_gemm_plan": ([c_vp, c_vp, c_vp], c_i32),
    "vd_gn_partial": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp], c_i32),
    "vd_gn_finalize": ([c_vp, c_i64, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp], c_i32),
    "vd_gn_finalize_g": ([c_vp, c_i64, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp], c_i32),
    "vd_gn_finalize_g_ranks": ([c_vp, c_i64, c_i32, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp], c_i32),
    "vd_gn_small": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_f32, c_vp, c_vp, c_i32, c_vp, c_i64,
                     c_vp], c_i32),
    "vd_gn_apply": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_i64, c_vp], c_i32),
    "vd_gn_apply_rev3": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_i64,
                          c_i64, c_i64, c_i64, c_vp], c_i32),
    "vd_gn_partial_g": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp], c_i32),
    "vd_gn_apply_g": ([c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_i32, c_f32, c_vp, c_vp, c_i32, c_vp, c_i64, c_i64, c_vp], c_i32),
    "vd_layernorm": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_f32, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "vd_attention": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i64, c_i32, c_i64, c_f32, c_vp], c_i32),
    "vd_attention_f32": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i64, c_i32, c_i64, c_f32, c_vp], c_i32),
    "vd_attention_ex": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i64, c_i32, c_i64, c_f32,
                         c_i32, c_i32, c_vp], c_i32),
    "vd_temporal_attention": ([c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_i32, c_f32, c_vp], c_i32),
    "vd_temporal_attention_valu": ([c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_i32, c_f32, c_vp], c_i32),
    "vd_temporal_attention_kv": ([c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i64, c_i32, c_i32, c_f32, c_vp], c_i32),
    "vd_motion_qkv_attention": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_i32, c_f32,
                                 c_vp, c_f32, c_vp], c_i32),
    "vd_motion_qkv_attention_takes": ([c_i64, c_i32, c_i64, c_i32, c_i32], c_i32),
    "vd_temporal_attention_rope": ([c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_i32, c_f32, c_f32, c_vp], c_i32),
    "vd_softmax_rows": ([c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "vd_frame_metrics": ([c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp], c_i32),
    "vd_farneback_workspace": ([c_i64, c_i32, c_i32, c_i32], c_i64),
    "vd_farneback_flow": ([c_vp, c_i64, c_i32, c_i32, c_i32, C.c_double, c_i32, c_i32, c_i32, c_i32, C.c_double,
                           c_vp, c_vp, c_i64, c_vp], c_i32),
    "vd_flow_warp_workspace": ([c_i64, c_i32], c_i64),
    "vd_flow_warp_stats": ([c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp], c_i32),
    "vd_timestep_embed": ([c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp], c_i32),
    "vd_pack_latents": ([c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_f32, c_vp], c_i32),
    "vd_unpack_nhwc": ([c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp], c_i32),
    "vd_ddim_cfg_step": ([c_vp, c_i64, c_i32, c_f32, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp], c_i32),
    "vd_euler_cfg_step": ([c_vp, c_i64, c_i32, c_f32, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp], c_i32),
    "vd_step_advance": ([c_vp, c_vp], c_i32),
    "vd_block_transpose": ([c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp], c_i32),
    "vd_patchify": ([c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_f32, c_vp, c_i64, c_vp], c_i32),
    "vd_unpatchify": ([c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp], c_i32),
    "vd_rope_qk": ([c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_vp], c_i32),
    "vd_attention_fp8_quant": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp], c_i32),
    "vd_attention_fp8_quant_rope": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_i64, c_i64, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp], c_i32),
    "vd_attention_fp8": ([c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_i64, c_i32, c_f32, c_vp], c_i32),
    "vd_rows_eltwise": ([c_i32, c_vp, c_i64, c_vp, c_i64, c_i32, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "vd_upsample_nearest2x": ([c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp], c_i32),
    "vd_res_ln_mod": ([c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32, c_vp], c_i32),
}


class GemmDesc(C.Structure):
    """Mirror of vd_gemm_desc (include/vdiff.h)."""

    _fields_ = [
        ("a0", c_vp), ("lda0", c_i64), ("k0", c_i64),
        ("a1", c_vp), ("lda1", c_i64),
        ("a_mode", c_i32),
        ("n_img", c_i32), ("h_in", c_i32), ("w_in", c_i32), ("h_out", c_i32), ("w_out", c_i32),
        ("stride", c_i32), ("upsample", c_i32),
        ("w", c_vp), ("ldw", c_i64),
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("bias", c_vp),
        ("rowbias", c_vp), ("ld_rb", c_i64), ("rb_div", c_i64),
        ("res", c_vp), ("ld_res", c_i64),
        ("act", c_i32),
        ("out", c_vp), ("ldc", c_i64), ("out_f32", c_i32),
        ("ws", c_vp), ("ws_bytes", c_i64),
        ("kt", c_i32), ("ks", c_i32), ("frames_in", c_i32), ("frames_out", c_i32), ("t_off", c_i32),
        ("ln_gamma", c_vp), ("ln_beta", c_vp), ("ln_eps", c_f32),
        ("ln_pe", c_vp), ("ln_pe_div", c_i64), ("ln_pe_period", c_i64),
        ("ln_out", c_vp), ("ld_ln", c_i64),
        ("path", c_i32), ("plan_m", c_i64),
        ("rmap_n1", c_i32), ("rmap_n2", c_i32), ("rmap_inner", c_i32),
        ("ln_fold_s", c_vp), ("ln_fold_eps", c_f32),
    ]


class VdiffError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the ctypes handle; raise if the HIP build is absent."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise VdiffError(
                f"{LIB_PATH} not found: build the HIP extension first "
                "(python video-diffusion-experiments_amd/build_ext.py or __graft_entry__.build())")
        h = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
        for name, (argt, rest) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = argt
            fn.restype = rest
        _check_build_hash(h)
        _lib = h
    return _lib


def _check_build_hash(h) -> None:
    """The library must be a build of the sources in this tree (build_ext.py embeds their
    content hash): a stale or foreign .so raises instead of silently running other kernels."""
    import sys
    pkg = str(Path(__file__).resolve().parents[1])
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    import build_ext
    from ._srchash import source_files, source_hash
    if not source_files():
        return  # an installed library without its sources: nothing to compare against
    want = source_hash(build_ext.HASH_FLAGS)
    got = h.vd_build_hash().decode()
    if got != want:
        raise VdiffError(f"{LIB_PATH.name} was built from other sources (hash {got}, tree {want}): "
                         "rebuild with python video-diffusion-experiments_amd/build_ext.py")
    _check_build_arch(h.vd_build_arch().decode())


def _check_build_arch(built: str) -> None:
    """The code objects must be for the requested arch (VDIFF_ARCH, when set) and for the GPU
    this process sees: a library built for another arch would otherwise load and only fail at
    the first kernel launch ("no binary for the GPU")."""
    req = os.environ.get("VDIFF_ARCH")
    if req and req != built:
        raise VdiffError(f"{LIB_PATH.name} was built for {built}, VDIFF_ARCH={req}: rebuild")
    if torch.cuda.device_count() > 0 and torch.cuda.is_available():
        dev = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
        if dev and dev != built:
            raise VdiffError(f"{LIB_PATH.name} was built for {built}, the GPU is {dev}: rebuild with VDIFF_ARCH={dev}")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().vd_strerror(rc).decode()
        raise VdiffError(f"{what}: {msg} (code {rc})")
