"""GEMM + LayerNorm fused epilogue (ops.gemm_ln) vs GEMM then vd_layernorm, L1 shapes.

python tools/gemm_ln_bench.py  -> us per call for: plain GEMM, fused, GEMM + separate LN."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, std=1.0):
    return (torch.randn(*s, device=dev, generator=g) * std).to(torch.bfloat16)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


M, N, K = 131072, 320, 320
a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
b = torch.zeros(N, device=dev)
gm, be = torch.ones(N, device=dev), torch.zeros(N, device=dev)
pe = torch.randn(32, N, device=dev)
for res in (False, True):
    r = rnd(M, N) if res else None
    out, ln = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for kw, tag in (({}, ""), (dict(pe=pe, pe_div=4096, pe_period=16), " +pe")):
        t_plain = timeit(lambda: ops.gemm(a, w, bias=b, res=r, out=out))
        t_fused = timeit(lambda: ops.gemm_ln(a, w, gm, be, bias=b, res=r, out=out, ln_out=ln, **kw))
        t_sep = timeit(lambda: (ops.gemm(a, w, bias=b, res=r, out=out),
                                ops.layer_norm(out, gm, be, out=ln, **kw)))
        print(f"M={M} N={N} K={K} res={int(res)}{tag}: plain {t_plain:.1f} us, fused {t_fused:.1f} us, "
              f"gemm+ln {t_sep:.1f} us", flush=True)
