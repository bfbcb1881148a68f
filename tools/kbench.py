"""Kernel microbenchmark over the UNet's real shapes (full config, 1 GPU).

python tools/kbench.py [filter]  -> one line per shape: us, TFLOP/s, effective GB/s
"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

flt = sys.argv[1] if len(sys.argv) > 1 else ""
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


def report(name, us, flop, byts):
    print(f"{name:58s} {us:9.1f} us {flop / us / 1e6:8.1f} TF/s {byts / us / 1e3:8.1f} GB/s", flush=True)


IMGS = int(__import__("os").environ.get("KB_IMGS", "32"))  # images per call (32 = 16 frames x CFG 2)
cases = []
# dense GEMMs (M, N, K, extra)
for lvl, (hw, C) in enumerate([(4096, 320), (1024, 640), (256, 1280), (64, 1280)]):
    M = IMGS * hw
    cases += [(f"L{lvl+1} dense proj   M={M} N={C} K={C} +res", "dense", M, C, C, True),
              (f"L{lvl+1} dense proj   M={M} N={C} K={C} nores", "dense", M, C, C, False),
              (f"L{lvl+1} dense qkv    M={M} N={3*C} K={C}", "dense", M, 3 * C, C, False),
              (f"L{lvl+1} dense ff2    M={M} N={C} K={4*C} +res", "dense", M, C, 4 * C, True),
              (f"L{lvl+1} geglu        M={M} N={8*C} K={C}", "geglu", M, 8 * C, C, False)]
cases += [("big 4096^3", "dense", 4096, 4096, 4096, False), ("big 8192^3", "dense", 8192, 8192, 8192, False),
          ("big M=32768 N=4096 K=1280", "dense", 32768, 4096, 1280, False)]
convs = [("L1 conv 320->320", IMGS, 64, 320, 320), ("L2 conv 640->640", IMGS, 32, 640, 640),
         ("L3 conv 1280->1280", IMGS, 16, 1280, 1280), ("L4 conv 1280->1280", IMGS, 8, 1280, 1280),
         ("L4 conv 2560->1280", IMGS, 8, 2560, 1280), ("L1 conv 640->320", IMGS, 64, 640, 320),
         ("L1 conv_out 320->4", IMGS, 64, 320, 4)]

for name, kind, M, N, K, res in cases:
    if flt not in name:
        continue
    a = rnd(M, K)
    w = rnd(N, K, std=K ** -0.5)
    b = torch.zeros(N, device=dev)
    r = rnd(M, N) if res else None
    for path in __import__("os").environ.get("KB_PATHS", "v2,v1").split(","):
        if path == "torch":  # vendor comparator: hipBLASLt through F.linear (no epilogue fusion)
            us = timeit(lambda: torch.nn.functional.linear(a, w))
            report(f"{name} [hipblaslt]", us, 2.0 * M * N * K, 2 * (M * K + N * K + M * N))
            continue
        ops._PLAN.path = {"auto": 0, "v1": 1, "v2": 2, "v3": 3, "v5": 5, "v6": 6, "v8": 8}[path]  # per-call vd_gemm_desc.path
        act = ops.ACT_GEGLU if kind == "geglu" else ops.ACT_NONE
        nout = N // 2 if kind == "geglu" else N
        out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.gemm(a, w, bias=b, res=r, act=act, out=out))
        byts = 2 * (M * K + N * K + M * nout + (M * N if res else 0))
        report(f"{name} [{path}]", us, 2.0 * M * N * K, byts)
    ops._PLAN.path = 0  # per-call vd_gemm_desc.path

for name, n, hw, ci, co in convs:
    if flt not in name:
        continue
    x = rnd(n * hw * hw, ci)
    w = rnd(co, 9 * ci, std=(9 * ci) ** -0.5)
    out = torch.empty(n * hw * hw, co, device=dev, dtype=torch.bfloat16)
    for path in __import__("os").environ.get("KB_PATHS", "v2,v1").split(","):
        if path == "torch":  # vendor comparator: MIOpen NCHW-channels_last conv
            xc = x.view(n, hw, hw, ci).permute(0, 3, 1, 2)
            wc = w.view(co, 3, 3, ci).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            us = timeit(lambda: torch.nn.functional.conv2d(xc, wc, padding=1))
            report(f"{name} M={n*hw*hw} K={9*ci} [miopen]", us, 2.0 * n * hw * hw * co * 9 * ci,
                   2 * (n * hw * hw * (ci + co) + co * 9 * ci))
            continue
        ops._PLAN.path = {"auto": 0, "v1": 1, "v2": 2, "v3": 3, "v5": 5, "v6": 6, "v8": 8}[path]  # per-call vd_gemm_desc.path
        us = timeit(lambda: ops.conv3x3(x, n, hw, hw, w, out=out))
        report(f"{name} M={n*hw*hw} K={9*ci} [{path}]", us, 2.0 * n * hw * hw * co * 9 * ci,
               2 * (n * hw * hw * (ci + co) + co * 9 * ci))
    ops._PLAN.path = 0  # per-call vd_gemm_desc.path

for name, n_img, S, d, skv in [("attn L1 self", 32, 4096, 40, 4096), ("attn L2 self", 32, 1024, 80, 1024),
                               ("attn L3 self", 32, 256, 160, 256), ("attn L1 cross", 32, 4096, 40, 77),
                               ("attn L1 model", 32, 4096, 40, 4096)]:
    if flt not in name:
        continue
    C = 8 * d
    qkv = rnd(n_img * S, 3 * C, std=1.5)
    if "model" in name:  # bench.py's roofline inputs: softmax scale d^-1/2 log2 e folded into q
        qkv[:, :C] = (qkv[:, :C].float() * (d ** -0.5 * math.log2(math.e))).to(torch.bfloat16)
    kv = rnd(2 * skv, 2 * C, std=1.5)
    out = torch.empty(n_img * S, C, device=dev, dtype=torch.bfloat16)
    if skv == S:
        fn = lambda: ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], n_img, 8, S, S, d, out=out)
    else:
        fn = lambda: ops.attention(qkv[:, :C], kv[:, :C], kv[:, C:], n_img, 8, S, skv, d, kv_div=16, out=out)
    us = timeit(fn)
    report(f"{name} S={S} d={d} skv={skv}", us, 4.0 * n_img * 8 * S * skv * d, 2 * n_img * S * C * 4)
    if skv == S:  # the model path: softmax scale folded into the Q projection (c == 1)
        us = timeit(lambda: ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], n_img, 8, S, S, d, out=out,
                                          scale=1.0 / math.log2(math.e)))
        report(f"{name} S={S} d={d} skv={skv} [unit c]", us, 4.0 * n_img * 8 * S * skv * d, 2 * n_img * S * C * 4)
    if "torch" in __import__("os").environ.get("KB_PATHS", ""):  # vendor comparator: SDPA
        q4 = qkv[:, :C].reshape(n_img, S, 8, d).transpose(1, 2)
        src = qkv if skv == S else kv
        k4 = src[: n_img * skv if skv == S else skv, C:2 * C].reshape(-1, skv, 8, d).transpose(1, 2)
        v4 = (qkv[:, 2 * C:] if skv == S else kv[:skv, C:]).reshape(-1, skv, 8, d).transpose(1, 2)
        if skv != S:
            k4, v4 = k4.expand(n_img, -1, -1, -1), v4.expand(n_img, -1, -1, -1)
        try:
            us = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q4, k4, v4))
            report(f"{name} S={S} d={d} skv={skv} [sdpa]", us, 4.0 * n_img * 8 * S * skv * d, 2 * n_img * S * C * 4)
        except Exception as e:  # noqa: BLE001
            print(f"{name} [sdpa] failed: {e}")

for name, hw, d in [("temporal L1", 4096, 40), ("temporal L2", 1024, 80), ("temporal L3", 256, 160)]:
    if flt not in name:
        continue
    C, F_, B = 8 * d, 16, 2
    qkv = rnd(B * F_ * hw, 3 * C, std=1.5)
    out = torch.empty(B * F_ * hw, C, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, F_, hw, 8, d, out=out))
    report(f"{name} F=16 pos={hw} d={d}", us, 4.0 * B * hw * 8 * F_ * F_ * d, 2 * B * F_ * hw * C * 4)

for name, n_inst, pix, C, groups in [("gn L1 image", 32, 4096, 320, 32), ("gn L1 motion", 2, 65536, 320, 32),
                                     ("gn L2 image", 32, 1024, 640, 32), ("gn L3 image", 32, 256, 1280, 32)]:
    if flt not in name:
        continue
    x = rnd(n_inst * pix, C)
    gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    us = timeit(lambda: ops.group_norm(x, n_inst, pix, groups, 1e-6, gam, bet, silu=True))
    report(f"{name} inst={n_inst} pix={pix} C={C}", us, 0, 2 * 2 * n_inst * pix * C + 2 * n_inst * pix * C)

for name, rows, C in [("ln L1", 131072, 320), ("ln L2", 32768, 640), ("ln L3", 8192, 1280)]:
    if flt not in name:
        continue
    x = rnd(rows, C)
    gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    out = torch.empty_like(x)
    us = timeit(lambda: ops.layer_norm(x, gam, bet, out=out))
    report(f"{name} rows={rows} C={C}", us, 0, 2 * 2 * rows * C)
