"""Check the lane map of the block-scaled fp8 MFMA 32x32x64 with exact small-integer data."""
import ctypes
import sys
from pathlib import Path

import torch

lib = ctypes.CDLL(str(Path(__file__).with_name("mb_fp8_probe.so")))
torch.manual_seed(0)
A = torch.randint(-3, 4, (32, 64)).float()
B = torch.randint(-3, 4, (64, 32)).float()
want = A @ B
f8 = torch.float8_e4m3fn


def lanes_a(M, kmap):  # M[row][k] -> [64 lanes][32 bytes]
    out = torch.empty(64, 32)
    for l in range(64):
        for j in range(32):
            out[l, j] = M[l & 31, kmap(l, j)]
    return out


def lanes_b(M, kmap):  # M[k][col]
    out = torch.empty(64, 32)
    for l in range(64):
        for j in range(32):
            out[l, j] = M[kmap(l, j), l & 31]
    return out


def run(a, b, sa=127, sb=127):
    ad = a.to(f8).view(torch.uint8).contiguous().cuda()
    bd = b.to(f8).view(torch.uint8).contiguous().cuda()
    c = torch.zeros(64 * 16, device="cuda")
    rc = lib.fp8_probe(ctypes.c_void_p(ad.data_ptr()), ctypes.c_void_p(bd.data_ptr()),
                       ctypes.c_void_p(c.data_ptr()), sa, sb)
    assert rc == 0, rc
    c = c.cpu().view(64, 16)
    C = torch.empty(32, 32)
    for l in range(64):
        for r in range(16):
            C[(r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31] = c[l, r]
    return C


maps = {"k=32h+j": lambda l, j: 32 * (l >> 5) + j,
        "k=16(j/16)+... interleave8": lambda l, j: 16 * (j // 8) + 8 * (l >> 5) + (j % 8),
        "k=j*2+h": lambda l, j: 2 * j + (l >> 5)}
for name, km in maps.items():
    C = run(lanes_a(A, km), lanes_b(B, km))
    print(f"{name:30s} max|err| = {(C - want).abs().max().item():.3f}", flush=True)
km = maps["k=32h+j"]
C2 = run(lanes_a(A, km), lanes_b(B, km), sa=128, sb=126)
print("scales 2^1 * 2^-1:", (C2 - want).abs().max().item())
C3 = run(lanes_a(A, km), lanes_b(B, km), sa=129, sb=127)
print("scale a 2^2:", (C3 - 4 * want).abs().max().item())
