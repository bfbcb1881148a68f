"""Instruction mix of a kernel's largest loop in a hipcc .s file.

usage: python tools/isa_loop.py <file.s> <kernel-name substring>
(make the .s with: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S -o x.s csrc/x.hip)
"""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split("\n")
st = next(i for i, l in enumerate(txt) if re.match(r"^_Z\w*:", l) and sys.argv[2] in l.split(":")[0])
en = next(i for i, l in enumerate(txt) if i > st and ".Lfunc_end" in l)
L = txt[st:en]
labels = {m.group(1): i for i, l in enumerate(L) if (m := re.match(r"^(\.LBB\w+):", l))}
best = None
for i, l in enumerate(L):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i and (best is None or i - labels[t] > best[1] - best[0]):
            best = (labels[t], i)
c = collections.Counter()
for b in L[best[0]:best[1] + 1]:
    b = b.strip()
    if not b or b.startswith((".", ";")) or b.endswith(":"):
        continue
    op = b.split()[0]
    if op.startswith("v_mfma"):
        c["MFMA"] += 1
    elif op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq")):
        c["trans"] += 1
    elif op.startswith("v_"):
        c["valu"] += 1
        c["  " + op] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
        c["  " + op] += 1
    elif op.startswith(("global_", "buffer_")):
        c["vmem"] += 1
    elif op.startswith("s_waitcnt"):
        c["s_waitcnt"] += 1
    elif op.startswith("s_nop"):
        c["s_nop"] += 1
    elif op.startswith("s_"):
        c["salu/branch"] += 1
print(f"largest loop: lines {best[0]}..{best[1]} of the function")
for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"  {k:32s} {v}")
