"""Summarise tools/mfma_busy.sh: per kernel family, dispatch-weighted MFMA-busy share
= sum SQ_VALU_MFMA_BUSY_CYCLES / sum (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).
usage: python tools/mfma_busy.py <pmc dir> [out.json]  (the JSON holds the L1 spatial
self-attention's share — flash40_kernel<true> dispatches (round 3; flash32_kernel<40, true> longer
than 300 us before it) — which
bench.py reports as roofline.mfma_busy)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import roof_src_hash  # noqa: E402

SETUP = ("at::native", "__amd_rocclr")  # weight init / copies outside the denoising step
disp = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        disp[(f, r["Dispatch_Id"])].update({"k": r["Kernel_Name"], r["Counter_Name"]: float(r["Counter_Value"])})
busy, act, n = collections.Counter(), collections.Counter(), collections.Counter()
for d in disp.values():
    if "GRBM_GUI_ACTIVE" not in d or "SQ_VALU_MFMA_BUSY_CYCLES" not in d:
        continue
    k = d["k"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    fam = k.split("<")[0]
    if k.startswith("flash40_kernel<true"):
        fam = "flash40<unit-c> L1 self-attn"
    elif k.startswith("flash32_kernel<40, true"):
        # > 300 us at ~2.4 GHz x 8 XCDs: the L1 self-attention; shorter ones are cross-attention
        fam = "flash32<40,unit-c> L1 self-attn" if d["GRBM_GUI_ACTIVE"] > 8 * 2.4e9 * 300e-6 else "flash32<40,unit-c> cross-attn"
    busy[fam] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
    act[fam] += d["GRBM_GUI_ACTIVE"]
    n[fam] += 1
share = lambda f: busy[f] / (1024 * act[f] / 8)  # noqa: E731
step = [f for f in act if not f.startswith(SETUP)]
ta = sum(act[f] for f in step)
print("MFMA-busy share = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8), PMC over a bench.py run")
print(f"{'kernel family':36s} {'dispatches':>10s} {'time share':>10s} {'MFMA busy':>10s}")
for f in sorted(step, key=lambda f: -act[f]):
    print(f"{f:36s} {n[f]:10d} {act[f] / ta * 100:9.1f}% {share(f) * 100:9.1f}%")
print(f"{'ALL (model kernels)':36s} {sum(n[f] for f in step):10d} {100.0:9.1f}% "
      f"{sum(busy[f] for f in step) / (1024 * ta / 8) * 100:9.1f}%")
key = "flash40<unit-c> L1 self-attn" if act["flash40<unit-c> L1 self-attn"] else "flash32<40,unit-c> L1 self-attn"
if len(sys.argv) > 2 and act[key]:
    json.dump({"kernel": ("flash40_kernel<true>" if key.startswith("flash40") else "flash32_kernel<40, true>") +
               " (L1 spatial self-attention)", "mfma_busy_frac": round(share(key), 4),
               "dispatches": n[key], "counters": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)",
               "kernel_src_hash": roof_src_hash()},
              open(sys.argv[2], "w"), indent=1)
