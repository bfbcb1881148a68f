"""Summarise a rocprofv3 kernel trace: per-kernel-shape time per denoising step.
usage: python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    key = (short[:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in agg.values())
fam = collections.defaultdict(int)
for k, v in agg.items():
    fam[k[0].split("<")[0]] += sum(v)
print(f"total {tot / 1e6:.2f} ms over trace; per step ~{tot / 1e6 / steps:.2f} ms")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:14]:
    print(f"  {v / tot * 100:5.1f}%  {v / 1e6 / steps:7.2f} ms/step  {k}")
print("top shapes:")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:28]:
    print(f"  {sum(v) / 1e6 / steps:6.2f} ms/step n={len(v):5d} avg={sum(v) / len(v) / 1e3:8.1f}us {k}")
