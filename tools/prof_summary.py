"""Summarise a rocprofv3 kernel trace of bench.py: time per denoising step by kernel family and shape.

usage: python tools/prof_summary.py gpurun_out/prof/.../run_kernel_trace.csv

The step count is the number of ddim_cfg_kernel launches in the trace (one per step,
priming and warmup included); kernel groups launched fewer times than that (weight
init, graph-capture probes) are one-off work and are left out of the per-step table.
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    key = (n[:44], r["Grid_Size_X"], r["Workgroup_Size_X"])
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
steps = sum(len(v) for k, v in agg.items() if k[0].startswith("ddim_cfg_kernel"))
if steps == 0:
    sys.exit("no ddim_cfg_kernel launches in the trace")
per = {k: v for k, v in agg.items() if len(v) >= steps}
tot = sum(sum(v) for v in per.values()) / steps
fam = collections.defaultdict(float)
for k, v in per.items():
    fam[k[0].split("<")[0]] += sum(v) / steps
print(f"{steps} steps in the trace; per-step kernel time {tot / 1e6:.2f} ms")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:16]:
    print(f"  {v / tot * 100:5.1f}%  {v / 1e6:7.3f} ms/step  {k}")
print("top shapes (per step):")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"  {sum(v) / steps / 1e3:8.1f} us  x{len(v) / steps:5.1f}  avg {sum(v) / len(v) / 1e3:8.1f} us  "
          f"{k[0]} grid={k[1]} wg={k[2]}")
