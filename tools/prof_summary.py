"""Summarise a rocprofv3 kernel trace of bench.py: time per denoising step by kernel family and shape.

usage: python tools/prof_summary.py gpurun_out/prof/.../run_kernel_trace.csv

Only the steady-state steps are counted: the window runs from the end of the 3rd
ddim_cfg_kernel launch (one per step; priming, weight init and graph capture come
before it) to the end of the last one, and everything launched inside it is divided
by the number of steps it spans.  The bench's own roofline timing of the attention
kernel runs after the last step and falls outside the window.
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ddim = [r for r in rows if "ddim_cfg_kernel" in r["Kernel_Name"]]
if len(ddim) < 5:
    sys.exit("fewer than 5 ddim_cfg_kernel launches in the trace")
t0, t1 = int(ddim[2]["End_Timestamp"]), int(ddim[-1]["End_Timestamp"])
steps = len(ddim) - 3
win = [r for r in rows if t0 < int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= t1]
agg = collections.defaultdict(list)
for r in win:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    key = (n[:44], r["Grid_Size_X"], r["Workgroup_Size_X"])
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
busy = sum(sum(v) for v in agg.values()) / steps
fam = collections.defaultdict(float)
for k, v in agg.items():
    fam[k[0].split("<")[0]] += sum(v) / steps
print(f"{steps} steady-state steps; wall {(t1 - t0) / steps / 1e6:.2f} ms/step, kernel-busy {busy / 1e6:.2f} ms/step, "
      f"{len(win) / steps:.0f} launches/step")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:20]:
    print(f"  {v / busy * 100:5.1f}%  {v / 1e6:7.3f} ms/step  {k}")
print("top shapes (per step):")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"  {sum(v) / steps / 1e3:9.1f} us  x{len(v) / steps:5.1f}  avg {sum(v) / len(v) / 1e3:8.1f} us  "
          f"{k[0]} grid={k[1]} wg={k[2]}")

# the same kernel inside the step (the L1 spatial self-attention: flash40<unit-c>; before round 3
# flash32<40, unit-c> launches longer than 300 us, the shorter ones being its text cross-attention)
ROOF = "flash40_kernel<true>" if any("flash40_kernel<true>" in r["Kernel_Name"] for r in rows) else "flash40_kernel<true,"
ins = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win if ROOF in r["Kernel_Name"]]
ins = [x for x in ins if x > 300e3]
if ins:
    print(f"roofline kernel inside the step (L1 self-attention): {len(ins)} launches, avg {sum(ins) / len(ins) / 1e3:.1f} us"
          f" (min {min(ins) / 1e3:.1f}, max {max(ins) / 1e3:.1f})")

# bench.py's roofline kernel: after the last step, time_attention() launches the L1
# self-attention kernel (10 warm-up + attn_reps timed) on its own, first on model-scale inputs
# (the bench line's roofline.avg_launch_ms), then on the stress inputs (roofline.stress);
# those launches close the trace and their averages must agree with the bench line.
after = [r for r in rows if int(r["Start_Timestamp"]) > t1 and ROOF in r["Kernel_Name"]]
FIXK = "flash32_kernel<40, true, true, 2>"  # flash40's exact fix-up (round 4 template order: D, UNITC, FIX, QB)
fixk = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
        if int(r["Start_Timestamp"]) > t1 and FIXK in r["Kernel_Name"]]
if fixk:
    print(f"exact fix-up launches after the step loop ({FIXK}): {len(fixk)}, "
          f"avg {sum(fixk) / len(fixk) / 1e3:.1f} us")
# after the step loop: the operand-capture forward (5 level-1 self-attention launches), then three
# timed sets of WARM + reps launches each: the step's own operands (the bench line's roofline),
# the synthetic N(0, 1.5^2) inputs (roofline.synthetic) and the stress inputs (roofline.stress)
WARM = 10  # bench.py WARM_ATTN
cap = 5 if len(after) >= 5 and (len(after) - 5) % 3 == 0 else 0
per = (len(after) - cap) // 3
sets = [after[cap + i * per: cap + (i + 1) * per] for i in range(3)] if per > WARM else [after]
for tag, part in zip(("the step's own operands = the bench line", "synthetic inputs", "stress inputs"), sets):
    if len(part) <= WARM:
        continue
    timed = part[WARM:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    print(f"roofline kernel (bench time_attention, {tag}): {len(d)} timed launches of "
          f"{timed[0]['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:60]} "
          f"grid={timed[0]['Grid_Size_X']}, avg {sum(d) / len(d) / 1e3:.1f} us "
          + (f"(first 5 {sum(d[:5]) / 5e3:.1f}, last 5 {sum(d[-5:]) / 5e3:.1f} us)" if len(d) >= 10 else ""))
