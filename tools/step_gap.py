"""Host-side view of the step graph replays (the ~8 ms idle gap between consecutive step
graphs in the rocprof trace): host time inside replay(), wall per step, GPU time per step.

    python tools/step_gap.py [frames]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import DDIMScheduler, DenoiseLoop  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 16
unet = materialize_synthetic("full", device="cuda", seed=0)
unet.prepare()
lat = torch.randn((1, 4, frames, 64, 64), generator=torch.Generator().manual_seed(42)).cuda()
ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).cuda()
sched = DDIMScheduler.from_config(DDIMScheduler().config, beta_schedule="linear", steps_offset=1, clip_sample=False)
sched.set_timesteps(50)
loop = DenoiseLoop(unet, sched, lat, ehs, 7.5)
loop.prime()
g = loop.graph
print("graph captured:", g is not None, loop.graph_error)
loop.run(3)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
host = []
t0 = time.perf_counter()
ev[0].record()
for i in range(10):
    h0 = time.perf_counter()
    g.replay()
    host.append(time.perf_counter() - h0)
    ev[i + 1].record()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host ms in replay():", " ".join(f"{1e3 * h:.1f}" for h in host))
print("event ms per step  :", " ".join(f"{ev[i].elapsed_time(ev[i + 1]):.1f}" for i in range(10)))
print(f"wall {1e3 * (t2 - t0) / 10:.2f} ms/step; host loop done at {1e3 * (t1 - t0):.1f} ms")

# ---- node types of the captured step graph (hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset,
# 3 host, 4 graph, 5 empty, 6 wait event, 7 event record, ...)
import collections  # noqa: E402
import ctypes  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
loop.reset(lat)
gk = torch.cuda.CUDAGraph(keep_graph=True)
with torch.cuda.graph(gk):
    loop.step()
raw = ctypes.c_void_p(gk.raw_cuda_graph())
n = ctypes.c_size_t(0)
assert hip.hipGraphGetNodes(raw, None, ctypes.byref(n)) == 0
nodes = (ctypes.c_void_p * n.value)()
assert hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n)) == 0
types = collections.Counter()
for nd in nodes:
    t = ctypes.c_int(-1)
    hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
    types[t.value] += 1
print("graph nodes:", n.value, dict(types))
ne = ctypes.c_size_t(0)
hip.hipGraphGetEdges(raw, None, None, ctypes.byref(ne))
print("edges:", ne.value)

# ---- two steps per graph
loop.reset(lat)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    loop.step()
    loop.step()
loop.reset(lat)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
e[0].record()
for i in range(5):
    g2.replay()
    e[i + 1].record()
torch.cuda.synchronize()
print("two-step graph, event ms per 2 steps:", " ".join(f"{e[i].elapsed_time(e[i + 1]):.1f}" for i in range(5)))
