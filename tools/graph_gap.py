"""Does a hipGraph replay wait for the previous replay of the same graph?  (bench.py's step
trace shows an ~8 ms idle gap between consecutive replays of the ~760-node step graph.)

    python tools/graph_gap.py
Replays a graph of N small kernels back to back and reports, per replay, the host time spent
inside replay() and the wall time per replay; then the same with two graph instances of
the same work alternated."""
import time

import torch

N, R = 760, 12
x = torch.randn(1024, 1024, device="cuda")
w = torch.randn(1024, 1024, device="cuda")
s = torch.cuda.Stream()


def work():
    y = x
    for _ in range(N):
        y = torch.mm(y, w) * 1e-3
    return y


def capture():
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        work()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            work()
    torch.cuda.synchronize()
    return g


ga, gb = capture(), capture()
torch.cuda.synchronize()
# eager GPU time of the work
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ga.replay()
torch.cuda.synchronize()
e0.record()
ga.replay()
e1.record()
torch.cuda.synchronize()
print(f"one replay (events): {e0.elapsed_time(e1):.2f} ms for {N} kernels")
for name, seq in (("same graph", [ga] * R), ("alternating two graphs", [ga, gb] * (R // 2))):
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for g in seq:
        h0 = time.perf_counter()
        g.replay()
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:24s}: wall {1e3 * (t2 - t0) / len(seq):7.2f} ms/replay, host in replay() "
          f"{1e3 * sum(host) / len(host):7.2f} ms (first {1e3 * host[0]:.2f}, last {1e3 * host[-1]:.2f}), "
          f"host loop ends {1e3 * (t1 - t0):.1f} ms before sync {1e3 * (t2 - t0):.1f}")
