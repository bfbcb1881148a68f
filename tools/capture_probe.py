"""Which collective + stream patterns survive hipGraph capture with RCCL (world size 1)?
    python tools/capture_probe.py <variant>
  single_side : all_to_all_single on a side stream forked/joined by events
  list_main   : list all_to_all on the capturing stream
  list_side   : list all_to_all on a side stream
  compute_side: all_to_all_single on the capturing stream, independent compute on a side
                stream forked/joined by events (the roles swapped)
  single_async: all_to_all_single(async_op=True) issued on the capturing stream, waited later
                (the collective runs on the process group's own stream meanwhile)"""
import os
import socket
import sys

import torch
import torch.distributed as dist

s = socket.socket()
s.bind(("127.0.0.1", 0))
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
s.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
variant = sys.argv[1]
x = torch.randn(4096, 320, device="cuda")
y = torch.empty_like(x)
side = torch.cuda.Stream()


def body():
    main = torch.cuda.current_stream()
    z = x * 2
    if variant == "list_main":
        dist.all_to_all([y], [z])
        return y + 1
    if variant == "compute_side":
        side.wait_stream(main)
        with torch.cuda.stream(side):
            u = z * 3
            ev = torch.cuda.Event()
            ev.record(side)
        dist.all_to_all_single(y, z)
        main.wait_event(ev)
        return y + 1 + u * 0
    if variant == "single_async":
        work = dist.all_to_all_single(y, z, async_op=True)
        u = z * 3  # independent work while the collective runs
        work.wait()
        return y + 1 + u * 0
    side.wait_stream(main)
    with torch.cuda.stream(side):
        if variant == "single_side":
            dist.all_to_all_single(y, z)
        else:
            dist.all_to_all([y], [z])
        ev = torch.cuda.Event()
        ev.record(side)
    main.wait_event(ev)
    w = y + 1
    main.wait_stream(side)
    return w


body()
torch.cuda.synchronize()
print(variant, 'eager ok', flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = body()
print(variant, 'capture ok', flush=True)
g.replay()
torch.cuda.synchronize()
print(variant, "captured and replayed; correct:", torch.allclose(out, x * 2 + 1))
dist.destroy_process_group()
