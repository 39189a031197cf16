"""Diagnostic: what a captured fork/join costs when the side branch ends long before the main one
(round 5; tools/graph_gap_probe.py measured branches of similar length).  Per-replay time of
  serial : A -> B (main spin) -> D -> E -> F
  fork   : A -> {B main spin, C short side spin} -> (join) D -> E -> F
  late   : A -> {B, C} -> D -> E -> (join) F
(A, D, E, F tiny elementwise kernels; B 100 k cycles, C 10 k cycles of torch.cuda._sleep).  If
"late" costs what "serial" does, a join whose side branch has long finished is free, and moving a
join later (or replacing it by a device-side flag) pays."""
import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
x = torch.zeros(1 << 16, device=dev)


def tiny(v):
    x.add_(v)


def body(variant, side):
    cur = torch.cuda.current_stream()
    tiny(1.0)
    if variant == "serial":
        torch.cuda._sleep(100_000)
        tiny(2.0)
        tiny(3.0)
        tiny(4.0)
        return
    side.wait_stream(cur)
    torch.cuda._sleep(100_000)
    with torch.cuda.stream(side):
        torch.cuda._sleep(10_000)
    if variant == "fork":
        cur.wait_stream(side)
    tiny(2.0)
    tiny(3.0)
    if variant == "late":
        cur.wait_stream(side)
    tiny(4.0)


for variant in ("serial", "fork", "late", "serial", "fork", "late"):
    side = torch.cuda.Stream(device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(variant, side)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(variant, side)
    torch.cuda.synchronize()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    print(variant, f"{a.elapsed_time(b) / 50 * 1e3:.1f} us per replay", flush=True)
