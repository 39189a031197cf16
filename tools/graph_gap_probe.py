"""Diagnostic: cross-stream fork/join latency inside a captured HIP graph (run under rocprofv3
--kernel-trace; tools/graph_gap_summary.py prints the gaps).  Each variant replays a graph
A -> {B on main, C on a side stream} -> D, where A/D are tiny kernels and B/C GPU spins.
  order   : capture the side branch first ("side") or the main branch first ("main")
  marker  : tag kernels by distinct spin lengths so the trace can be attributed"""
import sys

import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
x = torch.zeros(1 << 16, device=dev)


def tiny(v):
    x.add_(v)  # one elementwise kernel


def body(order, side, fork=True):
    cur = torch.cuda.current_stream()
    tiny(1.0)
    if not fork:
        torch.cuda._sleep(100_000)
        torch.cuda._sleep(150_000)
        tiny(2.0)
        return
    side.wait_stream(cur)
    if order == "side":
        with torch.cuda.stream(side):
            torch.cuda._sleep(150_000)
        torch.cuda._sleep(100_000)
    else:
        torch.cuda._sleep(100_000)
        with torch.cuda.stream(side):
            torch.cuda._sleep(150_000)
    cur.wait_stream(side)
    tiny(2.0)


for variant in ("serial", "main", "side"):
    side = torch.cuda.Stream(device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(variant, side, fork=variant != "serial")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(variant, side, fork=variant != "serial")
    torch.cuda.synchronize()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    print(variant, f"{a.elapsed_time(b) / 20 * 1e3:.1f} us per replay", flush=True)
    tiny(0.0)
    torch.cuda._sleep(1_000_000)  # separator in the trace
    torch.cuda.synchronize()
