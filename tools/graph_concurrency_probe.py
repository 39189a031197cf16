"""Diagnostic: do independent branches of a captured HIP graph run concurrently on this runtime?
Two GPU spins captured on two streams (fork/join) vs one stream; prints replay times."""
import torch

dev = torch.device("cuda:0")
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
cycles = 2_000_000  # ~0.8 ms spin


def body(two):
    if two:
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda._sleep(cycles)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cycles)
        torch.cuda.current_stream().wait_stream(side)
    else:
        torch.cuda._sleep(cycles)
        torch.cuda._sleep(cycles)


for two in (False, True):
    s = torch.cuda.Stream()
    s.wait_stream(main)
    with torch.cuda.stream(s):
        body(two)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(two)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    print("two streams" if two else "one stream ", f"{a.elapsed_time(b) / 10:.3f} ms per replay", flush=True)
