"""Diagnostic: time ncn_adam_step (prep + apply over the bench model's 11.4 M parameters, zero_grad
folded in, a sparse gradient like a training step's) for the main library and tools/_build/optim_*.so
variants (built from csrc/optim.hip with -D knobs), and check that every variant's parameters and
moments are bit-identical to the main library's.  Not part of the product."""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import F32, F64, I32, I64, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
n = 11_443_072 + 10_240  # hash table (5.72 M x 2) + MLP weights
n0 = 11_443_072
g = torch.Generator(device="cuda").manual_seed(0)
p0 = torch.randn(n, device=dev, generator=g) * 1e-2
m0 = torch.randn(n, device=dev, generator=g) * 1e-4
v0 = torch.rand(n, device=dev, generator=g) * 1e-6
grad0 = torch.randn(n, device=dev, generator=g) * 1e-4
grad0[torch.rand(n, device=dev, generator=g) < 0.85] = 0  # sparse like the table gradient
nwork = int(_lib.lib().ncn_adam_step_work_floats())


def state():
    work = torch.zeros(nwork, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    return p0.clone(), grad0.clone(), m0.clone(), v0.clone(), work, step


def run(lib, st):
    p, gr, m, v, work, step = st
    return lib.ncn_adam_step(ptr(p), ptr(gr), ptr(m), ptr(v), I64(n), I64(n0), F32(1.0), F32(0.05), F32(1e-2),
                             F64(0.9), F64(0.99), F32(1e-15), F32(0.0), F32(1e-6), ptr(None), ptr(step), ptr(work),
                             I32(1), ptr(None), ptr(None), stream())


def ev_time(lib, reps=20):
    ts = []
    for _ in range(reps):
        st = state()
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(100000)
        a.record()
        assert run(lib, st) == 0
        e.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e) * 1e3)
    return float(np.median(ts))


libs = [("main", _lib.lib())]
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "optim_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_adam_step.argtypes = _lib.SIGNATURES["ncn_adam_step"]
    L.ncn_adam_step.restype = ctypes.c_int
    libs.append((os.path.basename(so)[6:-3], L))
ref = None
for name, L in libs:
    t = ev_time(L)
    st = state()
    assert run(L, st) == 0
    torch.cuda.synchronize()
    out = (st[0], st[2], st[3], st[1])
    if ref is None:
        ref = out
    same = all(torch.equal(a, b) for a, b in zip(out, ref))
    print(f"  {name:24s} adam_step {t:7.1f} us  bit-identical to main: {same}", flush=True)
