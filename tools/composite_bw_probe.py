"""Diagnostic: time the training composite backward (ncn_composite_train_bw_bg without dL_dws, the
step's form) on a marched bench batch for the main library and tools/_build/vren_*.so variants
(csrc/vren.hip built with -D knobs), and check bit-identity of dL/dsigma and dL/draws against the
main library.  Not part of the product."""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib, vren  # noqa: E402
from ncnerf_amd._lib import F32, I32, I64, ptr, stream  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import march_train_fused  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
b = scene.torch_batch(8192, seed=1, device=dev)
mk = march_train_fused(model, b["rays_o"].contiguous(), b["rays_d"].contiguous(), 0.01, 1024,
                       noise=torch.rand(8192, device=dev))
n = int(mk["counter"][0].item())
rays_a = mk["rays_a"].contiguous()
deltas, ts = mk["deltas"][:n].contiguous(), mk["ts"][:n].contiguous()
g = torch.Generator(device="cuda").manual_seed(2)
sig = (torch.randn(n, device=dev, generator=g) * 20).abs()
raws = torch.rand(n, 3, device=dev, generator=g)
_, opacity, depth, rend, ws, _ = vren.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, 1e-4, bg=1.0)
R = rays_a.shape[0]
dop = torch.randn(R, device=dev, generator=g) * 1e-3
ddep = torch.randn(R, device=dev, generator=g) * 1e-3
drgb = torch.randn(R, 3, device=dev, generator=g) * 1e-3
dsig = torch.empty_like(sig)
draws = torch.empty_like(raws)
print("samples", n, flush=True)


def run(lib):
    return lib.ncn_composite_train_bw_bg(ptr(dop), ptr(ddep), ptr(drgb), ptr(None), ptr(sig), ptr(raws), ptr(ws),
                                         ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(n), I32(3), ptr(opacity),
                                         ptr(depth), ptr(rend), F32(1e-4), F32(1.0), ptr(dsig), ptr(draws), stream())


def ev_time(lib, reps=40):
    run(lib)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(100000)
        a.record()
        assert run(lib) == 0
        e.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(e) for a, e in evs]) * 1e3)


libs = [("main", _lib.lib())]
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "vren_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_composite_train_bw_bg.argtypes = _lib.SIGNATURES["ncn_composite_train_bw_bg"]
    L.ncn_composite_train_bw_bg.restype = ctypes.c_int
    libs.append((os.path.basename(so)[5:-3], L))
ref = None
for name, L in libs:
    t = ev_time(L)
    dsig.zero_()
    draws.zero_()
    assert run(L) == 0
    torch.cuda.synchronize()
    out = (dsig.clone(), draws.clone())
    if ref is None:
        ref = out
    same = all(torch.equal(a, b) for a, b in zip(out, ref))
    print(f"  {name:24s} composite_bw {t:7.2f} us  bit-identical to main: {same}", flush=True)
