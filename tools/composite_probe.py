"""Diagnostic: time ncn_composite_train_fw of libncnerf.so and of diagnostic variant builds
(tools/_build/vren_*.so, tools/build_vren_variants.sh) on realistic marched samples, and check that
the variants agree.  Not part of the product."""
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
from ncnerf_amd.custom_functions import RayAABBIntersector  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
R = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
b = scene.torch_batch(R, seed=1, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
_, hits_t, _ = RayAABBIntersector.apply(o, d, model.center, model.half_size, 1)
t0 = hits_t[:, 0, 0]
t0.masked_fill_((t0 >= 0) & (t0 < 0.01), 0.01)
noise = torch.rand(R, device=dev)
rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(o, d, hits_t[:, 0].contiguous(),
                                                                 model.density_bitfield, 1, 0.5, 0.0, noise, 128, 1024)
S = xyzs.shape[0]
g = torch.Generator(device="cuda").manual_seed(0)
sig = (torch.randn(S, device=dev, generator=g) * 2).exp() * 5
rgb = torch.rand(S, 3, device=dev, generator=g)
print("rays", R, "samples", S, "per ray", S / R)


def outs():
    return [torch.empty(R, dtype=torch.int64, device=dev), torch.empty(R, device=dev), torch.empty(R, device=dev),
            torch.empty(R, 3, device=dev), torch.empty(S, device=dev)]


def fw(lib, o_):
    return lib.ncn_composite_train_fw(ptr(sig), ptr(rgb), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S), I32(3),
                                      F32(1e-4), *[ptr(t) for t in o_], stream())


def timeit(f, lib, o_, reps=50):
    f(lib, o_)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(60000)  # GPU busy while Python issues the launch (events bracket the kernel)
        a.record()
        f(lib, o_)
        e.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(e) for a, e in evs])) * 1e3


ref = None
libs = [("main", _lib.lib())]
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "vren_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_composite_train_fw.argtypes = _lib.SIGNATURES["ncn_composite_train_fw"]
    L.ncn_composite_train_fw.restype = ctypes.c_int
    libs.append((os.path.basename(so)[5:-3], L))
for name, L in libs:
    o_ = outs()
    us = timeit(fw, L, o_)
    tot = o_[0].sum().item()
    byts = 24.0 * tot + 4.0 * S + 52.0 * R
    print(f"{name:20s} fw {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s  S_vr {tot}", flush=True)
    if ref is None:
        ref = o_
    else:
        for a, b_, nm in zip(ref, o_, ("total", "opacity", "depth", "rend", "ws")):
            err = (a.double() - b_.double()).abs().max().item()
            print(f"   max|diff| {nm}: {err:.3g}")
