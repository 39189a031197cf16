"""Diagnostic (not product): time the composite-forward variants of tools/composite_lab.hip on
realistic marched samples (bench scene, 8192 rays), back to back behind a GPU spin, and check that
they agree with the product kernel.  Build: hipcc ... tools/composite_lab.hip -> tools/_build/lab.so."""
import ctypes
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
variants = [int(v) for v in sys.argv[2].split(",") if v] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 5, 6, 7, 8, 100, 101, 102, 103]
b = scene.torch_batch(R, seed=0, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
_, hits_t, _ = RayAABBIntersector.apply(o, d, model.center, model.half_size, 1)
t0 = hits_t[:, 0, 0]
t0.masked_fill_((t0 >= 0) & (t0 < 0.01), 0.01)
noise = torch.rand(R, device=dev)
rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(o, d, hits_t[:, 0].contiguous(),
                                                                 model.density_bitfield, 1, 0.5, 0.0, noise, 128, 1024)
S = xyzs.shape[0]
with torch.no_grad():
    out = model(xyzs, dirs)
sig, rgb = out["sigmas"].float().contiguous(), out["rgbs"].float().contiguous()
Nr = rays_a[:, 2]
print("rays", R, "samples", S, "per ray", S / R, "long(>256)", int((Nr > 256).sum()), "max", int(Nr.max()),
      "samples in long rays", int(Nr[Nr > 256].sum()), flush=True)
if os.environ.get("LAB_LONG_FIRST"):  # the training step's row order (long rays first)
    rays_a = torch.cat([rays_a[Nr > 256], rays_a[Nr <= 256]]).contiguous()

lab = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "lab.so"))
lab.lab_composite_fw.restype = ctypes.c_int


def outs():
    return [torch.zeros(R, dtype=torch.int64, device=dev), torch.zeros(R, device=dev), torch.zeros(R, device=dev),
            torch.zeros(R, 3, device=dev), torch.zeros(S, device=dev)]


def run_main(o_):
    return _lib.lib().ncn_composite_train_fw(ptr(sig), ptr(rgb), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S),
                                             I32(3), F32(1e-4), *[ptr(t) for t in o_], stream())


def run_lab(v):
    def f(o_):
        return lab.lab_composite_fw(ctypes.c_int(v), ptr(sig), ptr(rgb), ptr(deltas), ptr(ts), ptr(rays_a), I64(R),
                                    F32(1e-4), *[ptr(t) for t in o_], stream())
    return f


def timeit(f, o_, reps=50):
    assert f(o_) == 0
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(3):
        torch.cuda._sleep(2_000_000)
        a.record()
        for _ in range(reps):
            f(o_)
        e.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(e) * 1e3 / reps)
    return min(res)


ref = outs()
us = timeit(run_main, ref)
tot = ref[0].sum().item()
byts = 24.0 * tot + 4.0 * S + 52.0 * R
print(f"{'main':12s} {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s  S_vr {tot}", flush=True)
g_o, g_d, g_r = torch.rand(R, device=dev), torch.rand(R, device=dev), torch.rand(R, 3, device=dev)
d_s, d_r = torch.empty(S, device=dev), torch.empty(S, 3, device=dev)


def run_bw(o_):
    return _lib.lib().ncn_composite_train_bw(ptr(g_o), ptr(g_d), ptr(g_r), None, ptr(sig), ptr(rgb), ptr(ref[4]),
                                             ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S), I32(3), ptr(ref[1]),
                                             ptr(ref[2]), ptr(ref[3]), F32(1e-4), ptr(d_s), ptr(d_r), stream())


us = timeit(run_bw, None)
byts_bw = 24.0 * tot + 16.0 * S + 40.0 * R
print(f"{'main bw':12s} {us:7.2f} us  {byts_bw / us / 1e3:7.1f} GB/s", flush=True)
for v in variants:
    o_ = outs()
    us = timeit(run_lab(v), o_)
    line = f"{'v%d' % v:12s} {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s"
    if v < 4 or 6 <= v < 100:
        errs = [(a.double() - b_.double()).abs().max().item() for a, b_ in zip(ref, o_)]
        line += "  maxdiff " + " ".join(f"{e:.2g}" for e in errs)
    print(line, flush=True)

lab.lab_flat_stream.restype = ctypes.c_int
for blocks in (256, 512, 1024, 2048, 4096, max(1, S // 1024)):
    o_ = outs()

    def fs(o2, blocks=blocks):
        return lab.lab_flat_stream(ctypes.c_int(blocks), ptr(sig), ptr(rgb), ptr(deltas), ptr(ts), ptr(rays_a),
                                   I64(R), I64(S), *[ptr(t) for t in o2], stream())
    us = timeit(fs, o_)
    fb = 28.0 * (S // 4 * 4) + 52.0 * R
    print(f"{'flat%d' % blocks:12s} {us:7.2f} us  {fb / us / 1e3:7.1f} GB/s (flat-stream floor)", flush=True)

# attribution of the product kernel's time (tools/composite_lab2.hip)
lab2 = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "lab2.so"))
lab2.lab2_cfw.restype = ctypes.c_int
names = {0: "prod", 1: "no-ws", 2: "one-round", 3: "fake-seg", 4: "rows8", 5: "rows2", 6: "no-ws+1round",
         7: "no-ws+fake", 8: "nows+fake+1row", 9: "rows8 no-ws", 10: "blocks"}
for v in range(11):
    o_ = outs()

    def f2(o2, v=v):
        return lab2.lab2_cfw(ctypes.c_int(v), ptr(sig), ptr(rgb), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S),
                             F32(1e-4), *[ptr(t) for t in o2], stream())
    us = timeit(f2, o_)
    line = f"{'L2-' + names[v]:18s} {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s"
    if v in (0, 4, 5, 10):
        errs = [(a.double() - b_.double()).abs().max().item() for a, b_ in zip(ref, o_)]
        line += "  maxdiff " + " ".join(f"{e:.2g}" for e in errs)
    print(line, flush=True)
