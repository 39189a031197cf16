"""Diagnostic: time ncn_field_bwd / ncn_field_fwd variants on realistic marched samples.

Variants are diagnostic builds of csrc/field.hip (tools/build_field_variants.sh) with parts of the
backward compiled out, to attribute the kernel time.  Not part of the product."""
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
with torch.no_grad():
    model.flat_params()[: model._n_table].uniform_(-1e-2, 1e-2)
b = scene.torch_batch(8192, seed=1, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
_, hits_t, _ = RayAABBIntersector.apply(o, d, model.center, model.half_size, 1)
t0 = hits_t[:, 0, 0]
t0.masked_fill_((t0 >= 0) & (t0 < 0.01), 0.01)
noise = torch.rand(8192, device=dev)
rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(o, d, hits_t[:, 0].contiguous(),
                                                                 model.density_bitfield, 1, 0.5, 0.0, noise, 128, 1024)
n = xyzs.shape[0]
print("samples", n, "per ray", n / 8192)
packed = model._pack_weights()
groups = (n + 15) // 16
enc = torch.empty(groups * 2 * 64 * 4, dtype=torch.float16, device=dev)
sig = torch.empty(n, device=dev)
rgb = torch.empty(n, 3, device=dev)
table = model.flat_params()[: model._n_table]


def fwd(lib):
    return lib.ncn_field_fwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(None), ptr(table), model._levels_ptr,
                             F32(model._xyz_min),
                             F32(model._xyz_extent), ptr(packed), I32(0), I32(0), ptr(sig), ptr(rgb), ptr(enc), stream())


main = _lib.lib()
assert fwd(main) == 0
gen = torch.Generator(device="cuda").manual_seed(0)
dsig = torch.randn(n, device=dev, generator=gen) * 1e-3
drgb = torch.randn(n, 3, device=dev, generator=gen) * 1e-3
gtab = torch.zeros_like(table)
nb = main.ncn_field_bwd_blocks(I64(n))
slab = torch.empty(nb * 19712, device=dev)
dE_ws = torch.empty(int(main.ncn_field_bwd_dE_floats(I64(n))), device=dev)
lmax = torch.empty(16 * 256, device=dev)


def bwd(lib):
    return lib.ncn_field_bwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(None), model._levels_ptr, F32(model._xyz_min),
                             F32(model._xyz_extent), ptr(packed), I32(0), ptr(enc), ptr(dsig), ptr(drgb), ptr(None), ptr(gtab),
                             ptr(slab),
                             ptr(dE_ws), ptr(lmax), stream())


def timeit(f, lib, reps=20):
    f(lib)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(60000)  # GPU busy while Python issues the launch
        a.record()
        assert f(lib) == 0
        e.record()
    torch.cuda.synchronize()
    return np.mean([a.elapsed_time(e) for a, e in evs]) * 1e3


# the grid refresh's density pass (mode 1): ~1 M points, one per grid cell, cells in Morton order
cells = vren.morton3D_invert(torch.arange(0, 128 ** 3, 2, dtype=torch.int32, device=dev))
pts = ((cells.float() + torch.rand(cells.shape, device=dev, generator=torch.Generator(device="cuda").manual_seed(1)))
       / 128 - 0.5).contiguous()
sig1 = torch.empty(pts.shape[0], device=dev)


def fwd1(lib):
    return lib.ncn_field_fwd(ptr(pts), ptr(None), I64(pts.shape[0]), ptr(None), ptr(None), ptr(table),
                             model._levels_ptr, F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(0),
                             I32(1), ptr(sig1), ptr(None), ptr(None), stream())


libs = [("main", main)]
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "field_*.so"))):
    L = ctypes.CDLL(so)
    for name in ("ncn_field_fwd", "ncn_field_bwd"):
        getattr(L, name).argtypes = _lib.SIGNATURES[name]
        getattr(L, name).restype = ctypes.c_int
    libs.append((os.path.basename(so)[6:-3], L))
gref = None
for name, L in libs:
    gtab.zero_()
    assert bwd(L) == 0
    torch.cuda.synchronize()
    g1 = gtab.clone()
    if gref is None:
        gref = g1
    else:
        rel = ((g1 - gref).norm() / gref.norm()).item()
        big = gref.abs() > 1e-3 * gref.abs().max()
        relb = ((g1 - gref)[big].abs() / gref[big].abs()).max().item()
        print(f"   table-grad vs main: rel-L2 {rel:.3e}, max rel on entries > 1e-3 max: {relb:.3e}")
    print(f"{name:16s} fwd {timeit(fwd, L):8.1f} us   bwd {timeit(bwd, L):8.1f} us   "
          f"fwd mode 1 ({pts.shape[0]} grid points) {timeit(fwd1, L):8.1f} us", flush=True)
    if hasattr(L, "ncn_diag_sc_times"):
        # (NCN_DIAG_SC_TIMES: wave 0 of each workgroup, cycles summed over its fine-level units, in
        # the odd slots of [256][10]: level setup, grabs (loads + set reads + claims + adds), its own
        # LDS ops draining, the unit's closing barrier, the flush)
        buf = (ctypes.c_ulonglong * (256 * 10))()
        L.ncn_diag_sc_times(buf, 1)
        assert bwd(L) == 0
        torch.cuda.synchronize()
        L.ncn_diag_sc_times(buf, 0)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 10).astype(np.float64)
        names = ["setup", "grabs", "lds drain", "barrier", "flush"]
        tot = sum(a[:, 2 * i + 1].mean() for i in range(5))
        print("   scatter fine-level cycles per WG (wave 0, mean over WGs):",
              "  ".join(f"{nm} {a[:, 2 * i + 1].mean():.0f} ({a[:, 2 * i + 1].mean() / tot:.0%})"
                        for i, nm in enumerate(names)))
    if hasattr(L, "ncn_diag_read_phases"):
        buf = (ctypes.c_ulonglong * 8)()
        L.ncn_diag_read_phases(buf)
        print("   scatter phases (cycles, wave 0 of WG 7): compute", buf[0], "lds", buf[1], "barrier", buf[2],
              "flush", buf[3])
