"""Diagnostic (not product): the level-major hash-grid encoding of tools/encode_lab.hip against the
product forward (same enc_cache bytes), timed on the bench's marched samples and on the grid
refresh's ~1 M points.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared
-munsafe-fp-atomics tools/encode_lab.hip normal-clustering-nerf_amd/csrc/errors.cpp -o tools/_build/encode_lab.so"""
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
with torch.no_grad():
    model.flat_params()[: model._n_table].uniform_(-1e-2, 1e-2)
b = scene.torch_batch(8192, seed=1, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
_, hits_t, _ = RayAABBIntersector.apply(o, d, model.center, model.half_size, 1)
t0 = hits_t[:, 0, 0]
t0.masked_fill_((t0 >= 0) & (t0 < 0.01), 0.01)
rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(o, d, hits_t[:, 0].contiguous(),
                                                                 model.density_bitfield, 1, 0.5, 0.0,
                                                                 torch.rand(8192, device=dev), 128, 1024)
packed = model._pack_weights()
table = model.flat_params()[: model._n_table]
cells = vren.morton3D_invert(torch.arange(0, 128 ** 3, 2, dtype=torch.int32, device=dev))
pts = ((cells.float() + torch.rand(cells.shape, device=dev)) / 128 - 0.5).contiguous()
lab = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "encode_lab.so"))
lab.lab_encode_levels.restype = ctypes.c_int
main = _lib.lib()


def timeit(f, reps=20):
    assert f() == 0
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(60000)
        a.record()
        assert f() == 0
        e.record()
    torch.cuda.synchronize()
    return np.mean([a.elapsed_time(e) for a, e in evs]) * 1e3


for name, X, D in (("samples", xyzs, dirs), ("grid points", pts, None)):
    n = X.shape[0]
    groups = (n + 15) // 16
    enc = torch.zeros(groups * 64 * 8, dtype=torch.float16, device=dev)
    enc2 = torch.zeros_like(enc)
    sig, rgb = torch.empty(n, device=dev), torch.empty(n, 3, device=dev)
    mode = 0 if D is not None else 1

    def prod():
        return main.ncn_field_fwd(ptr(X), ptr(D), I64(n), ptr(None), ptr(None), ptr(table), model._levels_ptr,
                                  F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(0), I32(mode),
                                  ptr(sig), ptr(rgb) if mode == 0 else ptr(None), ptr(enc), stream())

    def enc_lab(spt):
        return lambda: lab.lab_encode_levels(ptr(X), I64(n), ptr(table), model._levels_ptr, F32(model._xyz_min),
                                             F32(model._xyz_extent), ctypes.c_int(spt), ptr(enc2), stream())

    tp = timeit(prod)
    t1, t4, t0 = timeit(enc_lab(1)), timeit(enc_lab(4)), timeit(enc_lab(0))
    torch.cuda.synchronize()
    k = (n // 16) * 512  # whole groups (the product also encodes the padding lanes of the last one)
    same = torch.equal(enc[:k].view(torch.int16), enc2[:k].view(torch.int16))
    print(f"{name:12s} n={n}: product fwd (mode {mode}, encode + MLP) {tp:7.1f} us | level-major encode "
          f"spt1 {t1:7.1f} us, spt4 {t4:7.1f} us, xcd-partitioned {t0:7.1f} us | enc bytes identical: {same}", flush=True)
