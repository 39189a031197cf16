"""Diagnostic: the field forward of tools/_build/field_*.so variants against the product library on
the same marched samples — sigmas, rgbs and the encoding cache compared bit for bit."""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
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
_, xyzs, dirs, _, _, _ = vren.raymarching_train(o, d, hits_t[:, 0].contiguous(), model.density_bitfield, 1, 0.5, 0.0,
                                                noise, 128, 1024)
n = xyzs.shape[0]
packed = model._pack_weights()
table = model.flat_params()[: model._n_table]


def run(lib):
    enc = torch.zeros(((n + 15) // 16) * 2 * 64 * 4, dtype=torch.float16, device=dev)
    sig = torch.zeros(n, device=dev)
    rgb = torch.zeros(n, 3, device=dev)
    assert lib.ncn_field_fwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(None), ptr(table), model._levels_ptr,
                             F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(0), I32(0), ptr(sig),
                             ptr(rgb), ptr(enc), stream()) == 0
    torch.cuda.synchronize()
    return sig, rgb, enc


ref = run(_lib.lib())
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "field_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_field_fwd.argtypes = _lib.SIGNATURES["ncn_field_fwd"]
    L.ncn_field_fwd.restype = ctypes.c_int
    out = run(L)
    diffs = [int((a.view(torch.int16 if a.dtype == torch.float16 else torch.int32) !=
                  r.view(torch.int16 if r.dtype == torch.float16 else torch.int32)).sum()) for a, r in zip(out, ref)]
    enc_bad = (out[2] != ref[2]).nonzero()
    print(os.path.basename(so), "bitwise mismatches sig / rgb / enc:", diffs,
          "first enc idx", enc_bad[:4].flatten().tolist(), flush=True)
