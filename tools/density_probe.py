"""Diagnostic: time the grid refresh's density pass (ncn_field_fwd mode 2: encode_xcd_kernel +
sigma_net) per library — the main one and tools/_build/field_*.so variants — on the hit list of a
real refresh of the bench's synthetic room, and check that every variant's sigmas are
bit-identical to the main library's.  Not part of the product."""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import F32, I32, I64, ptr, stream  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
with torch.no_grad():
    model.flat_params()[: model._n_table].uniform_(-1e-2, 1e-2)
    if os.environ.get("DENSITY_PROBE_BENCH_GRID"):  # the bench's grid (the room's density x 10)
        model.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
    else:
        model.density_grid.copy_((torch.rand_like(model.density_grid) < 0.05).float())
thr = 0.01 * 1024 / 3 ** 0.5
model.update_density_grid(thr, warmup=False, seed=7)  # fills the hit list of the (single) cascade
torch.cuda.synchronize()
ws = model._grid_ws()
N = model.grid_size ** 3
n_list = ws["scal"][0:1]
print("hit cells", int(n_list.item()), flush=True)
packed = model._take_packed()
table = model.xyz_encoder.params


def run(lib, mode=2):
    return lib.ncn_field_fwd(ptr(ws["xyzs"]), ptr(None), I64(N), ptr(n_list), ptr(None), ptr(table), model._levels_ptr,
                             F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(model._prec), I32(mode),
                             ptr(ws["sigmas"]), ptr(None), ptr(ws["enc"]), stream())


def ev_time(f, reps=20):
    f()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, e in evs:
        torch.cuda._sleep(100000)
        a.record()
        assert f() == 0
        e.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(e) for a, e in evs]) * 1e3)


libs = [("main", _lib.lib())]
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "_build", "field_*.so"))):
    L = ctypes.CDLL(so)
    L.ncn_field_fwd.argtypes = _lib.SIGNATURES["ncn_field_fwd"]
    L.ncn_field_fwd.restype = ctypes.c_int
    libs.append((os.path.basename(so)[6:-3], L))
ref = None
for name, L in libs:
    t = ev_time(lambda: run(L))
    n = int(n_list.item())
    sig = ws["sigmas"][:n].clone()
    if ref is None:
        ref = sig
    print(f"  {name:24s} density pass {t:7.1f} us  bit-identical to main: {torch.equal(sig, ref)}", flush=True)
    if name == "main":  # the sample-major density pass (mode 1: encoding + sigma_net in one launch)
        t1 = ev_time(lambda: run(L, 1))
        print(f"  {'main, mode 1':24s} density pass {t1:7.1f} us  bit-identical to mode 2: "
              f"{torch.equal(ws['sigmas'][:n], ref)}", flush=True)
