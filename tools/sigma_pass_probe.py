"""Diagnostic: the split MLP backward's sigma pass (ncn_field_bwd_mlp_part part 2) timed at several
grid sizes on the bench batch (512 = two workgroups per CU, the product; 256 = one) — how much
the pass gains from co-resident workgroups.  Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
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
xyzs, dirs = mk["xyzs"][:n].contiguous(), mk["dirs"][:n].contiguous()
L = _lib.lib()
packed = model._pack_weights()
enc = torch.empty(((n + 15) // 16) * 64 * 8, dtype=torch.float16, device=dev)
sig = torch.empty(n, device=dev)
rgb = torch.empty(n, 3, device=dev)
table = model.flat_params()[: model._n_table]
assert L.ncn_field_fwd(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(None), ptr(table), model._levels_ptr,
                       F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(0), I32(0), ptr(sig), ptr(rgb),
                       ptr(enc), stream()) == 0
gen = torch.Generator(device="cuda").manual_seed(0)
dsig = torch.randn(n, device=dev, generator=gen) * 1e-3
drgb = torch.randn(n, 3, device=dev, generator=gen) * 1e-3
nb1 = int(L.ncn_field_bwd_part_blocks(I64(n), I32(1)))
slab = torch.empty(max(768, nb1, int(L.ncn_field_bwd_part_blocks(I64(n), I32(2)))) * 10240, device=dev)  # (every grid timed below)
dE = torch.empty(int(L.ncn_field_bwd_dE_floats(I64(n))), device=dev)
lmax = torch.zeros(16 * 1024, device=dev)
stash = torch.empty(int(L.ncn_field_bwd_stash_floats(I64(n))), device=dev)


def part(p, nb):
    return L.ncn_field_bwd_mlp_part(ptr(xyzs), ptr(dirs), I64(n), ptr(None), ptr(None), ptr(packed), I32(0), ptr(enc),
                                    ptr(dsig if p == 2 else None), ptr(None), ptr(drgb if p == 1 else None), ptr(None),
                                    I32(p), I32(nb), ptr(slab), ptr(dE), ptr(lmax), ptr(stash), stream())


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


assert part(1, 240) == 0
print("samples", n, "rgb pass (240 workgroups) %.1f us" % ev_time(lambda: part(1, 240)), flush=True)
for nb in (768, 512, 384, 256):
    print(f"sigma pass, {nb} workgroups: {ev_time(lambda: part(2, nb)):.1f} us", flush=True)
