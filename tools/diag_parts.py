"""Diagnostic: where the split MLP passes differ from the one-pass backward (slab tiles / dE)."""
import sys

import torch

sys.path.insert(0, "normal-clustering-nerf_amd")
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import I32, I64, ptr, stream  # noqa: E402
from ncnerf_amd.ngp_mt import N_W, NGPMT  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
g = torch.Generator(device=dev).manual_seed(n)
m = NGPMT(scale=0.5, grid_size=128, precision="fp16").to(dev)
with torch.no_grad():
    m.flat_params()[: m._n_table].uniform_(-0.3, 0.3, generator=g)
m.amp_state[0] = 4.0
x = (torch.rand(n, 3, device=dev, generator=g) - 0.5) * 0.99
d = torch.nn.functional.normalize(torch.randn(n, 3, device=dev, generator=g), dim=1)
n_dev = torch.tensor([n - 7], dtype=torch.int32, device=dev)
with torch.no_grad():
    _, _, enc, packed, order = m._field_fwd(x, d, n_dev, 0, True)
dsig = torch.randn(n, device=dev, generator=g) * 1e-2
drgb = torch.randn(n, 3, device=dev, generator=g) * 1e-2
L = _lib.lib()
nb = int(L.ncn_field_bwd_blocks(I64(n)))
dE_n = int(L.ncn_field_bwd_dE_floats(I64(n)))
scale = m._bwd_loss_scale()
s0 = torch.full((nb * N_W,), float("nan"), device=dev)
e0 = torch.zeros(dE_n, device=dev)
l0 = torch.full((16 * 256,), -1.0, device=dev)
_lib.call("ncn_field_bwd_mlp", ptr(d), I64(n), ptr(n_dev), ptr(order), ptr(packed), I32(0), ptr(enc), ptr(dsig),
          ptr(drgb), ptr(scale), ptr(s0), ptr(e0), ptr(l0), stream())
s1 = torch.full((nb * N_W,), float("nan"), device=dev)
e1 = torch.zeros(dE_n, device=dev)
l1 = torch.full((16 * 256,), -1.0, device=dev)
st = torch.zeros(int(L.ncn_field_bwd_stash_floats(I64(n))), device=dev)
for part, ds in ((1, None), (2, dsig)):
    _lib.call("ncn_field_bwd_mlp_part", ptr(d), I64(n), ptr(n_dev), ptr(order), ptr(packed), I32(0), ptr(enc), ptr(ds),
              ptr(None), ptr(drgb), ptr(scale), I32(part), I32(nb), ptr(s1), ptr(e1), ptr(l1), ptr(st), stream())
torch.cuda.synchronize()
S0, S1 = s0.view(nb, N_W), s1.view(nb, N_W)
offs = {"W1": (0, 2048), "W2": (2048, 3072), "W3": (3072, 5120), "W4": (5120, 9216), "W5": (9216, 10240)}
for k, (a, b) in offs.items():
    dd = (S0[:, a:b] - S1[:, a:b]).abs()
    print(k, "max diff", float(torch.nan_to_num(dd, nan=1e30).max()), "nan0", int(S0[:, a:b].isnan().sum()),
          "nan1", int(S1[:, a:b].isnan().sum()), "ndiff", int((S0[:, a:b] != S1[:, a:b]).sum()))
print("dE max diff", float((e0 - e1).abs().max()), "ndiff", int((e0 != e1).sum()))
print("lmax equal", torch.equal(l0[: 16 * nb], l1[: 16 * nb]))
ns = (n + 3) & ~3
E0, E1 = e0.view(16, ns, 2), e1.view(16, ns, 2)
idx = (E0 != E1).any(-1).any(0).nonzero().flatten().tolist()
print("samples with dE diffs:", idx[:20])
for s_ in idx[:3]:
    print(s_, "dsig", float(dsig[s_]), "E0", E0[:, s_, 0][:4].tolist(), "E1", E1[:, s_, 0][:4].tolist())
