"""Diagnostic (not product): time the training marcher's walk pass on the bench batch (8192 rays):
the wave-parallel kernel (exp_step_factor == 0) against the serial lane-per-ray kernel (taken for
exp_step_factor = 1e-9, which yields the same constant dt), back to back behind a GPU spin, and check
they agree.  usage: python tools/march_lab.py [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd import _lib  # noqa: E402
from ncnerf_amd._lib import F32, I32, I64, ptr, stream  # noqa: E402
from ncnerf_amd.custom_functions import RayAABBIntersector  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
b = scene.torch_batch(R, seed=0, device=dev)
o, d = b["rays_o"].contiguous(), b["rays_d"].contiguous()
_, hits_t, _ = RayAABBIntersector.apply(o, d, model.center, model.half_size, 1)
t0 = hits_t[:, 0, 0]
t0.masked_fill_((t0 >= 0) & (t0 < 0.01), 0.01)
ht = hits_t[:, 0].contiguous()
noise = torch.rand(R, device=dev)
MS = 1024
pos = ((ht[:, 1] - ht[:, 0]).clamp(min=0) / (1.7320508 / 1024)).ceil()
print(f"rays {R}  chain positions/ray mean {pos.mean().item():.1f} max {pos.max().item():.0f}", flush=True)


def outs():
    return (torch.zeros(R, dtype=torch.int32, device=dev), torch.zeros(R * MS * 3, device=dev),
            torch.zeros(R * MS, device=dev), torch.zeros(R * MS, device=dev))


def run(esf, oo):
    return _lib.lib().ncn_march_train_walk(ptr(o), ptr(d), ptr(ht), ptr(noise), I64(R), ptr(model.density_bitfield),
                                           I32(1), F32(0.5), F32(esf), I32(128), I32(MS), *[ptr(t) for t in oo],
                                           stream())


def timeit(esf, oo, reps=20):
    assert run(esf, oo) == 0
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        torch.cuda._sleep(2_000_000)
        a.record()
        for _ in range(reps):
            run(esf, oo)
        e.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(e) * 1e3 / reps)
    return best


ow, os_ = outs(), outs()
tw = timeit(0.0, ow)
ts = timeit(1e-9, os_)
cnt = ow[0].long()
S = int(cnt.sum())
same = torch.equal(ow[0], os_[0])
mask = (torch.arange(MS, device=dev)[None, :] < cnt[:, None]).reshape(-1)
for x, y in zip(ow[1:], os_[1:]):
    k = x.numel() // (R * MS)
    m = mask.repeat_interleave(k) if k > 1 else mask
    same = same and torch.equal(x[m], y[m])
print(f"walk wave   {tw:8.2f} us", flush=True)
print(f"walk serial {ts:8.2f} us   S={S} ({S / R:.1f}/ray)  identical={same}", flush=True)
