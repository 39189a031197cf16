"""Host/device breakdown of one training step (diagnostic; not part of the product)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd.losses import NeRFMTLoss  # noqa: E402,F401
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import render  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10)
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
tr = Trainer(model, update_grid=False)
batches = [scene.torch_batch(8192, seed=i, device=dev) for i in range(4)]
for k in range(5):
    tr.step(batches[k % 4], 3000 + k)
torch.cuda.synchronize()
stages = {"render": 0.0, "loss": 0.0, "backward": 0.0, "opt": 0.0}
N = 10
for k in range(N):
    b = batches[k % 4]
    t = time.perf_counter()
    tr.opt.zero_grad()
    res = render(model, b["rays_o"], b["rays_d"], **dict(tr.render_kwargs, global_step=3000))
    torch.cuda.synchronize(); t1 = time.perf_counter(); stages["render"] += t1 - t
    ld = tr.loss(res, b, global_step=3000)
    torch.cuda.synchronize(); t2 = time.perf_counter(); stages["loss"] += t2 - t1
    ld["total"].backward()
    torch.cuda.synchronize(); t3 = time.perf_counter(); stages["backward"] += t3 - t2
    tr.opt.step()
    torch.cuda.synchronize(); t4 = time.perf_counter(); stages["opt"] += t4 - t3
print({k: round(1e3 * v / N, 3) for k, v in stages.items()}, "ms/step (synced stages)")
t = time.perf_counter()
for k in range(N):
    tr.step(batches[k % 4], 3000 + k)
torch.cuda.synchronize()
print("unsynced ms/step", round(1e3 * (time.perf_counter() - t) / N, 3))
pr = cProfile.Profile()
pr.enable()
for k in range(N):
    tr.step(batches[k % 4], 3000 + k)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
