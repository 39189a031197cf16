"""Diagnostic: host-side time per Trainer.step (no synchronisation) vs wall time per step, for the
plain graph step and the pipelined one (is the step host-bound?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
batches = [scene.torch_batch(8192, seed=i, device=dev) for i in range(8)]
for pipe in (False, True, False, True):
    torch.manual_seed(0)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    with torch.no_grad():
        m.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
        m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    tr = Trainer(m, update_grid=False, use_graph=True)
    for k in range(5):
        tr.step(batches[k % 8], 3001 + k, next_batch=batches[(k + 1) % 8] if pipe else None)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for k in range(5, 105):
        a = time.perf_counter()
        tr.step(batches[k % 8], 3001 + k, next_batch=batches[(k + 1) % 8] if pipe else None)
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 100
    host.sort()
    print(f"pipe={pipe}: wall {wall * 1e6:7.1f} us/step, host median {host[50] * 1e6:7.1f} us, "
          f"p90 {host[90] * 1e6:7.1f} us", flush=True)
