"""Diagnostic: PSNR curve of the HIP training step on the synthetic room from step 0 (grid refresh
on, mark_invisible_cells first, as train_nerf.py's on_train_start + training_step do).
python tools/psnr_curve.py --steps 3000 --rays 2048"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import render  # noqa: E402
from ncnerf_amd import synthetic  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402


def psnr_of(model, scene, dev, n_batches=2, n=8192, gt="surface"):
    se, npx = 0.0, 0
    for e in range(n_batches):
        b = scene.torch_batch(n, seed=90_000 + e, device=dev, gt=gt)
        with torch.no_grad():
            r = render(model, b["rays_o"], b["rays_d"], near_distance=0.01, max_samples=1024, test_time=True)
        se += float(((r["rgb"].clamp(0, 1) - b["rgb"]) ** 2).sum())
        npx += n * 3
    return -10 * math.log10(se / npx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--rays", type=int, default=2048)
    ap.add_argument("--every", type=int, default=250)
    ap.add_argument("--gt", default="surface")
    ap.add_argument("--no-invisible", action="store_true")
    ap.add_argument("--no-grid-update", action="store_true", help="keep the synthetic occupancy bitfield")
    ap.add_argument("--grad-clip", type=float, default=0.05)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--cluster-w", type=float, default=2e-3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    scene = SyntheticScene()
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    if not a.no_invisible:
        fx = (synthetic.IMG_W / 2) / math.tan(synthetic.HFOV / 2)
        K = torch.tensor([[fx, 0, synthetic.IMG_W / 2], [0, fx, synthetic.IMG_H / 2], [0, 0, 1]], dtype=torch.float32)
        m.mark_invisible_cells(K, dev, torch.from_numpy(scene.poses).to(dev), (synthetic.IMG_W, synthetic.IMG_H), 0.01)
    if a.no_grid_update:
        m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    h = dict(grad_clip=a.grad_clip, lr=a.lr, loss_norm_D_C_ort_dot_w=a.cluster_w, loss_norm_D_C_centr_dot_w=a.cluster_w,
             loss_norm_D_C_centr_L1_w=a.cluster_w)
    tr = Trainer(m, hparams=h, update_grid=not a.no_grid_update, use_graph=True)
    curve = []
    t0 = time.time()
    for k in range(a.steps):
        b = scene.torch_batch(a.rays, seed=10_000 + k, device=dev, gt=a.gt)
        _, ld = tr.step(b, global_step=k)
        if (k + 1) % a.every == 0:
            p = psnr_of(m, scene, dev, gt=a.gt)
            occ = float((m.density_bitfield != 0).float().mean())
            curve.append((k + 1, round(p, 3), round(float(ld["total"].detach()), 5)))
            print(f"step {k + 1} psnr {p:.3f} loss {float(ld['total'].detach()):.5f} bitfield_bytes_nonzero {occ:.3f} "
                  f"t {time.time() - t0:.1f}s", flush=True)
    print(json.dumps({"curve": curve}))


if __name__ == "__main__":
    main()
