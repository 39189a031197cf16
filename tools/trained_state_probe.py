"""Diagnostic: how far the bench's trained states get towards early ray termination.  Trains the
bench model (Trainer, graph step, 8192-ray batches of the surface_bright target) on the
procedural occupancy grid (fixed, or refreshed from the model as train_nerf.py does) and prints,
every `--every` steps, the marched and composited samples per ray of the last 50 steps (a ray
that terminates early composites fewer samples than it marched).  Not part of the product."""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd import synthetic  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=4000)
ap.add_argument("--every", type=int, default=500)
ap.add_argument("--state", choices=("procedural", "refreshed"), default="procedural")
ap.add_argument("--refresh", action="store_true", help="refresh the procedural grid from the model every 16 steps")
ap.add_argument("--gt", default="surface_bright")
ap.add_argument("--distill", type=int, default=0, help="first fit the densities to the room's occupancy (steps)")
args = ap.parse_args()
dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
tr = Trainer(model, update_grid=args.state == "refreshed" or args.refresh, use_graph=True, defer_optimizer=True)
acc = torch.zeros(2, dtype=torch.float64, device=dev)
tr.render_kwargs["count_acc"] = acc
if args.state == "refreshed":
    fx = (synthetic.IMG_W / 2) / math.tan(synthetic.HFOV / 2)
    K = torch.tensor([[fx, 0, synthetic.IMG_W / 2], [0, fx, synthetic.IMG_H / 2], [0, 0, 1]])
    model.mark_invisible_cells(K, dev, torch.from_numpy(scene.poses).to(dev), (synthetic.IMG_W, synthetic.IMG_H), 0.01)
else:
    with torch.no_grad():
        model.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
        model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
if args.distill:
    sys.path.insert(0, ROOT)
    from bench import distill_opaque
    print(json.dumps({"distill": distill_opaque(model, tr, scene, dev, steps=args.distill)}), flush=True)
pool = [scene.torch_batch(8192, seed=1000 + i, device=dev, gt=args.gt) for i in range(64)]
for k in range(args.steps):
    if k % args.every == args.every - 50:
        acc.zero_()
    tr.step(pool[k % len(pool)], global_step=k)
    if k % args.every == args.every - 1:
        tr.flush_optimizer()
        a = acc.cpu().tolist()
        n = 50 * 8192
        print(json.dumps({"step": k + 1, "rm_per_ray": round(a[0] / n, 2), "vr_per_ray": round(a[1] / n, 2),
                          "vr_over_rm": round(a[1] / max(a[0], 1), 3)}), flush=True)
