"""The test-time render of full 1024x768 images (render(..., test_time=True): rendering.py:45-149's
host-driven loop) timed per image, for a rocprofv3 kernel trace: `torch.cuda._sleep` spin kernels
mark the image boundaries; tools/eval_render_summary.py turns the trace into the GPU-busy share of
each image's wall time.  The model is the bench's: 500 training steps on the procedural grid
(Trainer, graph step), or --distill N (bench.distill_opaque).  Not part of the product."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import render  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pretrain", type=int, default=500)
ap.add_argument("--distill", type=int, default=0)
ap.add_argument("--images", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
with torch.no_grad():
    model.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
    model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
tr = Trainer(model, use_graph=True, defer_optimizer=True)
if args.distill:
    from bench import distill_opaque
    distill_opaque(model, tr, scene, dev, steps=args.distill)
pool = [scene.torch_batch(8192, seed=1000 + i, device=dev, gt="surface_bright") for i in range(16)]
for k in range(args.pretrain):
    tr.step(pool[k % len(pool)], global_step=k)
tr.flush_optimizer()
kw = dict(near_distance=0.01, max_samples=1024, test_time=True)
res = []
with torch.no_grad():
    o, d = scene.image_rays(0, dev)
    render(model, o, d, **kw)
    for cam in range(1, args.images + 1):
        o, d = scene.image_rays(cam, dev)
        torch.cuda.synchronize()
        torch.cuda._sleep(200000)  # marker
        torch.cuda.synchronize()
        st = {}
        t0 = time.perf_counter()
        out = render(model, o, d, loop_stats=st, **kw)
        torch.cuda.synchronize()
        res.append({"cam": cam, "wall_ms": round((time.perf_counter() - t0) * 1e3, 3), **st,
                    "mean_opacity": float(out["opacity"].mean())})
    torch.cuda._sleep(200000)  # marker
    torch.cuda.synchronize()
print(json.dumps({"images": res}))
