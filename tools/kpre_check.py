"""Diagnostic: the training marcher's outputs under the library named by
NCN_LIB_PATH (e.g. the -amdgpu-kernarg-preload-count=16 build) on many random batches that mix
rays missing the box, rays starting inside it and axis-parallel rays; writes one digest per batch
so two builds can be compared bit for bit (python tools/kpre_check.py out.json)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]
import torch  # noqa: E402
from ncnerf_amd import vren  # noqa: E402
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.rendering import march_train_fused  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticScene()
model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
digests = []
for it in range(int(os.environ.get("KPRE_BATCHES", "60"))):
    g = torch.Generator(device="cpu").manual_seed(it)
    R = 8192
    o = (torch.rand(R, 3, generator=g) * 2.4 - 1.2)  # many rays start outside and miss the box
    d = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=1)
    d[: R // 16, 1:] = 0.0  # axis-parallel rays
    d[: R // 16, 0] = 1.0
    o, d = o.to(dev).contiguous(), d.to(dev).contiguous()
    noise = torch.rand(R, generator=g).to(dev)
    mk = march_train_fused(model, o, d, 0.01, 1024, noise=noise)
    n = int(mk["counter"][0].item())
    h = hashlib.sha256()
    for k in ("rays_a", "xyzs", "dirs", "deltas", "ts"):
        t = mk[k]
        t = t[:n] if k != "rays_a" else t
        h.update(t.detach().contiguous().cpu().numpy().tobytes())
    # the eager vren path (walk / scan / pack) too
    _, hits, _ = vren.ray_aabb_intersect(o, d, torch.zeros(1, 3, device=dev), torch.full((1, 3), 0.5, device=dev), 1)
    ht = hits[:, 0].contiguous()
    out = vren.raymarching_train(o, d, ht, model.density_bitfield, 1, 0.5, 0.0, noise, 128, 1024)
    for t in out:
        h.update(t.detach().contiguous().cpu().numpy().tobytes())
    miss = int((ht[:, 0] < 0).sum())
    digests.append({"batch": it, "samples": n, "missed_rays": miss, "sha": h.hexdigest()})
with open(sys.argv[1], "w") as f:
    json.dump({"lib": os.environ.get("NCN_LIB_PATH", "default"), "digests": digests}, f)
print("batches", len(digests), "samples", sum(x["samples"] for x in digests))
