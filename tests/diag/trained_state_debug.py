"""Where does a trained-state one-step gradient difference come from?  (tests/test_gpu_trained_state.py)

Trains the test's product run (PRESET, fp16) to the given steps, then from each snapshot runs the
HIP eager step and the oracle step three times — emulating the kernel's fp16 rounding with the HIP
step's labels and |.| branches (the test's comparison), the same in plain fp32, and emulating with
the HIP labels but its own branches — and prints the per-block gradient rel-L2 of the pairs, plus the
field forward on the same samples (sigmas / rgbs, HIP vs the emulating oracle).  If HIP vs the
emulating oracle is far below fp16-vs-fp32, the emulation pins the rounding; if the two are of the
same size the state's gradient is dominated by fp16 rounding noise that two correct statements
need not share.  Usage (GPU box): [PRESET=scannet_manhattan] python tests/diag/trained_state_debug.py [steps...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normal-clustering-nerf_amd"), os.path.join(ROOT, "tests")]

import test_gpu_trained_state as T  # noqa: E402
from oracle import field_ref, vren_ref  # noqa: E402


def _rel(a, b):
    nb = float(b.norm())
    return float((a - b).norm()) / nb if nb > 0 else float(a.norm())


def main():
    steps = tuple(int(s) for s in sys.argv[1:]) or (1000, 3000)
    dev = torch.device("cuda:0")
    preset, precision = os.environ.get("PRESET", "hypersim"), "fp16"
    snaps = T.train_snapshots(preset, precision, dev, steps=steps)
    for step in steps:
        snap = snaps[step]
        scene = T.SyntheticScene()
        batch = scene.batch(T.N_RAYS, seed=70_000 + step, gt="surface_bright")
        noise = torch.rand(T.N_RAYS, generator=torch.Generator().manual_seed(80_000 + step)).numpy()
        h = T._hip_step(preset, precision, snap, batch, noise, step, dev)
        signs = T.losses_ref.kink_signs(h["normals"][h["valid"]], h["labels"])
        kw = dict(force_labels=h["labels"], force_signs=signs)
        o16 = T._oracle_step(preset, precision, snap, batch, noise, step, **kw)
        o32 = T._oracle_step(preset, precision, snap, batch, noise, step, emulate=False, **kw)
        o16n = T._oracle_step(preset, precision, snap, batch, noise, step, force_labels=h["labels"])
        n_table = h["levels"][-1][0] + h["levels"][-1][1]
        rec = {"step": step, "amp": None if snap["amp"] is None else [float(x) for x in snap["amp"]],
               "samples": [h["samples"], o16["samples"], o32["samples"]],
               "skipped": [h["skipped"], o16["skipped"], o32["skipped"]],
               "loss_rgb": [h["rgb"], o16["rgb"], o32["rgb"]], "preset": preset,
               "kink_sign_mismatch": o16.get("sign_mismatch")}
        pairs = {"hip_vs_o16": (h["grad"], o16["grad"]), "hip_vs_o32": (h["grad"], o32["grad"]),
                 "o16_vs_o32": (o16["grad"], o32["grad"]), "hip_vs_o16_own_branches": (h["grad"], o16n["grad"])}
        for name, (a, b) in pairs.items():
            rec[name] = {bn: round(_rel(a[sl], b[sl]), 6) for bn, sl in T._blocks(h["levels"], n_table)}
        # the field forward on the same samples (the marcher is bit-exact)
        m = T.register_grid_buffers(T.NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev))
        with torch.no_grad():
            m.flat_params().copy_(snap["params"].to(dev))
        m.prepare_weights()
        o, d = batch["rays_o"], batch["rays_d"]
        _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
        ht = ht[:, 0].copy()
        near = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
        ht[near, 0] = 0.01
        _, xyzs, dirs, _, _, cnt = vren_ref.raymarching_train(o, d, ht, snap["bitfield"].numpy(), 1, 0.5, 0.0,
                                                              np.ascontiguousarray(noise, np.float32), 128, 1024)
        n = int(cnt[0])
        xs, ds = torch.from_numpy(xyzs[:n]), torch.from_numpy(dirs[:n])
        with torch.no_grad():
            out = m(xs.to(dev), ds.to(dev))
            sh, rh = out["sigmas"], out["rgbs"]
            P, levels = field_ref.init_params(seed=0)
            flat = snap["params"]
            off = 0
            ts = []
            for t in P.tensors():
                ts.append(flat[off:off + t.numel()].view_as(t).clone())
                off += t.numel()
            P = field_ref.FieldParams(*ts)
            so, ro, _ = field_ref.field_forward_autograd(xs, ds, P, levels, impl="c", emulate=precision)
        sh, rh = sh.float().cpu(), rh.float().cpu()
        rec["fwd"] = {"sigma_rel": _rel(sh, so), "sigma_maxabs": float((sh - so).abs().max()),
                      "sigma_max": float(so.abs().max()), "rgb_rel": _rel(rh, ro),
                      "rgb_maxabs": float((rh - ro).abs().max())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
