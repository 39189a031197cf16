"""PSNR parity after equal steps, long form (BASELINE.json north_star: "PSNR within +-0.05 dB of
reference after equal steps") — test infrastructure, not product code.

The reference trajectory is the oracle CPU step (oracle/train_ref.py: the reference algorithm in
plain PyTorch fp32 + the C marcher/compositor; AdamW + clip 0.05; cosine LR per 1000-step epoch)
with the occupancy grid maintained as train_nerf.py does it (mark_invisible_cells at the start,
update_density_grid every 16 steps, all cells for the first 256 steps; oracle/grid_ref.py, the
device's sampling restated).  The HIP trajectory is the product step (ncnerf_amd.trainer.Trainer,
whole step in a HIP graph, grid refresh on the device) fed the SAME batches (synthetic room,
8192-ray patch batches, gt "surface_bright"), the same marcher noise and the same refresh seeds,
from the same initial parameters (step 0: the clustering weight ramps in from step 500 as
losses.py:217 schedules it).

Two halves, so the slow one needs no GPU:
  python tests/psnr_trajectory.py ref --steps 3000 --out profiles/round2/psnr_ref_trajectory.json   (CPU)
  python tests/psnr_trajectory.py hip --ref profiles/round2/psnr_ref_trajectory.json \
         --out profiles/round2/psnr_parity_trajectory.json                                              (GPU)
PSNR is measured at the same checkpoints on the same held-out rays: the oracle side with the oracle
renderer (train path, zero noise), the HIP side with the HIP test renderer (the two renderers agree
on the same parameters: tests/test_gpu_psnr.py).  The HIP side runs twice with identical inputs:
the difference between those two runs (float-atomic summation order only) is the run-to-run floor
the reference-vs-HIP difference is read against.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

N_RAYS = 8192
GT = "surface_bright"
EVAL_SEEDS = (90_000, 90_001)
INIT_SEED = 4
THRESHOLD = 0.01 * 1024 / 3 ** 0.5  # train_nerf.py:316 (density_tresh_decay 1)


# Ensemble members (VERDICT r2 "do this" 1): member m draws its own initial parameters, batches,
# marcher noise and refresh seeds; m = None is the legacy single trajectory of round 2.
MEMBER_STRIDE = 1_000_000


def init_seed(member=None):
    return INIT_SEED if member is None else 100 + member


def _base(member):
    return 0 if member is None else MEMBER_STRIDE * (member + 1)


def batch_seed(k, member=None):
    return _base(member) + 10_000 + k


def noise_of(k, n=N_RAYS, member=None):
    return torch.rand(n, generator=torch.Generator().manual_seed(_base(member) + 20_000 + k))


def grid_seed(k, member=None):
    return _base(member) + 30_000 + k


def camera_K():
    from ncnerf_amd import synthetic
    fx = (synthetic.IMG_W / 2) / math.tan(synthetic.HFOV / 2)
    return np.array([[fx, 0, synthetic.IMG_W / 2], [0, fx, synthetic.IMG_H / 2], [0, 0, 1]], np.float32)


def _psnr(se, n):
    return -10.0 * math.log10(max(se / n, 1e-12))


# normal-clustering weights per preset (the three loss_norm_D_C_* terms; ncnerf_amd.trainer.PRESETS)
PRESET_CLUSTER_W = {"hypersim": 2e-3, "scannet_manhattan": 1e-2}


def run_ref(steps, every, threads, log, out=None, member=None, n_rays=N_RAYS, impl="torch", emulate=None,
            preset="hypersim", emulate_bwd=False, sampling="device"):
    from oracle import field_ref, grid_ref
    from oracle.train_ref import CPUTrainer, render_train_ref
    from ncnerf_amd import synthetic
    from ncnerf_amd.synthetic import SyntheticScene
    torch.set_num_threads(threads)
    scene = SyntheticScene()
    cpu = CPUTrainer(scene.bitfield, seed=init_seed(member), num_epochs=30, epoch_steps=1000, encode_impl=impl,
                     emulate=emulate, w_cluster=PRESET_CLUSTER_W[preset], emulate_bwd=emulate_bwd)
    grid, _ = grid_ref.mark_invisible_cells(camera_K(), scene.poses, (synthetic.IMG_W, synthetic.IMG_H), 0.01, 128,
                                            0.5)
    ev = [scene.batch(N_RAYS, seed=s, gt=GT) for s in EVAL_SEEDS]
    curve, t0 = [], time.time()
    for k in range(steps):
        if k % 16 == 0:
            dens = lambda x: field_ref.density(torch.from_numpy(x), cpu.P, cpu.levels, impl=impl,  # noqa: E731
                                               emulate=emulate).numpy()
            grid, thr, bf = grid_ref.grid_refresh(grid, dens, THRESHOLD, k < 256, grid_seed(k, member), 128, 0.5,
                                                  sampling=sampling)
            cpu.bitfield = np.ascontiguousarray(bf, np.uint8)
        b = scene.batch(n_rays, seed=batch_seed(k, member), gt=GT)
        loss, S = cpu.step(b, global_step=k, noise=noise_of(k, n_rays, member).numpy())
        if (k + 1) % every == 0 or k + 1 == steps:
            se, n = 0.0, 0
            with torch.no_grad():
                for e in ev:
                    r = render_train_ref(cpu.P, cpu.levels, e["rays_o"], e["rays_d"], cpu.bitfield,
                                         np.zeros(N_RAYS, np.float32), impl=impl, emulate=emulate)
                    se += float(((r["rgb"].clamp(0, 1) - torch.from_numpy(e["rgb"])) ** 2).sum())
                    n += e["rgb"].size
            curve.append({"step": k + 1, "psnr": _psnr(se, n), "loss": loss, "samples": S,
                          "occupied_frac": float(np.unpackbits(cpu.bitfield).mean()), "t_s": round(time.time() - t0, 1)})
            log(json.dumps(curve[-1]))
            res = {"side": "oracle CPU", "steps": k + 1, "rays_per_step": n_rays, "gt": GT,
                   "member": member, "init_seed": init_seed(member), "encode_impl": impl, "emulate": emulate,
                   "emulate_bwd": emulate_bwd, "grid_sampling": sampling, "amp_scale": cpu.amp_S,
                   "amp_skips": cpu.amp_skips, "preset": preset, "eval_rays": N_RAYS * len(EVAL_SEEDS), "cpu_threads": threads,
                   "curve": curve}
            if out:  # the trajectory so far (a partial run is usable up to its last checkpoint)
                with open(out, "w") as f:
                    f.write(json.dumps(res) + "\n")
    return res


def host_batches(steps, n_rays, member=None):
    """The training batches of a trajectory (host arrays), to reuse across repeated HIP runs."""
    from ncnerf_amd.synthetic import SyntheticScene
    scene = SyntheticScene()
    return [scene.batch(n_rays, seed=batch_seed(k, member), gt=GT) for k in range(steps)]


def run_hip(steps, every, log, cross_check=False, member=None, n_rays=N_RAYS, trainer_kw=None, batches=None):
    from ncnerf_amd import synthetic
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.rendering import render
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    from oracle import field_ref
    dev = torch.device("cuda:0")
    scene = SyntheticScene()
    P, _ = field_ref.init_params(seed=init_seed(member))
    ev = [scene.torch_batch(N_RAYS, seed=s, device=dev, gt=GT) for s in EVAL_SEEDS]
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    flat, off = m.flat_params(), 0
    with torch.no_grad():
        for W in P.tensors():
            flat[off:off + W.numel()].copy_(W.reshape(-1))
            off += W.numel()
    m.mark_invisible_cells(torch.from_numpy(camera_K()), dev, torch.from_numpy(scene.poses).to(dev),
                           (synthetic.IMG_W, synthetic.IMG_H), 0.01)
    tr = Trainer(m, update_grid=True, use_graph=True, **(trainer_kw or {}))
    tr.grid_seed = lambda k: grid_seed(k, member)
    curve, t0 = [], time.time()
    for k in range(steps):
        if batches is not None:
            b = {kk: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) and not kk.endswith("_offsets_local")
                      else v) for kk, v in batches[k].items()}
        else:
            b = scene.torch_batch(n_rays, seed=batch_seed(k, member), device=dev, gt=GT)
        b["march_noise"] = noise_of(k, n_rays, member).to(dev)
        _, ld = tr.step(b, global_step=k)
        if (k + 1) % every == 0 or k + 1 == steps:
            se, se_tr, se_or, n = 0.0, 0.0, 0.0, 0
            P_cpu, bf_cpu = None, None
            if cross_check:  # the same parameters and bitfield through the oracle's renderer (CPU)
                from oracle.train_ref import render_train_ref
                flat = m.flat_params().detach().cpu()
                Pc, levels = field_ref.init_params(seed=init_seed(member))
                off, ts_ = 0, []
                for W in Pc.tensors():
                    ts_.append(flat[off:off + W.numel()].view_as(W).clone())
                    off += W.numel()
                P_cpu, bf_cpu = field_ref.FieldParams(*ts_), m.density_bitfield.cpu().numpy()
            with torch.no_grad():
                for e in ev:
                    r = render(m, e["rays_o"], e["rays_d"], near_distance=0.01, max_samples=1024, test_time=True)
                    se += float(((r["rgb"].clamp(0, 1) - e["rgb"]) ** 2).sum())
                    n += e["rgb"].numel()
                    if cross_check:
                        rt = render(m, e["rays_o"], e["rays_d"], near_distance=0.01, max_samples=1024,
                                    test_time=False, march_noise=torch.zeros(N_RAYS, device=dev))
                        se_tr += float(((rt["rgb"].clamp(0, 1) - e["rgb"]) ** 2).sum())
                        ro = render_train_ref(P_cpu, levels, e["rays_o"].cpu().numpy(), e["rays_d"].cpu().numpy(),
                                              bf_cpu, np.zeros(N_RAYS, np.float32))
                        se_or += float(((ro["rgb"].clamp(0, 1) - e["rgb"].cpu()) ** 2).sum())
            extra = {"psnr_train_render": _psnr(se_tr, n), "psnr_oracle_render": _psnr(se_or, n)} if cross_check else {}
            curve.append({"step": k + 1, "psnr": _psnr(se, n), **extra, "loss": float(ld["total"].detach()),
                          "occupied_frac": float((m.density_bitfield.cpu().numpy()[:, None] >> np.arange(8) & 1).mean()),
                          "t_s": round(time.time() - t0, 1)})
            log(json.dumps(curve[-1]))
    return {"side": "HIP", "member": member, "rays_per_step": n_rays, "curve": curve}


def main():
    global GT
    ap = argparse.ArgumentParser()
    ap.add_argument("side", choices=("ref", "hip"))
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--every", type=int, default=500)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--ref", default=None, help="(hip) the oracle trajectory JSON")
    ap.add_argument("--repeats", type=int, default=2, help="(hip) identical-input HIP runs")
    ap.add_argument("--out", default=None)
    ap.add_argument("--member", type=int, default=None, help="ensemble member (seeds); default: legacy seeds")
    ap.add_argument("--rays", type=int, default=N_RAYS, help="rays per training step")
    ap.add_argument("--preset", default="hypersim", choices=sorted(PRESET_CLUSTER_W),
                    help="hyper-parameter preset (the normal-clustering weights)")
    ap.add_argument("--impl", default="torch", choices=("torch", "c"), help="(ref) the oracle's hash-grid statement")
    ap.add_argument("--emulate", default=None, choices=("fp16", "bf16"),
                    help="(ref) round the MLP operands as tcnn's fp16 FullyFusedMLP / the HIP kernel do")
    ap.add_argument("--emulate-bwd", action="store_true",
                    help="(ref, with --emulate) also round the field backward's gradients as the kernel's loss-scaled "
                         "fp16 chain (with the GradScaler)")
    ap.add_argument("--sampling", default="device", choices=("device", "reference"),
                    help="(ref) the grid refresh's cell sampling: the device's (deviation 7) or the reference's draws")
    ap.add_argument("--gt", default="surface_bright",
                    help="target variant (ncnerf_amd.synthetic SyntheticScene.batch gt=...)")
    ap.add_argument("--cross-check", action="store_true",
                    help="(hip) also render the HIP parameters with the train-path renderer and the oracle's")
    a = ap.parse_args()
    GT = a.gt
    log = lambda s: print(s, flush=True)  # noqa: E731
    if a.side == "ref":
        res = run_ref(a.steps, a.every, a.threads, log, a.out, member=a.member, n_rays=a.rays, impl=a.impl,
                      emulate=a.emulate, preset=a.preset, emulate_bwd=a.emulate_bwd, sampling=a.sampling)
    else:
        ref = json.load(open(a.ref)) if a.ref else None
        steps = ref["steps"] if ref else a.steps
        runs = [run_hip(steps, a.every, log, cross_check=(i == 0 and a.cross_check), member=a.member, n_rays=a.rays)
                for i in range(a.repeats)]
        res = {"steps": steps, "rays_per_step": a.rays, "gt": GT, "hip_runs": runs}
        last = [r["curve"][-1]["psnr"] for r in runs]
        res["psnr_hip"] = last
        res["hip_run_to_run_db"] = max(last) - min(last)
        if ref:
            res["ref"] = ref
            res["psnr_ref"] = ref["curve"][-1]["psnr"]
            res["delta_db"] = [p - res["psnr_ref"] for p in last]
            # per-checkpoint deltas (same steps on both sides)
            rc = {c["step"]: c["psnr"] for c in ref["curve"]}
            res["delta_curve"] = [[c["step"], round(c["psnr"] - rc[c["step"]], 4)] for c in runs[0]["curve"]
                                  if c["step"] in rc]
    line = json.dumps(res)
    print(line)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
