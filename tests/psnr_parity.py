"""PSNR parity after equal steps (BASELINE.json north_star: "PSNR within +-0.05 dB of reference
after equal steps") — test infrastructure, not product code.

Two trainings from the same initial parameters on the same batches with the same marcher noise:
  * "ref": the oracle CPU step (oracle/train_ref.py: the reference algorithm restated in plain
    PyTorch fp32 + the C marcher/compositor, AdamW + clip 0.05 as train_nerf.py:262-291, 955);
  * "hip": the product step (ncnerf_amd.trainer.Trainer, HIP kernels, whole step in a HIP graph).
Scene: the synthetic textured room (ncnerf_amd.synthetic, gt="surface"), fixed occupancy grid,
clustering loss at full weight (global_step >= 3000, losses.py:217).  Both parameter sets are then
rendered on held-out rays by the same HIP test renderer (rendering.py:45-149) and, on a subset, the
oracle's train renderer with zero noise, and PSNR = -10 log10(MSE) is compared.

Usage on a GPU box:  python tests/psnr_parity.py --steps 200 --rays 2048 --out profiles/<round>/psnr_parity.json
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

from oracle import field_ref  # noqa: E402
from oracle.train_ref import CPUTrainer, render_train_ref  # noqa: E402


def _psnr(mse):
    return -10.0 * math.log10(max(float(mse), 1e-12))


def _load_params(model, tensors):
    flat, off = model.flat_params(), 0
    with torch.no_grad():
        for W in tensors:
            flat[off:off + W.numel()].copy_(W.detach().reshape(-1))
            off += W.numel()


def run(steps=60, n_rays=1024, eval_batches=4, eval_rays=8192, oracle_eval_rays=1024, seed=4, step0=3000,
        threads=None, use_graph=True, log=None, precision="fp16", emulate=None):
    """precision: the HIP field's MLP operand type (config #3: "bf16"); emulate: the oracle's operand
    and backward-chain rounding (None: plain fp32; "fp16"/"bf16": as the kernel rounds, with the
    fp16 GradScaler) — returns the PSNRs and the per-step losses of both sides."""
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.rendering import render
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer

    if threads:
        torch.set_num_threads(threads)
    dev = torch.device("cuda:0")
    scene = SyntheticScene()
    cpu = CPUTrainer(scene.bitfield, seed=seed, emulate=emulate, emulate_bwd=emulate is not None)
    init = [t.detach().clone() for t in cpu.params]
    bf = torch.from_numpy(scene.bitfield).to(dev)

    def gpu_model(tensors):
        m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev))
        _load_params(m, tensors)
        m.density_bitfield.copy_(bf)
        return m

    m = gpu_model(init)
    tr = Trainer(m, update_grid=False, use_graph=use_graph)
    t_cpu = t_gpu = 0.0
    losses = []
    for k in range(steps):
        b = scene.batch(n_rays, seed=10_000 + k)
        noise = torch.rand(n_rays, generator=torch.Generator().manual_seed(20_000 + k))
        t = time.perf_counter()
        l_cpu, _ = cpu.step(b, global_step=step0 + k, noise=noise.numpy())
        t_cpu += time.perf_counter() - t
        bt = {kk: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for kk, v in b.items()}
        bt["march_noise"] = noise.to(dev)
        t = time.perf_counter()
        _, ld = tr.step(bt, global_step=step0 + k)
        l_gpu = float(ld["total"].detach())
        t_gpu += time.perf_counter() - t
        losses.append((l_cpu, l_gpu))
        if log and (k % 20 == 0 or k == steps - 1):
            log(f"step {k}: loss ref {l_cpu:.5f} hip {l_gpu:.5f}")

    m_ref = gpu_model(cpu.params)  # the oracle-trained parameters on the same HIP renderer
    se = {"hip": 0.0, "ref": 0.0}
    n_px = 0
    for e in range(eval_batches):
        b = scene.torch_batch(eval_rays, seed=90_000 + e, device=dev)
        for key, model in (("hip", m), ("ref", m_ref)):
            with torch.no_grad():
                res = render(model, b["rays_o"], b["rays_d"], near_distance=0.01, max_samples=1024, test_time=True)
            se[key] += float(((res["rgb"].clamp(0, 1) - b["rgb"]) ** 2).sum())
        n_px += eval_rays * 3
    out = {"steps": steps, "rays_per_step": n_rays, "step0": step0, "eval_rays": eval_batches * eval_rays,
           "precision": precision, "oracle_emulate": emulate, "losses_ref_hip": losses,
           "psnr_hip": _psnr(se["hip"] / n_px), "psnr_ref": _psnr(se["ref"] / n_px)}
    out["delta_db"] = out["psnr_hip"] - out["psnr_ref"]
    # renderer pin: the oracle's own (train-path, zero-noise) render of the oracle-trained
    # parameters vs the HIP test renderer of the same parameters on the same rays
    b = scene.batch(oracle_eval_rays, seed=90_000)
    P = field_ref.FieldParams(*[t.detach() for t in cpu.params])
    with torch.no_grad():
        r_or = render_train_ref(P, cpu.levels, b["rays_o"], b["rays_d"], scene.bitfield,
                                np.zeros(oracle_eval_rays, np.float32))
        bt = scene.torch_batch(oracle_eval_rays, seed=90_000, device=dev)
        r_hip = render(m_ref, bt["rays_o"], bt["rays_d"], near_distance=0.01, max_samples=1024, test_time=True)
    gt = torch.from_numpy(b["rgb"])
    out["psnr_ref_oracle_render"] = _psnr(((r_or["rgb"].clamp(0, 1) - gt) ** 2).mean())
    out["psnr_ref_hip_render_same_rays"] = _psnr(((r_hip["rgb"].cpu().clamp(0, 1) - gt) ** 2).mean())
    out["train_s_ref_cpu"] = round(t_cpu, 2)
    out["train_s_hip"] = round(t_gpu, 2)
    out["cpu_threads"] = torch.get_num_threads()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rays", type=int, default=2048)
    ap.add_argument("--eval-batches", type=int, default=8)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = run(steps=a.steps, n_rays=a.rays, eval_batches=a.eval_batches, seed=a.seed, threads=a.threads,
              log=lambda s: print(s, flush=True))
    line = json.dumps(res)
    print(line)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
