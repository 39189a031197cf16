"""Diagnostic: the oracle CPU trainer and the HIP trainer side by side on identical inputs (the
psnr_trajectory setup) for a few steps: per-step loss, marched samples, and the occupancy after
each grid refresh.  python tests/diag/parity_probe.py --steps 64 [--no-refresh] [--rays 8192]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import psnr_trajectory as pt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--no-refresh", action="store_true")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from oracle import field_ref, grid_ref
    from oracle.train_ref import CPUTrainer
    from ncnerf_amd import synthetic
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    dev = torch.device("cuda:0")
    scene = SyntheticScene()
    cpu = CPUTrainer(scene.bitfield, seed=pt.INIT_SEED, num_epochs=30, epoch_steps=1000)
    grid, _ = grid_ref.mark_invisible_cells(pt.camera_K(), scene.poses, (synthetic.IMG_W, synthetic.IMG_H), 0.01,
                                            128, 0.5)
    P, _ = field_ref.init_params(seed=pt.INIT_SEED)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    flat, off = m.flat_params(), 0
    with torch.no_grad():
        for W in P.tensors():
            flat[off:off + W.numel()].copy_(W.reshape(-1))
            off += W.numel()
    m.mark_invisible_cells(torch.from_numpy(pt.camera_K()), dev, torch.from_numpy(scene.poses).to(dev),
                           (synthetic.IMG_W, synthetic.IMG_H), 0.01)
    if a.no_refresh:
        cpu.bitfield = np.ascontiguousarray(scene.bitfield)
        m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    tr = Trainer(m, update_grid=not a.no_refresh, use_graph=True)
    tr.grid_seed = pt.grid_seed
    for k in range(a.steps):
        rec = {"step": k}
        if not a.no_refresh and k % 16 == 0:
            dens = lambda x: field_ref.density(torch.from_numpy(x), cpu.P, cpu.levels).numpy()  # noqa: E731
            grid, thr, bf = grid_ref.grid_refresh(grid, dens, pt.THRESHOLD, k < 256, pt.grid_seed(k), 128, 0.5)
            cpu.bitfield = np.ascontiguousarray(bf, np.uint8)
            rec["occ_cpu"] = float(np.unpackbits(cpu.bitfield).mean())
            rec["thr_cpu"] = thr
        b = scene.batch(a.rays, seed=pt.batch_seed(k), gt=pt.GT)
        noise = pt.noise_of(k, a.rays)
        loss_c, S_c = cpu.step(b, global_step=k, noise=noise.numpy())
        bt = scene.torch_batch(a.rays, seed=pt.batch_seed(k), device=dev, gt=pt.GT)
        bt["march_noise"] = noise.to(dev)
        _, ld = tr.step(bt, global_step=k)
        if not a.no_refresh and k % 16 == 0:
            rec["occ_hip"] = float((m.density_bitfield.cpu().numpy()[:, None] >> np.arange(8) & 1).mean())
            rec["bitfield_diff_frac"] = float(np.unpackbits(cpu.bitfield ^ m.density_bitfield.cpu().numpy()).mean())
        rec.update(loss_cpu=round(loss_c, 6), loss_hip=round(float(ld["total"].detach()), 6), S_cpu=S_c)
        # parameter drift: relative L2 of the flat parameters
        pc = torch.cat([t.detach().reshape(-1) for t in cpu.params])
        ph = m.flat_params().detach().cpu()
        rec["param_rel_diff"] = float((pc - ph).norm() / pc.norm())
        rec["table_rel_diff"] = float((pc[:m._n_table] - ph[:m._n_table]).norm() / pc[:m._n_table].norm())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
