"""Diagnostic: the first step's parameter gradient, HIP (eager render + NeRFMTLoss + backward) vs
the oracle CPU trainer, on the psnr_trajectory inputs (step 0, after mark_invisible_cells and the
warm-up refresh): relative L2 per block, zero patterns and sign agreement of the table gradient."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import psnr_trajectory as pt  # noqa: E402


def main():
    torch.set_num_threads(16)
    from oracle import field_ref
    from oracle.train_ref import CPUTrainer
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.rendering import render
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    dev = torch.device("cuda:0")
    scene = SyntheticScene()
    n = int(os.environ.get("RAYS", 8192))
    cpu = CPUTrainer(scene.bitfield, seed=pt.INIT_SEED)
    P, _ = field_ref.init_params(seed=pt.INIT_SEED)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    flat, off = m.flat_params(), 0
    with torch.no_grad():
        for W in P.tensors():
            flat[off:off + W.numel()].copy_(W.reshape(-1))
            off += W.numel()
    m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    tr = Trainer(m)
    b = scene.batch(n, seed=pt.batch_seed(0), gt=pt.GT)
    noise = pt.noise_of(0, n)
    cpu.step(b, global_step=0, noise=noise.numpy())
    gc = torch.cat([t.grad.reshape(-1) for t in cpu.params])
    bt = scene.torch_batch(n, seed=pt.batch_seed(0), device=dev, gt=pt.GT)
    m.flat_grad().zero_()
    res = render(m, bt["rays_o"], bt["rays_d"], march_noise=noise.to(dev), **tr.render_kwargs)
    ld = tr.loss(res, bt, global_step=0)
    ld["total"].backward()
    gh = m.flat_grad().detach().cpu().clone()
    nt = m._n_table
    sc = gc.norm() / gh.norm()
    print("norms cpu %.6e hip %.6e ratio %.6f" % (gc.norm(), gh.norm(), sc))
    gh = gh * sc  # (the oracle's gradient is clipped in place)
    for name, sl in (("table", slice(0, nt)), ("mlp", slice(nt, None))):
        a, h = gc[sl], gh[sl]
        print(f"{name}: rel-L2 {float((a - h).norm() / a.norm()):.3e}  nz cpu {int((a != 0).sum())} nz hip "
              f"{int((h != 0).sum())}  cpu-only {int(((a != 0) & (h == 0)).sum())}  hip-only "
              f"{int(((a == 0) & (h != 0)).sum())}  sign-disagree {int(((a * h) < 0).sum())}")
    lv, _ = field_ref.grid_levels()
    a, h = gc[:nt].view(-1, 2), gh[:nt].view(-1, 2)
    for l, L in enumerate(lv):
        s = slice(L["offset"], L["offset"] + L["params"])
        aa, hh = a[s].reshape(-1), h[s].reshape(-1)
        mag = aa.abs()[aa != 0]
        print(f"  L{l:2d} rel {float((aa - hh).norm() / max(aa.norm(), 1e-30)):.2e} nz {int((aa != 0).sum()):8d} "
              f"cpu-only {int(((aa != 0) & (hh == 0)).sum()):7d} hip-only {int(((aa == 0) & (hh != 0)).sum()):7d} "
              f"sign-dis {int(((aa * hh) < 0).sum()):7d}  |g| median {float(mag.median()) if mag.numel() else 0:.2e}")


if __name__ == "__main__":
    main()
