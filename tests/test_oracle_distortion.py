"""CPU: the oracle's distortion loss (losses.cu restated, O(N) prefix-sum form) equals the definition
it implements (sum_ij w_i w_j |t_i - t_j| + 1/3 sum w_i^2 delta_i), and its backward equals torch
autograd of that definition.  Tolerances: f32 vs f64, 1e-5 relative."""
import numpy as np
import torch

from oracle import losses_ref


def _rays(rng, counts):
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rays_a = np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)
    S = int(np.sum(counts))
    ws = rng.uniform(0, 0.1, S).astype(np.float32)
    deltas = rng.uniform(1e-3, 3e-3, S).astype(np.float32)
    ts = np.zeros(S, np.float32)
    for r, s0, n in rays_a:
        ts[s0:s0 + n] = np.cumsum(deltas[s0:s0 + n]) + rng.uniform(0, 0.5)
    return ws, deltas, ts, rays_a


def test_distortion_oracle_matches_definition():
    rng = np.random.default_rng(0)
    ws, deltas, ts, rays_a = _rays(rng, [0, 1, 2, 7, 64, 65, 130])
    loss, _, _ = losses_ref.distortion_loss_fw(ws, deltas, ts, rays_a)
    W = torch.from_numpy(ws).double().requires_grad_(True)
    ref = losses_ref.distortion_loss_naive(W, torch.from_numpy(deltas).double(), torch.from_numpy(ts).double(), rays_a)
    np.testing.assert_allclose(loss, ref.detach().numpy(), rtol=1e-5, atol=1e-9)
    g = np.linspace(0.5, 1.5, len(rays_a)).astype(np.float32)
    (ref * torch.from_numpy(g).double()).sum().backward()
    _, wsi, wtsi = losses_ref.distortion_loss_fw(ws, deltas, ts, rays_a)
    dws = losses_ref.distortion_loss_bw(g, wsi, wtsi, ws, deltas, ts, rays_a)
    np.testing.assert_allclose(dws, W.grad.numpy(), rtol=1e-4, atol=1e-7)
