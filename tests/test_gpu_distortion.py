"""HIP distortion loss (ncn_distortion_loss_fw/bw behind vren / losses.DistortionLoss) vs the CPU
oracle (oracle/losses_ref.py: losses.cu restated; pinned to the definition by
tests/test_oracle_distortion.py).  Tolerance on the loss: 1e-4 relative + 1e-7 absolute (the O(N) form subtracts products of prefix sums: f32 summation order is amplified); scans 1e-5 (wave-scan vs serial f32
summation order).  Edge rays: no samples, one sample, segments spanning several 64-sample rows, rays
in a permuted row order; and NeRFMTLoss's distortion term with quirk q5 (ws := ts, losses.py:290)."""
import numpy as np
import pytest
import torch

from oracle import losses_ref
from ncnerf_amd import vren
from ncnerf_amd.losses import DistortionLoss

pytestmark = pytest.mark.gpu


def _rays(rng, counts, permute=False):
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rays_a = np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)
    if permute:
        rays_a = rays_a[rng.permutation(len(counts))]
    S = int(np.sum(counts))
    ws = rng.uniform(0, 0.1, S).astype(np.float32)
    deltas = rng.uniform(1e-3, 3e-3, S).astype(np.float32)
    ts = np.zeros(S, np.float32)
    for r, s0, n in rays_a:
        ts[s0:s0 + n] = np.cumsum(deltas[s0:s0 + n]) + rng.uniform(0, 0.5)
    return ws, deltas, ts, rays_a


@pytest.mark.parametrize("permute", [False, True])
def test_distortion_fw_bw(dev, permute):
    rng = np.random.default_rng(1)
    counts = np.concatenate([[0, 1, 2, 63, 64, 65, 200, 466], rng.integers(0, 150, 500)])
    ws, deltas, ts, rays_a = _rays(rng, counts, permute)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    loss, wsi, wtsi = vren.distortion_loss_fw(T(ws), T(deltas), T(ts), T(rays_a))
    rl, rwsi, rwtsi = losses_ref.distortion_loss_fw(ws, deltas, ts, rays_a)
    np.testing.assert_allclose(loss.cpu().numpy(), rl, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(wsi.cpu().numpy(), rwsi, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(wtsi.cpu().numpy(), rwtsi, rtol=1e-5, atol=1e-7)
    g = rng.uniform(0.5, 1.5, len(counts)).astype(np.float32)
    dws = vren.distortion_loss_bw(T(g), wsi, wtsi, T(ws), T(deltas), T(ts), T(rays_a))
    ref = losses_ref.distortion_loss_bw(g, rwsi, rwtsi, ws, deltas, ts, rays_a)
    np.testing.assert_allclose(dws.cpu().numpy(), ref, rtol=1e-4, atol=1e-8)
    # the autograd Function
    W = T(ws).requires_grad_(True)
    (DistortionLoss.apply(W, T(deltas), T(ts), T(rays_a)) * T(g)).sum().backward()
    np.testing.assert_allclose(W.grad.cpu().numpy(), ref, rtol=1e-4, atol=1e-8)


def test_nerf_loss_distortion_term(dev):
    """NeRFMTLoss with loss_distortion_w > 0: distortion_w * mean(DistortionLoss(ts, deltas, ts,
    rays_a)) — the reference passes the sample positions as weights (quirk q5)."""
    from ncnerf_amd.losses import NeRFMTLoss
    rng = np.random.default_rng(2)
    counts = rng.integers(0, 100, 64)
    ws, deltas, ts, rays_a = _rays(rng, counts)
    R = len(counts)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    pred = {"rgb": torch.rand(R, 3, device=dev), "depth": torch.rand(R, device=dev),
            "opacity": torch.rand(R, device=dev), "rays_o": torch.rand(R, 3, device=dev),
            "rays_d": torch.rand(R, 3, device=dev), "ts": T(ts), "deltas": T(deltas), "ws": T(ws),
            "rays_a": T(rays_a)}
    target = {"rgb": torch.rand(R, 3, device=dev)}
    h = dict(loss_opacity_w=0.0, loss_distortion_w=1e-3)
    loss_d = NeRFMTLoss(h)(pred, target, global_step=0)
    ref, _, _ = losses_ref.distortion_loss_fw(ts, deltas, ts, rays_a)
    np.testing.assert_allclose(float(loss_d["distortion"]), 1e-3 * float(np.mean(ref)), rtol=1e-5)
