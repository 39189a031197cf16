"""The sample-major training compositor (ncn_composite_train_fw_sm) against the CPU oracle
(oracle/vren_ref.c, volumerendering.cu:97-137 restated) and against the ray-major kernel.

Tolerance as tests/test_gpu_vren.py::test_composite_fw_parity: |d| <= 2e-5 + 2e-4 |ref| on
opacity / depth / rend / ws (the transmittance enters each lane through a segmented wave product scan,
the segment sums are differences of wave prefix sums, __expf vs expf); total_samples exact except where a stop is
borderline (T within 1e-3 relative of T_threshold).  Segment layouts cover every boundary the
kernel has: 4-sample lane quads, 256-sample wave ranges, the one-row look-ahead and the row-at-a-time
continuation (a 256-sample ray starting at a range's last sample), rays without samples, rays of
257..1024 samples (the long-ray workgroups), stops on the first / last lane of a row and a
segment ending at the sample count."""
import numpy as np
import pytest
import torch

from oracle import vren_ref
from ncnerf_amd import vren
from ncnerf_amd.synthetic import SyntheticScene

pytestmark = pytest.mark.gpu
T_THR = 1e-4


def _codes(rays_a, S):
    """The marcher's per-sample ray codes: ray + 1, or -(ray + 1) for rays of more than 256 samples."""
    code = np.zeros(S, np.int32)
    for r, st, n in rays_a:
        if n:
            code[st:st + n] = -(r + 1) if n > 256 else r + 1
    return code


def _layout(lens, rng, opaque=()):
    """Segments of the given lengths in ray (= sample) order; rows long-first as the fused marcher
    orders them.  opaque: sample positions (global) given sigma 1e5 (a stop there)."""
    rows, start = [], 0
    for i, n in enumerate(lens):
        rows.append([i, start, int(n)])
        start += int(n)
    rays_a = np.array(rows, np.int64).reshape(-1, 3)
    long_ = rays_a[:, 2] > 256
    rays_a = np.concatenate([rays_a[long_], rays_a[~long_]])
    S = start
    sig = np.abs(rng.normal(0, 0.3, S)).astype(np.float32)  # T stays well above 1e-4 ...
    for k in opaque:
        if k < S:
            sig[k] = 1e5  # ... until an opaque sample
    raws = rng.random((S, 3), dtype=np.float32)
    deltas = np.full(S, 1.7e-3, np.float32)
    ts = (np.arange(S) % 977 * 1.7e-3).astype(np.float32)
    return rays_a, sig, raws, deltas, ts


def _run_sm(dev, rays_a, sig, raws, deltas, ts, codes, device_count=False, grid_samples=None, bg=1.0):
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    S = sig.shape[0]
    if not device_count:
        return vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(rays_a), T_THR, bg=bg,
                                             sample_ray=T(codes))
    # capacity-sized arrays (garbage past S, as the training step's) and the count on the device
    cap = S + 1000
    pad = lambda a, v: np.concatenate([a, np.full((cap - S,) + a.shape[1:], v, a.dtype)])
    n_dev = torch.tensor([S, rays_a.shape[0]], dtype=torch.int32, device=dev)
    out = vren.composite_train_multi_fw(T(pad(sig, 7.0)), T(pad(raws, 0.5)), T(pad(deltas, 1e-3)), T(pad(ts, 1.0)),
                                        T(rays_a), T_THR, bg=bg, sample_ray=T(pad(codes, 5)), n_samples_dev=n_dev,
                                        grid_samples=grid_samples)
    out[4] = out[4][:S]
    return out


def _check(out, ref, rays_a=None, sig=None, deltas=None, borderline_ok=False):
    tot, ref_tot = out[0].cpu().numpy(), ref[0]
    if borderline_ok:
        assert np.mean(tot == ref_tot) > 0.999 and np.max(np.abs(tot - ref_tot)) <= 1
    else:
        assert np.array_equal(tot, ref_tot), np.argwhere(tot != ref_tot)[:5]
    for a, r, name in zip(out[1:5], ref[1:], ("opacity", "depth", "rend", "ws")):
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=2e-4, atol=2e-5, err_msg=name)
    # background blend (rendering.py:232-240)
    rgb_bg = out[5].cpu().numpy()
    np.testing.assert_allclose(rgb_bg, ref[3] + 1.0 * (1 - ref[1])[:, None], rtol=2e-4, atol=3e-5)


def _boundary_lens(rng):
    """Lengths that put segment starts and ends on every boundary class: rows of 64, ranges of 256."""
    lens = [0, 1, 63, 1, 64, 0, 127, 129, 256, 255, 1, 0, 0, 2, 190, 66]
    # a 256-sample ray starting on the last sample of a 256-sample range: the row-at-a-time path
    s = sum(lens)
    lens.append(256 * ((s // 256) + 2) - 1 - s)
    lens.append(256)
    lens += [1, 256, 300, 1024, 0, 5, 257, 511]
    lens += list(rng.integers(0, 120, 300))
    lens += [64] * 8 + [256] * 4 + [17]
    return [int(x) for x in lens]


@pytest.mark.parametrize("seed", [0, 1])
def test_sm_boundaries_vs_oracle(dev, seed):
    rng = np.random.default_rng(seed)
    lens = _boundary_lens(rng)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    # stops: the first sample of some rays, lane 63 / lane 0 of rows, the last sample of a range,
    # inside long rays, and past-the-end (none)
    opaque = [starts[2], starts[7] + 10, 63, 64 * 9, 64 * 12 - 1, 256 * 3 - 1, 256 * 5]
    for i, n in enumerate(lens):
        if n > 256:
            opaque.append(starts[i] + int(rng.integers(0, 2 * n)))
        elif n > 0 and rng.random() < 0.3:
            opaque.append(starts[i] + int(rng.integers(0, n)))
    rays_a, sig, raws, deltas, ts = _layout(lens, rng, opaque)
    codes = _codes(rays_a, sig.shape[0])
    ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, T_THR)
    out = _run_sm(dev, rays_a, sig, raws, deltas, ts, codes)
    _check(out, ref)
    # the device-count form over capacity-sized arrays, with a grid covering only part of the
    # samples (waves loop over the rest) and with the exact grid: bit-identical to the host form
    for gs in (None, 1000):
        out2 = _run_sm(dev, rays_a, sig, raws, deltas, ts, codes, device_count=True,
                       grid_samples=gs or sig.shape[0])
        for a, b, name in zip(out, out2, ("total", "opacity", "depth", "rend", "ws", "rgb_bg")):
            assert torch.equal(a, b), (gs, name)


def test_sm_segment_ends_at_count(dev):
    """The last segment ends exactly at S, on lane 63 of a row and inside a row."""
    rng = np.random.default_rng(5)
    for lens in ([100, 28], [100, 30], [64], [256], [256, 256], [1], [300, 20]):
        rays_a, sig, raws, deltas, ts = _layout(lens, rng)
        ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, T_THR)
        _check(_run_sm(dev, rays_a, sig, raws, deltas, ts, _codes(rays_a, sig.shape[0])), ref)


def test_sm_no_samples(dev):
    """S = 0 (every ray missed): every ray's outputs come from the rays_a pass."""
    rays_a = np.array([[0, 0, 0], [1, 0, 0], [2, 0, 0]], np.int64)
    e = np.zeros(0, np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.composite_train_multi_fw(T(e), T(np.zeros((0, 3), np.float32)), T(e), T(e), T(rays_a), T_THR, bg=1.0,
                                        sample_ray=T(np.zeros(0, np.int32)))
    assert out[0].tolist() == [0, 0, 0] and out[1].abs().sum() == 0 and torch.all(out[5] == 1.0)


@pytest.mark.parametrize("sigma_scale", [20.0, 400.0, 0.0])
def test_sm_fused_marcher_batch(dev, sigma_scale):
    """The training step's inputs: the fused marcher's rays_a + sample codes on an 8192-ray bench
    batch (codes checked against rays_a), sigmas |N(0, scale^2)|: sm == oracle, and sm == the
    ray-major kernel within the same tolerance."""
    from ncnerf_amd.rendering import march_buffers, march_train_fused
    scene = SyntheticScene()
    b = scene.torch_batch(8192, seed=21, device=dev)

    class _Box:
        _aabb = ((0.0, 0.0, 0.0), (0.5, 0.5, 0.5))
        density_bitfield = torch.from_numpy(scene.bitfield).to(dev)
        cascades, scale, grid_size = 1, 0.5, 128

    mk = march_train_fused(_Box, b["rays_o"], b["rays_d"], 0.01, 1024,
                           noise=torch.rand(8192, generator=torch.Generator().manual_seed(3)).to(dev),
                           out=march_buffers(8192, 1024, dev, codes=True))
    S = int(mk["counter"][0])
    rays_a = mk["rays_a"].cpu().numpy()
    codes = mk["sample_ray"][:S].cpu().numpy()
    assert np.array_equal(codes, _codes(rays_a, S))
    rng = np.random.default_rng(int(sigma_scale) + 1)
    sig = np.abs(rng.normal(0, sigma_scale, S)).astype(np.float32)
    raws = rng.random((S, 3), dtype=np.float32)
    deltas, ts = mk["deltas"][:S].cpu().numpy(), mk["ts"][:S].cpu().numpy()
    ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, T_THR)
    out = _run_sm(dev, rays_a, sig, raws, deltas, ts, codes)
    _check(out, ref, borderline_ok=True)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rm = vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(rays_a), T_THR, bg=1.0)
    assert float((out[0] != rm[0]).float().mean()) < 1e-3
    for a, r, name in zip(out[1:], rm[1:], ("opacity", "depth", "rend", "ws", "rgb_bg")):
        torch.testing.assert_close(a, r, rtol=2e-4, atol=2e-5, msg=name)
