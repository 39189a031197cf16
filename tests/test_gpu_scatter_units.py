"""The table scatter alone (ncn_field_scatter) against the oracle's serial scatter
(oracle/hashgrid_ref.c hashgrid_bwd) on the same encoding gradient, at a size that spans several
units of every level with a ragged last one (round 5: the coarse levels' carried runs), for both operand types of the stored gradient.

Samples lie on rays (consecutive samples share coarse cells for long runs, so runs cross the
4-sample chunks and the rounds of a unit); the encoding gradient is fp16 values with zero stretches
(runs with nothing to add, runs ending in zeros).  The kernel's sums are exact 64-bit fixed point per
unit, flushed with f32 atomics; the oracle adds in f32 serially — so the two agree to f32 summation
order: rel-L2 <= 1e-6 over the table, every entry within 1e-5 of the largest, and the same non-zero
set.  Measured (profiles/round5/scatter_units_test.log): rel-L2 1.4-1.8e-7, max |diff| 0.7-1.1e-6 of
the largest entry, 0 of 3.1-4.5 M non-zero entries on one side only."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import field_ref
from ncnerf_amd import _lib
from ncnerf_amd._lib import F32, I32, I64, ptr, stream
from ncnerf_amd.ngp_mt import NGPMT

pytestmark = pytest.mark.gpu


def _ray_samples(n, seed):
    rng = np.random.default_rng(seed)
    per = 70
    R = (n + per - 1) // per
    o = rng.uniform(0.3, 0.7, (R, 3))
    d = rng.standard_normal((R, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = (np.arange(per) + rng.uniform(0, 1, (R, 1))) * (0.28 / per)
    x01 = (o[:, None, :] + t[:, :, None] * d[:, None, :]).reshape(-1, 3)[:n]
    return x01.astype(np.float32)


@pytest.mark.parametrize("n,op,mode", [(70001, "fp16", "unit"), (40960, "fp16", "unit"), (70001, "bf16", "unit"),
                                       (70001, "fp16", "scaled"), (40960, "bf16", "scaled"), (40960, "fp16", "inf"),
                                       # fewer units than workgroups: most draw nothing from the unit queue
                                       (5, "fp16", "unit"), (301, "bf16", "scaled")])
def test_scatter_matches_serial_oracle(dev, n, op, mode):
    """mode "unit": the stored pairs are the gradient (header 1/S = 1); "scaled": the pairs carry the
    loss scale S = 2^23 (values ~2^-12 stored as ~2^11) and the scatter multiplies by the header's
    1/S — exact, so the oracle scatters the unscaled values; "inf": one fp16 pair
    overflowed (GradScaler's skip case) — that level's maximum is inf, the scatter adds the level
    straight to the table with f32 atomics, and the inf / NaN (0 x inf) entries match the oracle's."""
    m = NGPMT(scale=0.5, grid_size=128).to(dev)
    levels = field_ref.grid_levels(0.5)[0]
    xw = (_ray_samples(n, seed=n) - np.float32(0.5)).astype(np.float32)  # world positions
    xyzs = torch.from_numpy(xw).to(dev)
    x01 = (xw + np.float32(0.5)).astype(np.float32)  # what the kernel forms: (x - xyz_min) * (1 / extent), extent 1
    rng = np.random.default_rng(n + 1)
    tdt = torch.float16 if op == "fp16" else torch.bfloat16
    S = 2.0 ** 23 if mode == "scaled" else 1.0
    amp = 2.0 ** -12 if mode == "scaled" else 1.0
    gt_ = torch.from_numpy((rng.uniform(-1, 1, (n, 16, 2)) * amp * S).astype(np.float32)).to(tdt)  # stored (scaled)
    gt_[torch.from_numpy(rng.random((n, 16)) < 0.2)] = 0  # zero contributions
    gt_[n // 3: n // 3 + 500] = 0  # a stretch of samples with nothing to add
    if mode == "inf":
        gt_[n // 2, 12, 1] = float("inf")  # one overflowed pair on a fine level
    g = (gt_.float() / S).numpy()  # the unscaled operand-type values as f32 (exact: S is a power of two)
    # the dE workspace: header {1 / S, operand type (0 fp16, 1 bf16)}, then level-major [16][n_stride]
    # pairs of the operand type
    n_stride = (n + 3) & ~3
    ws = torch.zeros(int(_lib.lib().ncn_field_bwd_dE_floats(I64(n))), dtype=torch.float32)
    ws[0] = 1.0 / S
    ws[1] = 0.0 if op == "fp16" else 1.0
    pairs = torch.zeros(16, n_stride, 2, dtype=tdt)
    pairs[:, :n] = gt_.permute(1, 0, 2)
    ws[4:4 + 16 * n_stride] = pairs.contiguous().view(torch.float32).reshape(-1)  # (the scatter fills the rest)
    ws = ws.to(dev)
    lm_rows = int(_lib.lib().ncn_field_bwd_blocks(I64(n)))
    lmax = torch.zeros(lm_rows, 16, dtype=torch.float32)
    lmax[0] = torch.from_numpy(np.abs(g).max(axis=(0, 2)))  # (inf on the overflowed level, as the MLP pass records)
    lmax = lmax.to(dev)
    # oracle: serial f32 scatter of the same (fp16-valued) gradient
    ref = field_ref._HashEncodeC.backward(
        type("Ctx", (), {"saved_tensors": (torch.from_numpy(x01),), "levels": levels,
                         "n_table": (m._n_table, 2)})(),
        torch.from_numpy(np.ascontiguousarray(g.reshape(n, 32))))[1].numpy().astype(np.float64)
    # the positions in sample order (header flag 0: strided loads), then in the scatter's permuted
    # load order (ncn_field_scatter_positions, as the training step's MLP pass writes them)
    for permuted in (False, True):
        if permuted:
            assert _lib.lib().ncn_field_scatter_positions(ptr(xyzs), I64(n), ptr(None), ptr(ws), stream()) == 0
        grad = torch.zeros(m._n_table, 2, dtype=torch.float32, device=dev)
        rc = _lib.lib().ncn_field_scatter(ptr(xyzs), I64(n), ptr(None), ptr(None), m._levels_ptr, F32(m._xyz_min),
                                          F32(m._xyz_extent), ptr(ws), ptr(lmax), I32(0), I32(16), I32(0), ptr(grad),
                                          stream())
        assert rc == 0, _lib.lib().ncn_last_error()
        torch.cuda.synchronize()
        assert float(ws[2]) == (15.0 if permuted else 0.0)  # (the mask of the four unit classes)
        # the unit queue (the workspace's last 32 words) is left zero: the second pass draws from it again
        assert int(ws[-32:].view(torch.int32).abs().sum()) == 0
        _check(grad.cpu().numpy().astype(np.float64), ref.copy(), n, op, mode, permuted)


def _check(got, ref, n, op, mode, permuted):
    if mode == "inf":
        bad = ~np.isfinite(ref)
        assert bad.any() and np.isinf(ref).any()
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        np.testing.assert_array_equal(np.isinf(got), np.isinf(ref))
        np.testing.assert_array_equal(np.sign(got[np.isinf(ref)]), np.sign(ref[np.isinf(ref)]))
        got, ref = np.where(bad, 0.0, got), np.where(bad, 0.0, ref)
    nz_bad = int(((got != 0) ^ (ref != 0)).sum())
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    print(f"n {n} {op} {mode} permuted={permuted}: non-zero entries {int((ref != 0).sum())}, on one side only {nz_bad}, rel-L2 {rel:.2e}, "
          f"max |diff| / max |ref| {np.abs(got - ref).max() / np.abs(ref).max():.2e}")
    assert nz_bad <= 1e-4 * int((ref != 0).sum())
    assert rel <= 1e-6, rel
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()
