"""CPU tests of the oracle's arithmetic emulations used by the PSNR-parity ensembles (round 4):
the field backward's loss-scaled fp16 gradient rounding (oracle/field_ref.py bwd_scale), the
oracle trainer's GradScaler (oracle/train_ref.py emulate_bwd) and the reference's own grid-refresh
draws (oracle/grid_ref.py sampling="reference", ngp_mt.py:244-270)."""
import numpy as np
import torch

from oracle import field_ref, grid_ref


def _field_grads(bwd_scale, upstream=1.0, seed=0, n=512):
    torch.manual_seed(seed)
    P, levels = field_ref.init_params(seed=1, table_init=0.3)
    params = [t.requires_grad_(True) for t in P.tensors()]
    P = field_ref.FieldParams(*params)
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(n, 3, generator=g) - 0.5) * 0.98
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=1)
    sig, rgb, _ = field_ref.field_forward_autograd(x, d, P, levels, emulate="fp16", bwd_scale=bwd_scale)
    ws = torch.randn(n, generator=g) * upstream
    wr = torch.randn(n, 3, generator=g) * upstream
    ((sig.clamp(max=50.0) * ws).sum() + (rgb * wr).sum()).backward()
    return [p.grad.clone() for p in params]


def test_backward_rounding_is_close_to_straight_through():
    """At the kernel's scale (128 x 2^16) and a training step's upstream size (~1e-5 per sample) the
    rounded chain stays within fp16's relative precision of the straight-through (fp32) one, and
    differs from it."""
    a = _field_grads(None, upstream=1e-5)
    b = _field_grads(128.0 * 65536, upstream=1e-5)
    for x, y in zip(a, b):
        rel = float((x - y).norm() / x.norm().clamp_min(1e-30))
        assert rel < 5e-3, rel
    assert any(not torch.equal(x, y) for x, y in zip(a, b))


def test_backward_rounding_underflow_and_overflow():
    """Unscaled (K = 1) tiny upstream gradients underflow in fp16 — most MLP weight gradients come
    out zero — while the kernel's scale keeps them; a huge scale overflows to inf (the GradScaler
    then skips the step)."""
    tiny = _field_grads(1.0, upstream=1e-9)
    scaled = _field_grads(128.0 * 65536, upstream=1e-9)
    zeros = lambda gs: sum(int((g == 0).sum()) for g in gs[1:])  # MLP weight gradients  # noqa: E731
    assert zeros(tiny) > 2 * zeros(scaled) + 100
    big = _field_grads(2.0 ** 60, upstream=1.0)
    assert not all(bool(torch.isfinite(g).all()) for g in big)


def test_cpu_trainer_grad_scaler_skip_and_backoff():
    """emulate_bwd: a non-finite gradient (forced by an absurd scale) skips the optimizer step
    (parameters unchanged), halves the scale and counts the skip."""
    from oracle.train_ref import CPUTrainer
    from ncnerf_amd.synthetic import SyntheticScene
    scene = SyntheticScene()
    tr = CPUTrainer(scene.bitfield, seed=3, encode_impl="c", emulate="fp16", emulate_bwd=True)
    tr.amp_S = 2.0 ** 120
    before = [p.detach().clone() for p in tr.params]
    tr.step(scene.batch(256, seed=5), global_step=10)
    assert tr.amp_skips == 1 and tr.amp_S == 2.0 ** 119
    assert all(torch.equal(a, p.detach()) for a, p in zip(before, tr.params))
    tr.amp_S = 65536.0
    tr.step(scene.batch(256, seed=6), global_step=11)
    assert tr.amp_skips == 1 and tr.amp_tracker == 1
    assert any(not torch.equal(a, p.detach()) for a, p in zip(before, tr.params))


def test_reference_grid_sampling():
    """sampling="reference": M = G^3/4 uniform draws and M draws among the occupied cells, with
    replacement; a drawn cell gets the density of (one of) its draws, every other cell only decays."""
    G = 32
    N = G ** 3
    rng = np.random.default_rng(0)
    grid = np.zeros((1, N), np.float32)
    occ = rng.choice(N, 500, replace=False)
    grid[0, occ] = 100.0
    grid[0, :10] = -1.0  # invisible cells keep -1 (ngp_mt.py:360-363)
    dens = lambda x: np.full(x.shape[0], 1000.0, np.float32)  # noqa: E731
    g2, thr, bf = grid_ref.grid_refresh(grid, dens, 10.0, False, 1234, G, 0.5, sampling="reference")
    hit = g2[0] == 1000.0
    cells, coords, _ = grid_ref.reference_cells(grid[0], 10.0, (1234 + 0) % 2 ** 64, G)
    drawn = np.zeros(N, bool)
    drawn[cells] = True
    drawn[:10] = False
    assert np.array_equal(hit, drawn)
    assert np.all(g2[0, :10] == -1.0)
    assert np.all(g2[0, occ[~drawn[occ]]] == np.float32(100.0 * 0.95))  # occupied, not drawn: decayed
    # with replacement: ~1 - e^-0.25 of the cells uniformly, and the occupied ones almost all
    frac_u = drawn.mean()
    assert 0.2 < frac_u < 0.35
    assert drawn[occ].mean() > 0.99
    assert cells.shape[0] == 2 * (N // 4)
