"""Occupancy-grid refresh on the device (csrc/grid.hip via NGPMT.update_density_grid) against the
numpy restatement of ngp_mt.py:305-368 (oracle/vren_ref.py: density_grid_update, packbits).

What is exact: the hit cells' positions lie in their cell's jitter box (ngp_mt.py:318-319), their
densities are the field's density mode at those positions (bit-equal to NGPMT.density), the update
where(grid < 0, grid, max(grid*decay, tmp)) of every cell, the bitfield (packbits against
min(mean, threshold): the device threshold is within 1e-6 of the oracle's f64 mean, the bitfield is
packbits of the updated grid against it).
What is statistical (the sampling is random in the reference too): the fraction of cells hit vs the
marginal probability of M uniform + M occupied draws with replacement (5 sigma).
"""
import numpy as np
import pytest
import torch

from oracle import vren_ref
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers

pytestmark = pytest.mark.gpu


def _model(dev, G, seed=0):
    torch.manual_seed(seed)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=G).to(dev))
    with torch.no_grad():  # a table with structure: densities spread over ~[0.1, 20]
        m.flat_params()[: m._n_table].mul_(3e4)
    return m


def _init_grid(m, rng, frac_neg=0.05):
    N = m.grid_size ** 3
    g = rng.exponential(3.0, (m.cascades, N)).astype(np.float32)
    g[rng.random((m.cascades, N)) < 0.5] = 0.0
    g[rng.random((m.cascades, N)) < frac_neg] = -1.0  # cells marked invisible (mark_invisible_cells)
    with torch.no_grad():
        m.density_grid.copy_(torch.from_numpy(g))
    return g


def _hits(m):
    ws = m._gws
    n = int(ws["scal"][0].item())
    return n, ws["idx"][:n].cpu().numpy(), ws["xyzs"][:n].cpu().numpy(), ws["sigmas"][:n].cpu().numpy()


def _check_update(m, old, thr, decay=0.95):
    G, C = m.grid_size, m.cascades
    assert C == 1
    n, idx, xyz, sig = _hits(m)
    # each hit cell once
    assert len(np.unique(idx)) == n
    # positions inside the cell's jitter box
    centre, hg = vren_ref.grid_cell_positions(idx, G, min(2 ** (0 - 1), m.scale))
    assert np.all(np.abs(xyz - centre) <= hg * (1 + 1e-5) + 1e-7)
    # densities = the density mode of the field at those positions
    with torch.no_grad():
        ref_sig = m.density(torch.from_numpy(xyz).to(m.density_grid.device)).cpu().numpy()
    np.testing.assert_array_equal(sig, ref_sig)
    new_ref, thr_ref, _ = vren_ref.density_grid_update(old, idx, sig, decay, thr)
    new = m.density_grid.cpu().numpy()
    np.testing.assert_array_equal(new, new_ref)
    thr_dev = float(m._gws["scal"][1:2].view(torch.float32).item())
    if np.isnan(thr_ref):
        assert np.isnan(thr_dev)
        assert int(m.density_bitfield.sum().item()) == 0
        return n, idx
    assert abs(thr_dev - thr_ref) <= 1e-6 * abs(thr_ref)
    bf = m.density_bitfield.cpu().numpy()
    ref_bf = vren_ref.packbits(new, thr_dev)
    np.testing.assert_array_equal(bf, ref_bf)
    return n, idx


@pytest.mark.parametrize("G", [32, 128])
def test_grid_refresh_warmup_all_cells(dev, G):
    m = _model(dev, G)
    rng = np.random.default_rng(1)
    old = _init_grid(m, rng)
    m.update_density_grid(1e4, warmup=True, seed=123)  # threshold above the mean: min(mean, thr) = mean
    n, idx = _check_update(m, old, 1e4)
    assert n == G ** 3
    assert np.array_equal(np.sort(idx), np.arange(G ** 3))


def test_grid_refresh_sampled(dev):
    G = 128
    m = _model(dev, G)
    rng = np.random.default_rng(2)
    old = _init_grid(m, rng)
    thr = 0.01 * 1024 / 3 ** 0.5
    m.update_density_grid(thr, warmup=False, seed=7)
    n, idx = _check_update(m, old, thr)
    N = G ** 3
    occ = old[0] > thr
    p_u, p_o = vren_ref.grid_hit_probabilities(N, N // 4, int(occ.sum()))
    hit = np.zeros(N, bool)
    hit[idx] = True
    for mask, p in ((~occ, p_u), (occ, 1 - (1 - p_u) * (1 - p_o))):
        k = int(mask.sum())
        f = hit[mask].mean()
        assert abs(f - p) <= 5 * np.sqrt(p * (1 - p) / k), (f, p, k)


def test_grid_refresh_deterministic_and_seeded(dev):
    m = _model(dev, 64)
    old = _init_grid(m, np.random.default_rng(3))
    thr = 2.0
    outs = []
    for seed in (11, 11, 12):
        with torch.no_grad():
            m.density_grid.copy_(torch.from_numpy(old))
        m.update_density_grid(thr, warmup=False, seed=seed)
        outs.append((m.density_grid.clone(), m.density_bitfield.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert not torch.equal(outs[0][0], outs[2][0])


def test_grid_refresh_empty_grid_clears_bitfield(dev):
    """Quirk q12 (ngp_mt.py:365-368): no cell > 0 -> mean NaN -> packbits against NaN -> all zero."""
    m = _model(dev, 32)
    with torch.no_grad():
        m.density_grid.fill_(-1.0)
        m.density_bitfield.fill_(255)
    m.update_density_grid(0.5, warmup=True, seed=5)
    assert torch.all(m.density_grid == -1.0)
    assert int(m.density_bitfield.sum().item()) == 0


def test_grid_refresh_erode(dev):
    m = _model(dev, 32)
    rng = np.random.default_rng(4)
    old = _init_grid(m, rng, frac_neg=0.0)
    cnt = rng.integers(0, 4, old.shape).astype(np.float32)
    m.count_grid = torch.from_numpy(cnt).to(dev)
    m.update_density_grid(1e4, warmup=True, erode=True, seed=9)
    n, idx, xyz, sig = _hits(m)
    new_ref, _, _ = vren_ref.density_grid_update(old, idx, sig, 0.95, 1e4, count_grid=cnt)
    np.testing.assert_allclose(m.density_grid.cpu().numpy(), new_ref, rtol=1e-6, atol=0)


@pytest.mark.parametrize("branch", ["pinhole", "ndc"])
def test_mark_invisible_cells_golden(dev, branch):
    """NGPMT.mark_invisible_cells vs the reference's own (tests/golden/invisible_cells.npz, made by
    tests/golden/make_golden.py from models/ngp_mt.py:274-337 on a 32^3 grid, 20 synthetic poses):
    the 0 / -1 marks and the per-cell camera counts.  The projections run as fp32 matmuls on the
    device (the fixture: torch CPU), so a cell projecting within rounding of an image border or of
    the near plane may flip: at most 0.05 % of the cells."""
    import os
    from ncnerf_amd import synthetic
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "invisible_cells.npz"))
    G, n_cams = int(f["G"]), int(f["n_cams"])
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=G).to(dev))
    scene = synthetic.SyntheticScene()
    poses = torch.from_numpy(scene.poses[:n_cams].astype(np.float32)).to(dev)
    K = torch.from_numpy(f["K"]) if branch == "pinhole" else (torch.from_numpy(f["M_ndc"]), torch.from_numpy(f["M_uv"]),
                                                              [0.0, 0.0, 0.0], float(f["ndc_scale"]))
    m.mark_invisible_cells(K, dev, poses, (synthetic.IMG_W, synthetic.IMG_H), float(f["near"]), chunk=5000)
    dens = m.density_grid.cpu().numpy()
    cnt = np.rint(m.count_grid.cpu().numpy() * n_cams).astype(np.int64)
    bad_d = int((dens != f[branch + "_density"].astype(np.float32)).sum())
    bad_c = int((cnt != f[branch + "_count"].astype(np.int64)).sum())
    assert set(np.unique(dens).tolist()) <= {0.0, -1.0}
    assert bad_d <= 0.0005 * dens.size and bad_c <= 0.0005 * dens.size, (bad_d, bad_c)
