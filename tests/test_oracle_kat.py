"""Known-answer and property tests of the CPU oracle (oracle/vren_ref.c).  CPU only."""
import numpy as np
import pytest

from oracle import vren_ref

SQRT3 = np.float32(1.73205080757)


def test_morton_known_answers():
    c = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 1], [2, 0, 0], [127, 127, 127], [1023, 0, 0]],
                 np.int32)
    m = vren_ref.morton3D(c)
    assert m.tolist()[:6] == [0, 1, 2, 4, 7, 8]
    assert m[6] == (1 << 21) - 1
    assert m[7] == int("".join("001" for _ in range(10)), 2)
    assert np.array_equal(vren_ref.morton3D_invert(m), c)


def test_packbits_known_answer():
    g = np.zeros(16, np.float32)
    g[[0, 3, 7, 8, 15]] = 1.0
    g[9] = 0.5  # == threshold -> not set (strict >)
    bf = vren_ref.packbits(g, 0.5)
    assert bf.tolist() == [0b10001001, 0b10000001]


def test_aabb_known_answers():
    o = np.array([[-1, 0, 0], [0, 0, 0], [2, 2, 2], [-1, 0.25, 0]], np.float32)
    d = np.array([[1, 0, 0], [0, 0, 1], [1, 0, 0], [1, 0, 0]], np.float32)
    cnt, ht, hv = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
    assert cnt.tolist() == [1, 1, 0, 1]
    assert ht[0, 0].tolist() == [0.5, 1.5]
    assert ht[1, 0].tolist() == [0.0, 0.5]  # start inside: t1 clamped to 0 (intersection.cu:504)
    assert ht[2, 0].tolist() == [-1.0, -1.0] and hv[2, 0] == -1
    assert ht[3, 0].tolist() == [0.5, 1.5]  # axis-parallel: 1/d = inf handled by fminf/fmaxf


def test_aabb_multi_hits_sorted():
    rng = np.random.default_rng(0)
    c = rng.uniform(-1, 1, (6, 3)).astype(np.float32)
    h = np.full((6, 3), 0.3, np.float32)
    o = np.tile(np.array([[-3, 0, 0]], np.float32), (64, 1))
    d = rng.normal(size=(64, 3)).astype(np.float32)
    d[:, 0] = np.abs(d[:, 0]) + 2
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    cnt, ht, hv = vren_ref.ray_aabb_intersect(o, d, c, h, 6)
    for r in range(64):
        t1 = ht[r, :, 0]
        assert np.all(np.diff(t1) >= 0)
        assert (hv[r] >= 0).sum() == min(cnt[r], 6)


def _room_bitfield():
    from ncnerf_amd.synthetic import SyntheticScene
    return SyntheticScene()


def test_march_properties():
    sc = _room_bitfield()
    b = sc.batch(512, 0)
    _, ht, _ = vren_ref.ray_aabb_intersect(b["rays_o"], b["rays_d"], np.zeros((1, 3), np.float32),
                                          np.full((1, 3), 0.5, np.float32), 1)
    ht = ht[:, 0].copy()
    noise = np.random.default_rng(0).random(512, dtype=np.float32)
    rays_a, xyzs, dirs, deltas, ts, counter = vren_ref.raymarching_train(b["rays_o"], b["rays_d"], ht, sc.bitfield, 1,
                                                                         0.5, 0.0, noise, 128, 1024)
    S = int(counter[0])
    assert counter[1] == 512 and S == rays_a[:, 2].sum() and xyzs.shape == (S, 3)
    assert np.array_equal(rays_a[:, 0], np.arange(512))
    assert np.array_equal(rays_a[1:, 1], np.cumsum(rays_a[:, 2])[:-1])
    dt = SQRT3 / np.float32(1024)
    assert np.all(deltas == dt)  # exp_step_factor 0: constant dt = sqrt(3)/max_samples
    assert np.all(np.abs(xyzs) <= 0.5 + 1e-6)
    for r in range(0, 512, 37):
        s0, n = rays_a[r, 1], rays_a[r, 2]
        seg = ts[s0:s0 + n]
        assert np.all(np.diff(seg) >= dt * 0.999)
        o, d = b["rays_o"][r], b["rays_d"][r]
        assert np.allclose(xyzs[s0:s0 + n], o + seg[:, None] * d, atol=1e-6)
        assert np.all(dirs[s0:s0 + n] == d)
        # every sample lies in an occupied voxel
        v = np.clip(np.floor((xyzs[s0:s0 + n] + 0.5) * 128), 0, 127).astype(int)
        assert np.all(sc.occ[v[:, 0], v[:, 1], v[:, 2]])


def test_march_miss_and_max_samples():
    sc = _room_bitfield()
    o = np.array([[2, 2, 2], [0, 0, 0]], np.float32)
    d = np.array([[1, 0, 0], [0, 0, -1]], np.float32)
    ht = np.array([[-1, -1], [0.01, 100.0]], np.float32)  # far t2: voxel clamp keeps "occupied"
    rays_a, xyzs, *_ , counter = vren_ref.raymarching_train(o, d, ht, np.full_like(sc.bitfield, 255), 1, 0.5, 0.0,
                                                           np.zeros(2, np.float32), 128, 16)
    assert rays_a[0, 2] == 0  # miss: never perturbed, zero samples (quirk q9)
    assert rays_a[1, 2] == 16  # all occupied: capped at max_samples


def test_composite_closed_form():
    """Constant sigma*delta = c: T_k = exp(-k c) (up to rounding), weights geometric, stop at T <= T_thr."""
    n = 400
    c = np.float32(0.05)
    sig = np.full(n, 50.0, np.float32)
    dl = np.full(n, 1e-3, np.float32)
    ts = np.arange(n, dtype=np.float32) * 1e-3
    raws = np.tile(np.array([[0.2, 0.4, 0.6]], np.float32), (n, 1))
    rays_a = np.array([[0, 0, n]], np.int64)
    tot, op, de, rend, ws = vren_ref.composite_train_multi_fw(sig, raws, dl, ts, rays_a, 1e-4)
    k_stop = int(np.ceil(np.log(1e-4) / -0.05)) - 1  # first k with T_{k+1} <= 1e-4
    assert abs(int(tot[0]) - k_stop) <= 1
    a = 1 - np.exp(-c)
    np.testing.assert_allclose(ws[:5], a * np.exp(-c * np.arange(5)), rtol=1e-5)
    assert np.all(ws[int(tot[0]) + 1:] == 0)
    np.testing.assert_allclose(rend[0], op[0] * np.array([0.2, 0.4, 0.6]), rtol=1e-5)


@pytest.mark.parametrize("with_dws", [False, True])
def test_composite_bw_matches_finite_differences(with_dws):
    """volumerendering.cu:297-364's analytic backward vs central differences of the forward (float64 sums)."""
    rng = np.random.default_rng(3)
    n_rays, n = 6, 40
    rays_a = np.stack([np.arange(n_rays), np.arange(n_rays) * n, np.full(n_rays, n)], 1).astype(np.int64)
    S = n_rays * n
    sig = rng.uniform(0.5, 30, S).astype(np.float32)
    dl = rng.uniform(1e-3, 3e-3, S).astype(np.float32)
    ts = np.cumsum(dl).astype(np.float32)
    raws = rng.random((S, 3), dtype=np.float32)
    gO, gD, gR = rng.normal(size=n_rays), rng.normal(size=n_rays), rng.normal(size=(n_rays, 3))
    gW = rng.normal(size=S) if with_dws else None

    def L(s, r):
        _, op, de, rend, ws = vren_ref.composite_train_multi_fw(s, r, dl, ts, rays_a, 1e-4)
        v = (op * gO).sum() + (de * gD).sum() + (rend * gR).sum()
        return v + ((ws * gW).sum() if with_dws else 0.0)

    _, op, de, rend, ws = vren_ref.composite_train_multi_fw(sig, raws, dl, ts, rays_a, 1e-4)
    ds, dr = vren_ref.composite_train_multi_bw(gO.astype(np.float32), gD.astype(np.float32), gR.astype(np.float32),
                                               None if gW is None else gW.astype(np.float32), sig, raws, ws, dl, ts,
                                               rays_a, op, de, rend, 1e-4)
    idx = rng.choice(S, 25, replace=False)
    for i in idx:
        h = 1e-2 * max(1.0, abs(sig[i]))
        sp, sm = sig.copy(), sig.copy()
        sp[i] += h; sm[i] -= h
        fd = (L(sp, raws) - L(sm, raws)) / (2 * h)
        assert abs(fd - ds[i]) <= 2e-3 * max(1e-3, abs(fd)) + 1e-4, (i, fd, ds[i])
        for c in range(3):
            rp, rm = raws.copy(), raws.copy()
            rp[i, c] += 1e-2; rm[i, c] -= 1e-2
            fd = (L(sig, rp) - L(sig, rm)) / 2e-2
            assert abs(fd - dr[i, c]) <= 1e-3 * max(1e-3, abs(fd)) + 1e-5


def test_hashgrid_c_statement_matches_torch():
    """oracle/hashgrid_ref.c (the PSNR-ensemble trainer's encoding) vs field_ref.hash_encode (the
    primary torch statement): forward to f32 rounding of the 8-corner sum order, backward scatter
    with the identical non-zero set (box corners, the centre and random points at table init 0.5)."""
    import torch
    from oracle import field_ref as F
    P, levels = F.init_params(seed=3, table_init=0.5)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(20000, 3, generator=g) * 0.98 - 0.49
    x[:5] = torch.tensor([[-0.5, -0.5, -0.5], [0.5, 0.5, 0.5], [0, 0, 0], [0.4999, -0.25, 0.125], [-0.3, 0.3, 0.0]])
    x01 = x + 0.5
    t1 = P.table.clone().requires_grad_(True)
    t2 = P.table.clone().requires_grad_(True)
    a = F.hash_encode(x01, t1, levels)
    b = F.encode(x01, t2, levels, "c")
    assert float((a - b).abs().max()) <= 2e-7 * max(1.0, float(a.abs().max()))
    gup = torch.randn(a.shape, generator=g)
    a.backward(gup)
    b.backward(gup)
    assert torch.equal(t1.grad != 0, t2.grad != 0)
    assert float((t1.grad - t2.grad).abs().max()) <= 1e-6 * float(t1.grad.abs().max())


def test_mt19937_vectorised_draws():
    """losses_ref.Mt19937.draws (vectorised twist + tempering) == the scalar generator, and the
    C++ standard's known answer (the 10 000th output of default-seeded mt19937 is 4123659995)."""
    from oracle.losses_ref import Mt19937
    for seed in (0, 1234, 2 ** 31 + 7):
        a, b = Mt19937(seed), Mt19937(seed)
        x = np.array([a() for _ in range(1500)], np.uint64)
        y = np.concatenate([b.draws(700), b.draws(1), b.draws(799)])
        assert np.array_equal(x, y)
    assert int(Mt19937(5489).draws(10000)[-1]) == 4123659995
