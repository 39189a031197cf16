"""Parity of the HIP `vren` kernels (through the C ABI) with the CPU oracle (oracle/vren_ref.c).

Bit-exact: ray/AABB hits, the marcher (rays_a, xyzs, dirs, deltas, ts, counter), morton, packbits.
fp32 tolerance (stated per test): compositing forward/backward (the HIP transmittance is a wave
product scan, the oracle a serial product; __expf vs expf).
"""
import numpy as np
import pytest
import torch

from oracle import vren_ref
from ncnerf_amd import vren
from ncnerf_amd.synthetic import SyntheticScene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene():
    return SyntheticScene()


def _edge_rays(rng, n):
    """Random rays plus the reference edge cases: misses, starts inside, axis-parallel (1/d = inf)."""
    o = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 8, 1:] = 0.0  # parallel to x
    d[n // 8: n // 4, 0] = 0.0  # in the yz plane
    o[n // 4: n // 3] = rng.uniform(-0.2, 0.2, (n // 3 - n // 4, 3))  # inside the box
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


def test_ray_aabb_bitexact(dev):
    rng = np.random.default_rng(0)
    o, d = _edge_rays(rng, 4096)
    for V, M in ((1, 1), (5, 3), (9, 9)):
        c = rng.uniform(-0.5, 0.5, (V, 3)).astype(np.float32)
        h = rng.uniform(0.05, 0.5, (V, 3)).astype(np.float32)
        if V == 1:
            c[:] = 0; h[:] = 0.5
        out = vren.ray_aabb_intersect(*(torch.from_numpy(a).to(dev) for a in (o, d, c, h)), M)
        ref = vren_ref.ray_aabb_intersect(o, d, c, h, M)
        for a, r in zip(out, ref):
            assert np.array_equal(a.cpu().numpy(), r, equal_nan=True)


def test_morton_packbits_bitexact(dev):
    rng = np.random.default_rng(1)
    coords = rng.integers(0, 1024, (100000, 3)).astype(np.int32)
    m = vren.morton3D(torch.from_numpy(coords).to(dev))
    assert np.array_equal(m.cpu().numpy(), vren_ref.morton3D(coords))
    inv = vren.morton3D_invert(m)
    assert np.array_equal(inv.cpu().numpy(), vren_ref.morton3D_invert(m.cpu().numpy()))
    assert np.array_equal(inv.cpu().numpy(), coords)
    grid = rng.normal(size=(1, 128 ** 3)).astype(np.float32)
    bf = torch.zeros(128 ** 3 // 8, dtype=torch.uint8, device=dev)
    vren.packbits(torch.from_numpy(grid).to(dev), 0.3, bf)
    assert np.array_equal(bf.cpu().numpy(), vren_ref.packbits(grid, 0.3))
    vren.packbits(torch.from_numpy(grid).to(dev), float("nan"), bf)  # quirk q12: NaN threshold clears
    assert int(bf.sum()) == 0


def _march_inputs(scene, n, seed, dev, edge=False):
    rng = np.random.default_rng(seed)
    if edge:
        o, d = _edge_rays(rng, n)
    else:
        b = scene.batch(((n + 63) // 64) * 64, seed)
        o, d = b["rays_o"][:n].copy(), b["rays_d"][:n].copy()
    _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
    ht = ht[:, 0].copy()
    near = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)  # rendering.py:28 near clamp
    ht[near, 0] = 0.01
    noise = rng.random(n, dtype=np.float32)
    return o, d, ht, noise


@pytest.mark.parametrize("n,edge,ms", [(8192, False, 1024), (2048, True, 1024), (777, False, 64), (1, False, 1024)])
def test_raymarching_train_bitexact(dev, scene, n, edge, ms):
    o, d, ht, noise = _march_inputs(scene, n, 7 + n, dev, edge)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    bf = T(scene.bitfield)
    out = vren.raymarching_train(T(o), T(d), T(ht), bf, 1, 0.5, 0.0, T(noise), 128, ms)
    ref = vren_ref.raymarching_train(o, d, ht, scene.bitfield, 1, 0.5, 0.0, noise, 128, ms)
    names = ("rays_a", "xyzs", "dirs", "deltas", "ts", "counter")
    for a, r, name in zip(out, ref, names):
        a = a.cpu().numpy()
        assert a.shape == r.shape, name
        assert np.array_equal(a, r), f"{name}: {np.argwhere(a != r)[:5]}"
    if not edge and n >= 2048:
        S = int(ref[5][0])
        assert 20 < S / n < 1024, f"unexpected samples/ray {S / n}"


def _march_uniform_np(seed, ctr, n):
    """numpy restatement of march_uniform (csrc/vren.hip): splitmix64 of (seed, counter, ray)."""
    M = (1 << 64) - 1
    out = np.empty(n, np.float32)
    for r in range(n):
        z = (seed + 0x9E3779B97F4A7C15 * ((ctr * 0x100000001B3 + r + 1) & M)) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out[r] = np.float32((z >> 40) * (1.0 / 16777216.0))
    return out


class _Box:
    """The attributes march_train_fused reads from the model."""
    def __init__(self, bitfield):
        self._aabb = ((0.0, 0.0, 0.0), (0.5, 0.5, 0.5))
        self.density_bitfield, self.cascades, self.scale, self.grid_size = bitfield, 1, 0.5, 128


@pytest.mark.parametrize("n,edge,ms", [(8192, False, 1024), (2048, True, 1024), (777, False, 64), (1, False, 1024),
                                       (3, True, 1024)])
def test_fused_marcher_bitexact(dev, scene, n, edge, ms):
    """ncn_march_train_fused (intersect + near clamp + jitter + walk, then placement + pack: two
    launches) == the oracle's ray_aabb_intersect + near clamp + raymarching_train, bit for bit; the
    device RNG path == the oracle fed the same uniforms; repeated launches give identical results."""
    from ncnerf_amd.rendering import march_train_fused
    o, d, ht, noise = _march_inputs(scene, n, 11 + n, dev, edge)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    box = _Box(T(scene.bitfield))
    names = ("rays_a", "xyzs", "dirs", "deltas", "ts", "counter")
    ref = vren_ref.raymarching_train(o, d, ht, scene.bitfield, 1, 0.5, 0.0, noise, 128, ms)
    S = int(ref[5][0])
    for rep in range(3):
        out = march_train_fused(box, T(o), T(d), 0.01, ms, noise=T(noise))
        torch.cuda.synchronize()
        ra = out["rays_a"].cpu().numpy()
        # row order: rays with > 256 samples first, each class in ray order (any row order is the
        # reference's contract: its rows come in atomicAdd order)
        long_ = ra[:, 2] > 256
        nl = int(long_.sum())
        assert long_[:nl].all() and not long_[nl:].any()
        assert np.all(np.diff(ra[:nl, 0]) > 0) and np.all(np.diff(ra[nl:, 0]) > 0)
        for name, r in zip(names, ref):
            a = out[name].cpu().numpy()
            if name == "rays_a":
                a = a[np.argsort(a[:, 0], kind="stable")]
            if name in ("xyzs", "dirs", "deltas", "ts"):
                a = a[:S]
            assert np.array_equal(a, r), f"rep {rep} {name}: {np.argwhere(a != r)[:5]}"
    # device RNG: (seed, counter) -> the same uniforms as the numpy restatement
    seed, step = 1234567891234, 42
    out = march_train_fused(box, T(o), T(d), 0.01, ms, rng=(seed, torch.tensor(step, device=dev)))
    ref = vren_ref.raymarching_train(o, d, ht, scene.bitfield, 1, 0.5, 0.0, _march_uniform_np(seed, step, n), 128, ms)
    S = int(ref[5][0])
    for name, r in zip(names, ref):
        a = out[name].cpu().numpy()
        if name == "rays_a":
            a = a[np.argsort(a[:, 0], kind="stable")]
        if name in ("xyzs", "dirs", "deltas", "ts"):
            a = a[:S]
        assert np.array_equal(a, r), f"rng {name}"


def test_raymarching_train_exp_step_and_cascades(dev, scene):
    """exp_step_factor > 0 and cascades > 1 (scale 1.0 -> C=2) take the general mip path."""
    rng = np.random.default_rng(3)
    n = 1024
    o, d = _edge_rays(rng, n)
    o *= 2
    _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 1.0, np.float32), 1)
    ht = ht[:, 0].copy()
    noise = rng.random(n, dtype=np.float32)
    bf = np.concatenate([scene.bitfield, np.roll(scene.bitfield, 1000)])  # C=2 cascades
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.raymarching_train(T(o), T(d), T(ht), T(bf), 2, 1.0, 1 / 256, T(noise), 128, 1024)
    ref = vren_ref.raymarching_train(o, d, ht, bf, 2, 1.0, 1 / 256, noise, 128, 1024)
    for a, r in zip(out, ref):
        assert np.array_equal(a.cpu().numpy(), r)


def test_raymarching_test_bitexact(dev, scene):
    o, d, ht, _ = _march_inputs(scene, 3000, 11, dev)
    alive = np.arange(0, 3000, 2, dtype=np.int64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ht_dev = T(ht)
    ht_ref = ht.copy()
    for N in (1, 4, 64):
        out = vren.raymarching_test(T(o), T(d), ht_dev, T(alive), T(scene.bitfield), 1, 0.5, 0.0, 128, 1024, N)
        ref = vren_ref.raymarching_test(o, d, ht_ref, alive, scene.bitfield, 1, 0.5, 0.0, 128, 1024, N)
        for a, r in zip(out, ref):
            assert np.array_equal(a.cpu().numpy(), r)
        assert np.array_equal(ht_dev.cpu().numpy(), ht_ref)  # hits_t mutation (raymarching.cu:390)


def _composite_inputs(scene, n_rays, seed, sigma_scale=20.0, C=3):
    o, d, ht, noise = _march_inputs(scene, n_rays, seed, None)
    rays_a, xyzs, dirs, deltas, ts, counter = vren_ref.raymarching_train(o, d, ht, scene.bitfield, 1, 0.5, 0.0,
                                                                         noise, 128, 1024)
    rng = np.random.default_rng(seed + 1)
    S = int(counter[0])
    sig = np.abs(rng.normal(0, sigma_scale, S)).astype(np.float32)
    raws = rng.random((S, C), dtype=np.float32)
    return rays_a, deltas, ts, sig, raws


@pytest.mark.parametrize("sigma_scale", [20.0, 400.0, 0.0])
def test_composite_fw_parity(dev, scene, sigma_scale):
    """Tolerance: |Δ| <= 2e-5 + 2e-4*|ref| on opacity/depth/rend/ws; total_samples may differ by one
    sample only where the stop is borderline (T within 1e-3 relative of T_threshold)."""
    rays_a, deltas, ts, sig, raws = _composite_inputs(scene, 4096, 5, sigma_scale)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(rays_a), 1e-4)
    ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, 1e-4)
    tot, ref_tot = out[0].cpu().numpy(), ref[0]
    assert np.mean(tot == ref_tot) > 0.999 and np.max(np.abs(tot - ref_tot)) <= 1
    for a, r, name in zip(out[1:], ref[1:], ("opacity", "depth", "rend", "ws")):
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=2e-4, atol=2e-5, err_msg=name)


def test_composite_fw_edge(dev):
    """Empty segments (N=0), a single sample, an immediately opaque first sample."""
    rays_a = np.array([[0, 0, 0], [1, 0, 1], [2, 1, 3], [3, 4, 0], [4, 4, 300]], np.int64)
    S = 304
    rng = np.random.default_rng(0)
    sig = rng.random(S, dtype=np.float32) * 10
    sig[1] = 1e6  # opaque first sample of ray 2
    raws = rng.random((S, 3), dtype=np.float32)
    deltas = np.full(S, 1.7e-3, np.float32)
    ts = np.cumsum(deltas).astype(np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(rays_a), 1e-4)
    ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, 1e-4)
    assert np.array_equal(out[0].cpu().numpy(), ref[0])
    for a, r in zip(out[1:], ref[1:]):
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=2e-4, atol=2e-5)


def _long_first_inputs(seed, extra_long=0):
    """Segments of 257..1025 samples in the rows at the front of rays_a (the training step's row
    order: the compositors take them with one workgroup each), with transmittance that stops in
    each of the 4 waves' sample ranges or never; then short rays."""
    rng = np.random.default_rng(seed)
    lens = [257, 300, 511, 512, 513, 700, 768, 769, 1000, 1024, 1025, 1024, 600, 400] + list(rng.integers(0, 256, 200))
    lens += list(rng.integers(257, 1100, extra_long))  # more long rays than the compositors' 256 workgroups
    stop_at = [None, 100, 280, 500, None, 600, 260, 767, 900, None, 1010, 1023, None, 390]
    rows, start, sig_parts = [], 0, []
    for i, n in enumerate(lens):
        n = int(n)
        rows.append([i, start, n])
        s = np.abs(rng.normal(0, 0.2, n)).astype(np.float32)  # T stays well above 1e-4 ...
        if i < len(stop_at) and stop_at[i] is not None and stop_at[i] < n:
            s[stop_at[i]] = 1e5  # ... until an opaque sample
        elif i >= len(stop_at) and n > 256:  # the extra long rays: an opaque sample anywhere, or none (no borderline stops)
            k = int(rng.integers(0, 2 * n))
            if k < n:
                s[k] = 1e5
        elif i >= len(stop_at):
            s = np.abs(rng.normal(0, 20, n)).astype(np.float32)
        sig_parts.append(s)
        start += n
    order = rng.permutation(len(rows))  # segments not in row order (rows of the step: long first, ray order)
    rays_a = np.array(rows, np.int64)
    perm = np.concatenate([order[rays_a[order, 2] > 256], order[rays_a[order, 2] <= 256]])
    rays_a = rays_a[perm]
    S = start
    sig = np.concatenate(sig_parts)
    raws = rng.random((S, 3), dtype=np.float32)
    deltas = np.full(S, 1.7e-3, np.float32)
    ts = (np.arange(S) % 977 * 1.7e-3).astype(np.float32)
    return rays_a, deltas, ts, sig, raws


@pytest.mark.parametrize("extra_long", [0, 600])
def test_composite_long_rays_workgroup_path(dev, extra_long):
    """Rays of 257..1024 samples at the front of rays_a go through the one-workgroup-per-ray path
    (> 1024 stays single-wave; 600 extra long rays: workgroups take several rows each): fw exact
    counts and 2e-4 values, bw at the parity tolerance."""
    rays_a, deltas, ts, sig, raws = _long_first_inputs(3, extra_long)
    T = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(rays_a), 1e-4)
    ref = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, 1e-4)
    assert np.array_equal(out[0].cpu().numpy(), ref[0])
    for a, r, name in zip(out[1:], ref[1:], ("opacity", "depth", "rend", "ws")):
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=2e-4, atol=2e-5, err_msg=name)
    # rows in ray order (the eager marcher's): long rays on the single-wave path, bit-identical
    by_ray = rays_a[np.argsort(rays_a[:, 0])]
    out2 = vren.composite_train_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(by_ray), 1e-4)
    for a, b_ in zip(out, out2):
        assert torch.equal(a, b_)
    _, O, D, RE, ws = ref
    rng = np.random.default_rng(4)
    R, S = rays_a.shape[0], sig.shape[0]
    dO, dD = rng.normal(size=R).astype(np.float32), rng.normal(size=R).astype(np.float32)
    dR = rng.normal(size=(R, 3)).astype(np.float32)
    for dW in (None, rng.normal(size=S).astype(np.float32)):
        o2 = vren.composite_train_multi_bw(T(dO), T(dD), T(dR), T(dW), T(sig), T(raws), T(ws), T(deltas), T(ts),
                                           T(rays_a), T(O), T(D), T(RE), 1e-4)
        r2 = vren_ref.composite_train_multi_bw(dO, dD, dR, dW, sig, raws, ws, deltas, ts, rays_a, O, D, RE, 1e-4)
        for a, r, name in zip(o2, r2, ("dL_dsigmas", "dL_draws")):
            np.testing.assert_allclose(a.cpu().numpy(), r, rtol=1e-3, atol=1e-4 * np.abs(r).max(), err_msg=name)


@pytest.mark.parametrize("with_dws", [False, True])
def test_composite_bw_parity(dev, scene, with_dws):
    """Tolerance: |Δ| <= 1e-4*max|ref| + 1e-3*|ref| (cancellation in (R - r) terms)."""
    rays_a, deltas, ts, sig, raws = _composite_inputs(scene, 2048, 9, 20.0)
    ref_fw = vren_ref.composite_train_multi_fw(sig, raws, deltas, ts, rays_a, 1e-4)
    _, O, D, RE, ws = ref_fw
    rng = np.random.default_rng(2)
    R, S = rays_a.shape[0], sig.shape[0]
    dO = rng.normal(size=R).astype(np.float32)
    dD = rng.normal(size=R).astype(np.float32)
    dR = rng.normal(size=(R, 3)).astype(np.float32)
    dW = rng.normal(size=S).astype(np.float32) if with_dws else None
    T = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = vren.composite_train_multi_bw(T(dO), T(dD), T(dR), T(dW), T(sig), T(raws), T(ws), T(deltas), T(ts),
                                        T(rays_a), T(O), T(D), T(RE), 1e-4)
    ref = vren_ref.composite_train_multi_bw(dO, dD, dR, dW, sig, raws, ws, deltas, ts, rays_a, O, D, RE, 1e-4)
    for a, r, name in zip(out, ref, ("dL_dsigmas", "dL_draws")):
        a = a.cpu().numpy()
        np.testing.assert_allclose(a, r, rtol=1e-3, atol=1e-4 * np.abs(r).max(), err_msg=name)


def test_composite_test_parity(dev, scene):
    rng = np.random.default_rng(4)
    A, N, R = 2000, 8, 3000
    alive = np.sort(rng.choice(R, A, replace=False)).astype(np.int64)
    sig = np.abs(rng.normal(0, 50, (A, N))).astype(np.float32)
    raws = rng.random((A, N, 3), dtype=np.float32)
    deltas = np.full((A, N), 1.7e-3, np.float32)
    ts = rng.random((A, N), dtype=np.float32)
    n_eff = rng.integers(0, N + 1, A).astype(np.int32)
    op = rng.random(R, dtype=np.float32) * 0.5
    de = rng.random(R, dtype=np.float32)
    re = rng.random((R, 3), dtype=np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    al_d, op_d, de_d, re_d = T(alive), T(op), T(de), T(re)
    vren.composite_test_multi_fw(T(sig), T(raws), T(deltas), T(ts), T(np.zeros((R, 2), np.float32)), al_d, 1e-4,
                                 T(n_eff), op_d, de_d, re_d)
    al_r, op_r, de_r, re_r = alive.copy(), op.copy(), de.copy(), re.copy()
    vren_ref.composite_test_multi_fw(sig, raws, deltas, ts, None, al_r, 1e-4, n_eff, op_r, de_r, re_r)
    assert np.array_equal(al_d.cpu().numpy(), al_r)
    for a, r in ((op_d, op_r), (de_d, de_r), (re_d, re_r)):
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=1e-5, atol=1e-6)


def test_check_input_errors(dev):
    """CHECK_INPUT semantics (utils.h:4-6): CPU or non-contiguous tensors raise RuntimeError."""
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        vren.morton3D(x.int())
    y = torch.zeros(3, 4, dtype=torch.int32, device=dev).t()
    with pytest.raises(RuntimeError, match="must be contiguous"):
        vren.morton3D(y)


def test_ray_aabb_near_clamp_fused(dev):
    """ncn_ray_aabb_intersect_near == intersect + render()'s masked clamp of hits_t[:,0,0] (bit-exact)."""
    rng = np.random.default_rng(7)
    o, d = _edge_rays(rng, 4096)
    c, h = np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32)
    T = lambda a: torch.from_numpy(a).to(dev)
    for near in (0.01, 0.3):
        a = vren.ray_aabb_intersect(T(o), T(d), T(c), T(h), 1, near_distance=near)
        b = vren.ray_aabb_intersect(T(o), T(d), T(c), T(h), 1)
        t0 = b[1][:, 0, 0]
        t0.masked_fill_((t0 >= 0) & (t0 < near), near)
        assert (t0 == near).any()
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_composite_background_fused(dev, scene):
    """VolumeRendererBg (background blend inside the compositor) == VolumeRenderer + the torch
    blend of rendering.py:232-240: forward bit-exact, gradients within fp32 rounding (the opacity
    term -bg*sum(dL/drgb) is added inside the kernel instead of by autograd)."""
    from ncnerf_amd.custom_functions import VolumeRenderer, VolumeRendererBg
    rays_a, deltas, ts, sig, raws = _composite_inputs(scene, 2048, 11, 20.0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rng = np.random.default_rng(3)
    R = rays_a.shape[0]
    g_rgb, g_op, g_d = (T(rng.normal(size=s).astype(np.float32)) for s in ((R, 3), (R,), (R,)))
    res = []
    for fused in (False, True):
        s_, r_ = T(sig).requires_grad_(True), T(raws).requires_grad_(True)
        if fused:
            _, op, dp, rgb, _ = VolumeRendererBg.apply(s_, r_, T(deltas), T(ts), T(rays_a), 1e-4, 1.0)
        else:
            _, op, dp, rend, _ = VolumeRenderer.apply(s_, r_, T(deltas), T(ts), T(rays_a), 1e-4)
            rgb = rend + (1 - op)[:, None]
        ((rgb * g_rgb).sum() + (op * g_op).sum() + (dp * g_d).sum()).backward()
        res.append((rgb.detach(), op.detach(), s_.grad, r_.grad))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for a, b in zip(res[0][2:], res[1][2:]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * float(a.abs().max()))


def _assert_segment_sums(rays_a, ts, gx, gd, got_o, got_d):
    """HIP segment sums vs the oracle's sequential segment_csr, row by row within the fp32
    summation-order bound: two orders of the same n f32 terms differ by at most
    2 (n - 1) 2^-24 sum|terms| (each sum's error is <= (n - 1) u sum|terms|, u = 2^-24, to first order).
    A bound relative to the result would ignore cancellation: a row that cancels to 0.08 from terms
    of order 1 carries ~1e-5 of order noise (the round-5 driver failure)."""
    ra = np.asarray(rays_a)
    indptr = np.concatenate([ra[:, 1], ra[-1:, 1] + ra[-1:, 2]])
    gx = np.zeros((ts.shape[0], 3), np.float32) if gx is None else np.asarray(gx, np.float32)
    gd = np.zeros((ts.shape[0], 3), np.float32) if gd is None else np.asarray(gd, np.float32)
    ref_o, ref_d = vren_ref.raymarcher_backward(ra, ts, gx, gd)
    term_d = gx * np.asarray(ts, np.float32)[:, None] + gd
    abs_o = vren_ref.segment_csr(np.abs(gx), indptr).astype(np.float64)
    abs_d = vren_ref.segment_csr(np.abs(term_d), indptr).astype(np.float64)
    n = np.maximum(indptr[1:] - indptr[:-1], 1).astype(np.float64)[:, None]
    for got, ref, ab, what in ((got_o, ref_o, abs_o, "dL/drays_o"), (got_d, ref_d, abs_d, "dL/drays_d")):
        bound = 2.0 * (n - 1) * 2.0 ** -24 * ab * 1.01 + 1e-30
        err = np.abs(np.asarray(got, np.float64) - ref.astype(np.float64))
        bad = np.argwhere(err > bound)
        assert bad.size == 0, (f"{what}: {len(bad)} elements outside 2(n-1)u*sum|terms|; first {bad[:3].tolist()}: "
                               f"got {np.asarray(got)[tuple(bad[0])]} ref {ref[tuple(bad[0])]} "
                               f"bound {bound[tuple(bad[0])]}")


@pytest.mark.parametrize("n", [512, 1])
def test_raymarcher_backward_segment_csr(dev, scene, n):
    """RayMarcher.backward (custom_functions.py:102-112) against the reference's segment_csr
    restated (oracle.vren_ref.raymarcher_backward), incl. rays with no samples; against the
    geometry it differentiates (xyzs = o + t*d, dirs = d); and run to run: the HIP segment sum has a
    fixed order, so a second backward is bit-identical."""
    from ncnerf_amd.custom_functions import RayMarcher
    o, d, ht, noise = _march_inputs(scene, n, 3 + n, dev)
    if n > 1:
        ht[n // 2] = -1.0  # a missed ray (q9): an empty segment in the middle
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ro, rd = T(o).requires_grad_(), T(d).requires_grad_()
    rays_a, xyzs, dirs, deltas, ts, total = RayMarcher.apply(ro, rd, T(ht), T(scene.bitfield), 1, 0.5, 0.0, 128, 1024,
                                                             T(noise))
    g = torch.Generator(device=dev).manual_seed(n)
    wx = torch.randn(xyzs.shape, device=dev, generator=g)
    wd = torch.randn(dirs.shape, device=dev, generator=g)
    loss = (xyzs * wx).sum() + (dirs * wd).sum()
    loss.backward(retain_graph=True)
    g_o, g_d = ro.grad.clone(), rd.grad.clone()
    ro.grad = rd.grad = None
    loss.backward()
    assert torch.equal(ro.grad, g_o) and torch.equal(rd.grad, g_d), "RayMarcher.backward is not deterministic"
    _assert_segment_sums(rays_a.cpu().numpy(), ts.detach().cpu().numpy(), wx.cpu().numpy(), wd.cpu().numpy(),
                         g_o.cpu().numpy(), g_d.cpu().numpy())
    if n > 1:
        assert int(rays_a[n // 2, 2]) == 0 and float(ro.grad[n // 2].abs().sum()) == 0.0
        # rows are rays in ray order, so segment i is ray i's samples: d/do (o + t d) = I, d/dd = t I
        ra = rays_a.cpu().numpy()
        i = int(np.argmax(ra[:, 2]))
        s0, c = int(ra[i, 1]), int(ra[i, 2])
        w = wx[s0:s0 + c].cpu().numpy().astype(np.float64)
        bound = 2.0 * c * 2.0 ** -24 * np.abs(w).sum(0) * 1.01
        assert np.all(np.abs(ro.grad[i].cpu().numpy() - w.sum(0)) <= bound)


def test_segment_csr_ragged(dev):
    """ncn_segment_csr alone on hand-built segments: empty segments in the middle and at the end, a
    one-sample segment, segments just around the 64-lane width, and segments longer than 1024 and
    than 4096 samples; gradients of both kinds, one of them absent (None = zero), and the reference's
    indptr rule (a segment ends where the next row starts)."""
    from ncnerf_amd import vren
    lens = [3, 0, 1, 63, 64, 65, 1500, 0, 4100, 2, 0]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    S = int(np.sum(lens)) + 7  # trailing samples that belong to no segment
    ra = np.stack([np.arange(len(lens)), starts, np.asarray(lens)], 1).astype(np.int64)
    rng = np.random.default_rng(11)
    ts = rng.uniform(0.0, 3.0, S).astype(np.float32)
    gx = rng.normal(size=(S, 3)).astype(np.float32)
    gd = rng.normal(size=(S, 3)).astype(np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    for x, y in ((gx, gd), (gx, None), (None, gd)):
        d_o, d_d = vren.raymarching_train_backward(None if x is None else T(x), None if y is None else T(y), T(ts),
                                                   T(ra))
        d_o2, d_d2 = vren.raymarching_train_backward(None if x is None else T(x), None if y is None else T(y), T(ts),
                                                     T(ra))
        torch.cuda.synchronize()
        assert torch.equal(d_o, d_o2) and torch.equal(d_d, d_d2)
        _assert_segment_sums(ra, ts, x, y, d_o.cpu().numpy(), d_d.cpu().numpy())
        for i in np.flatnonzero(np.asarray(lens) == 0):
            assert float(d_o[i].abs().sum()) == 0.0 and float(d_d[i].abs().sum()) == 0.0
    with pytest.raises(RuntimeError):
        bad = ra.copy()
        bad[-1, 2] = 100  # past the last sample
        vren.raymarching_train_backward(T(gx), T(gd), T(ts), T(bad))
