"""Occupancy-grid maintenance restated in numpy — TEST INFRASTRUCTURE (oracle), never imported by
the product path.

* `mark_invisible_cells`: reference models/ngp_mt.py:274-337 (pinhole-K branch), numpy f32.
* `grid_refresh`: reference models/ngp_mt.py:340-368 (update_density_grid) with the cell sampling
  of ngp_mt.py:245-262 replaced by the documented deviation of csrc/grid.hip,
  or (sampling="reference") the reference's own draws (`reference_cells`):
  every cell is hit independently with the marginal probability of the reference's M uniform +
  M occupied draws with replacement, decided by the same counter-based hash of (seed, cell, stream)
  as the device (`gr_uniform`, grid.hip), and the hit cells' jitter drawn from the same hash.
  Given the same grid, seed and densities the HIP refresh and this one agree bit for bit on the
  hit set and the positions; the density itself comes from the caller (`density_fn`).

Parity: the update rule, threshold and packbits are pinned against the reference's own formulas
(vren_ref.density_grid_update, tests/test_gpu_grid.py); the hash is this repo's own (no reference
counterpart), so the sampling is pinned only to its marginal probabilities.
"""
import numpy as np

from . import vren_ref

M32 = np.uint64(0xFFFFFFFF)


def _u32(x):
    return (np.asarray(x, np.uint64) & M32).astype(np.uint64)


def gr_uniform(seed, cells, stream):
    """grid.hip gr_uniform: murmur3-finaliser hash of (seed, cell, stream) -> f32 in [0, 1), 24 bits."""
    seed = int(seed) % (1 << 64)
    c = np.asarray(cells, np.uint64)
    lo, hi = np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32)
    h = _u32(c * np.uint64(0x9E3779B1) + np.uint64((int(stream) * 0x85EBCA77) & 0xFFFFFFFF))
    h = lo ^ h
    h ^= h >> np.uint64(16); h = _u32(h * np.uint64(0x85EBCA6B))
    h ^= h >> np.uint64(13); h = _u32(h * np.uint64(0xC2B2AE35))
    h ^= h >> np.uint64(16)
    h = _u32(h + hi)
    h ^= h >> np.uint64(15); h = _u32(h * np.uint64(0x2C1B3C6D))
    h ^= h >> np.uint64(12); h = _u32(h * np.uint64(0x297A2D39))
    h ^= h >> np.uint64(15)
    return (h >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def mark_invisible_cells(K, poses, img_wh, near_distance, grid_size, scale, cascades=1, chunk=64 ** 3):
    """ngp_mt.py:274-337, pinhole branch: returns (density_grid (C, G^3) f32 with 0 for cells seen by
    some camera and not too near any of them, -1 otherwise; count_grid (C, G^3) f32)."""
    G = grid_size
    N = G ** 3
    poses = np.asarray(poses, np.float32)
    K = np.asarray(K, np.float32)
    n_cams = poses.shape[0]
    w2c_R = np.transpose(poses[:, :3, :3], (0, 2, 1))  # ngp_mt.py:286
    w2c_T = -w2c_R @ poses[:, :3, 3:]  # :287
    r = np.arange(G, dtype=np.int32)
    zz, yy, xx = np.meshgrid(r, r, r, indexing="ij")
    coords = np.stack([xx, yy, zz], -1).reshape(-1, 3)  # train_nerf.py grid_coords (kornia order)
    indices = vren_ref.morton3D(coords).astype(np.int64)
    density = np.zeros((cascades, N), np.float32)
    count = np.zeros((cascades, N), np.float32)
    for c in range(cascades):
        for i in range(0, N, chunk):
            xyzs = coords[i:i + chunk].astype(np.float32) / np.float32(G - 1) * np.float32(2) - np.float32(1)  # :302
            s = min(2 ** (c - 1), scale)
            half_grid_size = s / G
            xyzs_w = (xyzs * np.float32(s - half_grid_size)).T  # :305
            xyzs_c = w2c_R @ xyzs_w + w2c_T  # :306
            uvd = K @ xyzs_c  # :309
            uv = uvd[:, :2] / uvd[:, 2:]
            in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < img_wh[0]) & (uv[:, 1] >= 0) & \
                (uv[:, 1] < img_wh[1])  # :320-321
            covered = (uvd[:, 2] >= near_distance) & in_image
            cnt = (covered.sum(0) / np.float32(n_cams)).astype(np.float32)  # :323-324
            count[c, indices[i:i + chunk]] = cnt
            too_near = (uvd[:, 2] < near_distance) & in_image  # :326
            valid = (cnt > 0) & ~too_near.any(0)
            density[c, indices[i:i + chunk]] = np.where(valid, np.float32(0), np.float32(-1))  # :327-328
    return density, count


def hit_cells(grid_c, thr, warmup, seed):
    """grid.hip grid_occ + grid_select hit test: the Morton-ordered indices of the hit cells."""
    N = grid_c.shape[0]
    cells = np.arange(N, dtype=np.uint64)
    if warmup:
        return cells.astype(np.int64)
    M = N // 4
    p_u = np.float32(-np.expm1(M * np.log1p(-1.0 / N)))
    n_occ = int((grid_c > np.float32(thr)).sum())
    p_o = np.float32(-np.expm1(M * np.log1p(-1.0 / n_occ))) if n_occ > 0 else np.float32(0)
    hit = (gr_uniform(seed, cells, 0) < p_u) | ((grid_c > np.float32(thr)) & (gr_uniform(seed, cells, 1) < p_o))
    return np.nonzero(hit)[0].astype(np.int64)


def hit_positions(cells, seed, grid_size, s):
    """Jittered world positions of the hit cells (grid.hip grid_select pass 2; ngp_mt.py:346-349)."""
    G = grid_size
    hg = np.float32(s / G)
    s_hg = np.float32(s - s / G)
    coords = vren_ref.morton3D_invert(np.asarray(cells, np.int32)).astype(np.float32)
    out = np.empty((len(cells), 3), np.float32)
    for q in range(3):
        u = gr_uniform(seed, np.asarray(cells, np.uint64), 2 + q)
        x = coords[:, q] / np.float32(G - 1)
        x = x * np.float32(2) - np.float32(1)
        x = x * s_hg
        out[:, q] = x + (u * np.float32(2) - np.float32(1)) * hg
    return out


def reference_cells(grid_c, thr, seed, grid_size):
    """sample_uniform_and_occupied_cells (ngp_mt.py:244-270) for one cascade, the reference's own
    draws: M = G^3 / 4 uniform cells (random integer coordinates, with replacement) and M draws with
    replacement from the cells above the threshold; numpy's generator seeded by `seed` stands in for
    torch's device RNG.  Returns (Morton indices, integer coordinates) in the reference's order."""
    G = grid_size
    M = G ** 3 // 4
    rng = np.random.default_rng(int(seed) % 2 ** 63)
    coords1 = rng.integers(0, G, (M, 3)).astype(np.int32)
    idx1 = vren_ref.morton3D(coords1).astype(np.int64)
    occ = np.nonzero(grid_c > np.float32(thr))[0]
    idx2 = occ[rng.integers(0, len(occ), M)] if len(occ) > 0 else occ
    coords2 = vren_ref.morton3D_invert(idx2.astype(np.int32)).reshape(-1, 3)
    return np.concatenate([idx1, idx2]), np.concatenate([coords1, coords2]).astype(np.float32), rng


def grid_refresh(grid, density_fn, threshold, warmup, seed, grid_size, scale, decay=0.95, sampling="device"):
    """update_density_grid (ngp_mt.py:340-368): returns (new grid (C, G^3) f32, threshold used,
    bitfield).  `density_fn(xyzs (n,3) f32) -> (n,) f32`.  sampling "device": the HIP refresh's
    (every cell hit independently with the marginal probability of the reference's draws, DESIGN
    deviation 7); "reference": the reference's M uniform + M occupied draws with replacement
    (reference_cells), each drawn cell at its own jittered position, a cell drawn twice keeping the
    last draw's density (the assignment density_grid_tmp[c, indices] = ... of ngp_mt.py:353)."""
    g = np.array(grid, np.float32, copy=True)
    C = g.shape[0]
    for c in range(C):
        s = min(2 ** (c - 1), scale)
        sc = (int(seed) + 0x9E3779B97F4A7C15 * c) % 2 ** 64
        tmp = np.zeros(g.shape[1], np.float32)
        if sampling == "reference" and not warmup:
            cells, coords, rng = reference_cells(g[c], threshold, sc, grid_size)
            hg = np.float32(s / grid_size)
            xyzs = (coords / np.float32(grid_size - 1) * np.float32(2) - np.float32(1)) * np.float32(s - s / grid_size)
            xyzs = (xyzs + (rng.random(xyzs.shape, dtype=np.float32) * np.float32(2) - np.float32(1)) * hg)
            tmp[cells] = np.asarray(density_fn(xyzs.astype(np.float32)), np.float32)  # (last write wins)
        else:
            cells = hit_cells(g[c], threshold, warmup, sc)
            tmp[cells] = np.asarray(density_fn(hit_positions(cells, sc, grid_size, s)), np.float32)
        v = g[c]
        # torch.maximum semantics (NaN propagates) as grid.hip's torch_max
        g[c] = np.where(v < 0, v, np.maximum(v * np.float32(decay), tmp)).astype(np.float32)
    pos = g[g > 0]
    mean = np.float32(pos.astype(np.float64).sum() / pos.size) if pos.size else np.float32(np.nan)
    thr = np.float32(threshold) if threshold < float(mean) else mean
    return g, float(thr), vren_ref.packbits(g.reshape(-1), float(thr))
