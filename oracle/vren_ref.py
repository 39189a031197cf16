"""ORACLE — test infrastructure only (see oracle/vren_ref.c header).

numpy-facing ctypes wrapper around oracle/_build/libvren_ref.so, the plain-C CPU restatement of
the reference `vren` kernels (/root/reference/models/csrc/*.cu).  Signatures and return values
mirror the reference pybind functions (binding.cpp:330-349) but take/return numpy arrays (or CPU
torch tensors, converted).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libvren_ref.so")
_lib = None

f32p = ctypes.POINTER(ctypes.c_float)
i32p = ctypes.POINTER(ctypes.c_int32)
i64p = ctypes.POINTER(ctypes.c_int64)
u8p = ctypes.POINTER(ctypes.c_uint8)
I64 = ctypes.c_int64


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(os.path.join(_HERE, "vren_ref.c")):
            build()
        _lib = ctypes.CDLL(_SO)
    return _lib


def _np(x, dtype):
    try:
        import torch
        if isinstance(x, torch.Tensor):
            x = x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.ascontiguousarray(np.asarray(x, dtype=dtype))


def _p(a, t):
    return a.ctypes.data_as(t)


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """intersection.cu:59-100 -> (hit_cnt i32 (R), hits_t f32 (R,M,2), hits_voxel_idx i64 (R,M))"""
    o = _np(rays_o, np.float32); d = _np(rays_d, np.float32)
    c = _np(centers, np.float32); h = _np(half_sizes, np.float32)
    R, V = o.shape[0], c.shape[0]
    cnt = np.zeros(R, np.int32)
    ht = np.zeros((R, max_hits, 2), np.float32)
    hv = np.zeros((R, max_hits), np.int64)
    lib().ref_ray_aabb_intersect(_p(o, f32p), _p(d, f32p), I64(R), _p(c, f32p), _p(h, f32p), I64(V),
                                 ctypes.c_int(max_hits), _p(cnt, i32p), _p(ht, f32p), _p(hv, i64p))
    return cnt, ht, hv


def morton3D(coords):
    c = _np(coords, np.int32)
    out = np.zeros(c.shape[0], np.int32)
    lib().ref_morton3D(_p(c, i32p), I64(c.shape[0]), _p(out, i32p))
    return out


def morton3D_invert(indices):
    i = _np(indices, np.int32)
    out = np.zeros((i.shape[0], 3), np.int32)
    lib().ref_morton3D_invert(_p(i, i32p), I64(i.shape[0]), _p(out, i32p))
    return out


def packbits(density_grid, threshold, n_bytes=None):
    g = _np(density_grid, np.float32).reshape(-1)
    nb = g.size // 8 if n_bytes is None else n_bytes
    out = np.zeros(nb, np.uint8)
    lib().ref_packbits(_p(g, f32p), I64(nb), ctypes.c_float(threshold), _p(out, u8p))
    return out


def raymarching_train(rays_o, rays_d, hits_t, bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples):
    """raymarching.cu:283-332, ray-ordered.  Returns exactly-sized arrays
    (rays_a i64 (R,3), xyzs (S,3), dirs (S,3), deltas (S), ts (S), counter i32 (2))."""
    o = _np(rays_o, np.float32); d = _np(rays_d, np.float32)
    ht = _np(hits_t, np.float32).reshape(-1, 2)
    bf = _np(bitfield, np.uint8); nz = _np(noise, np.float32)
    R = o.shape[0]
    rays_a = np.zeros((R, 3), np.int64)
    counter = np.zeros(2, np.int32)
    L = lib()
    args = (_p(o, f32p), _p(d, f32p), _p(ht, f32p), I64(R), _p(bf, u8p), ctypes.c_int(cascades),
            ctypes.c_float(scale), ctypes.c_float(exp_step_factor), _p(nz, f32p), ctypes.c_int(grid_size),
            ctypes.c_int(max_samples))
    null = ctypes.cast(None, f32p)
    L.ref_raymarching_train(*args, _p(rays_a, i64p), null, null, null, null, _p(counter, i32p))
    S = int(counter[0])
    xyzs = np.zeros((S, 3), np.float32); dirs = np.zeros((S, 3), np.float32)
    deltas = np.zeros(S, np.float32); ts = np.zeros(S, np.float32)
    L.ref_raymarching_train(*args, _p(rays_a, i64p), _p(xyzs, f32p), _p(dirs, f32p), _p(deltas, f32p),
                            _p(ts, f32p), _p(counter, i32p))
    return rays_a, xyzs, dirs, deltas, ts, counter


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, bitfield, cascades, scale, exp_step_factor,
                     grid_size, max_samples, N_samples):
    """raymarching.cu:407-454.  hits_t (numpy f32 (R,2)) is mutated in place, as in the reference."""
    o = _np(rays_o, np.float32); d = _np(rays_d, np.float32)
    assert isinstance(hits_t, np.ndarray) and hits_t.dtype == np.float32 and hits_t.flags.c_contiguous
    al = _np(alive_indices, np.int64); bf = _np(bitfield, np.uint8)
    A = al.shape[0]
    xyzs = np.zeros((A, N_samples, 3), np.float32); dirs = np.zeros((A, N_samples, 3), np.float32)
    deltas = np.zeros((A, N_samples), np.float32); ts = np.zeros((A, N_samples), np.float32)
    n_eff = np.zeros(A, np.int32)
    lib().ref_raymarching_test(_p(o, f32p), _p(d, f32p), _p(hits_t, f32p), _p(al, i64p), I64(A), _p(bf, u8p),
                               ctypes.c_int(cascades), ctypes.c_float(scale), ctypes.c_float(exp_step_factor),
                               ctypes.c_int(grid_size), ctypes.c_int(max_samples), ctypes.c_int(N_samples),
                               _p(xyzs, f32p), _p(dirs, f32p), _p(deltas, f32p), _p(ts, f32p), _p(n_eff, i32p))
    return xyzs, dirs, deltas, ts, n_eff


def composite_train_multi_fw(sigmas, raws, deltas, ts, rays_a, T_threshold):
    """volumerendering.cu:140-176 -> (total_samples i64 (R), opacity (R), depth (R), rend (R,C), ws (S))"""
    sg = _np(sigmas, np.float32); rw = _np(raws, np.float32); dl = _np(deltas, np.float32)
    t = _np(ts, np.float32); ra = _np(rays_a, np.int64)
    R, S = ra.shape[0], sg.shape[0]
    C = rw.shape[1] if rw.ndim == 2 else 1
    tot = np.zeros(R, np.int64); op = np.zeros(R, np.float32); de = np.zeros(R, np.float32)
    rend = np.zeros((R, C), np.float32); ws = np.zeros(S, np.float32)
    lib().ref_composite_train_fw(_p(sg, f32p), _p(rw, f32p), _p(dl, f32p), _p(t, f32p), _p(ra, i64p), I64(R),
                                 I64(S), ctypes.c_int(C), ctypes.c_float(T_threshold), _p(tot, i64p),
                                 _p(op, f32p), _p(de, f32p), _p(rend, f32p), _p(ws, f32p))
    return tot, op, de, rend, ws


def composite_train_multi_bw(dL_dopacity, dL_ddepth, dL_drend, dL_dws, sigmas, raws, ws, deltas, ts, rays_a,
                             opacity, depth, rend, T_threshold):
    """volumerendering.cu:367-418 -> (dL_dsigmas (S), dL_draws (S,C)).  dL_dws may be None (== zeros)."""
    sg = _np(sigmas, np.float32); rw = _np(raws, np.float32); w = _np(ws, np.float32)
    dl = _np(deltas, np.float32); t = _np(ts, np.float32); ra = _np(rays_a, np.int64)
    R, S = ra.shape[0], sg.shape[0]
    C = rw.shape[1]
    dO = _np(dL_dopacity, np.float32); dD = _np(dL_ddepth, np.float32); dR = _np(dL_drend, np.float32)
    dW = None if dL_dws is None else _np(dL_dws, np.float32)
    O = _np(opacity, np.float32); D = _np(depth, np.float32); RE = _np(rend, np.float32)
    ds = np.zeros(S, np.float32); dr = np.zeros((S, C), np.float32)
    lib().ref_composite_train_bw(_p(dO, f32p), _p(dD, f32p), _p(dR, f32p),
                                 ctypes.cast(None, f32p) if dW is None else _p(dW, f32p),
                                 _p(sg, f32p), _p(rw, f32p), _p(w, f32p), _p(dl, f32p), _p(t, f32p), _p(ra, i64p),
                                 I64(R), I64(S), ctypes.c_int(C), _p(O, f32p), _p(D, f32p), _p(RE, f32p),
                                 ctypes.c_float(T_threshold), _p(ds, f32p), _p(dr, f32p))
    return ds, dr


def composite_test_multi_fw(sigmas, raws, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples,
                            opacity, depth, rend):
    """volumerendering.cu:553-586; mutates alive_indices, opacity, depth, rend (numpy, in place)."""
    sg = _np(sigmas, np.float32); rw = _np(raws, np.float32); dl = _np(deltas, np.float32)
    t = _np(ts, np.float32); ne = _np(N_eff_samples, np.int32)
    for a, dt in ((alive_indices, np.int64), (opacity, np.float32), (depth, np.float32), (rend, np.float32)):
        assert isinstance(a, np.ndarray) and a.dtype == dt and a.flags.c_contiguous
    A, N = sg.shape[0], sg.shape[1]
    C = rw.shape[2]
    lib().ref_composite_test_fw(_p(sg, f32p), _p(rw, f32p), _p(dl, f32p), _p(t, f32p), _p(alive_indices, i64p),
                                I64(A), ctypes.c_int(N), ctypes.c_int(C), ctypes.c_float(T_threshold), _p(ne, i32p),
                                _p(opacity, f32p), _p(depth, f32p), _p(rend, f32p))


# ---- occupancy-grid refresh (ngp_mt.py:305-368), numpy restatement -------------------------------
def grid_hit_probabilities(n_cells, M, n_occ):
    """Marginal probability that a cell is drawn at least once by M uniform draws over n_cells
    cells (sample_uniform_and_occupied_cells, ngp_mt.py:252-255) and by M draws over the n_occ
    occupied cells (:256-259), both with replacement."""
    p_u = -np.expm1(M * np.log1p(-1.0 / n_cells))
    p_o = -np.expm1(M * np.log1p(-1.0 / n_occ)) if n_occ > 0 else 0.0
    return float(p_u), float(p_o)


def grid_cell_positions(cells, grid_size, s):
    """Un-jittered world position of each cell (ngp_mt.py:318): (coords/(G-1)*2-1)*(s-half_grid), f32."""
    coords = morton3D_invert(np.asarray(cells, np.int32)).astype(np.float32)
    hg = s / grid_size
    x = coords / np.float32(grid_size - 1)
    x = x * np.float32(2) - np.float32(1)
    return x * np.float32(s - hg), hg


def density_grid_update(grid, cells, sigmas, decay, threshold, count_grid=None):
    """ngp_mt.py:320-326: density_grid_tmp[cells] = sigmas; grid = where(grid < 0, grid,
    max(grid*decay, tmp)) (decay per cell with erode: clamp(decay**(1/count), 0.1, 0.95));
    mean of the positive cells; bitfield = packbits(grid, min(mean, threshold)).  f32 arithmetic as
    torch; the mean in f64 (torch: f32 tree reduction).  Returns (grid, threshold_used, bitfield)."""
    g = np.asarray(grid, np.float32)
    tmp = np.zeros_like(g)
    tmp.reshape(-1)[np.asarray(cells, np.int64)] = np.asarray(sigmas, np.float32)
    d = np.float32(decay)
    if count_grid is not None:
        with np.errstate(divide="ignore"):
            d = np.clip(np.float32(decay) ** (np.float32(1) / np.asarray(count_grid, np.float32)),
                        np.float32(0.1), np.float32(0.95)).astype(np.float32)
    new = np.where(g < 0, g, np.maximum(g * d, tmp)).astype(np.float32)
    pos = new[new > 0]
    mean = np.float32(pos.astype(np.float64).mean()) if pos.size else np.float32(np.nan)
    thr = min(float(mean), threshold)
    return new, thr, packbits(new, thr)


def segment_csr(src, indptr):
    """torch_scatter.segment_csr(src, indptr) with reduce="sum" (the reference's RayMarcher.backward,
    custom_functions.py:107-110): out[i] = src[indptr[i]:indptr[i+1]].sum(0), sequential f32 adds;
    an empty or inverted segment sums to 0."""
    src = np.asarray(src, np.float32)
    out = np.zeros((len(indptr) - 1,) + src.shape[1:], np.float32)
    for i in range(len(indptr) - 1):
        acc = np.zeros(src.shape[1:], np.float32)
        for s in range(int(indptr[i]), int(indptr[i + 1])):
            acc = acc + src[s]
        out[i] = acc
    return out


def raymarcher_backward(rays_a, ts, dL_dxyzs, dL_ddirs):
    """custom_functions.py:102-112: (dL/drays_o, dL/drays_d) of RayMarcher by segment_csr over
    indptr = [rays_a[:, 1], rays_a[-1, 1] + rays_a[-1, 2]]."""
    rays_a = np.asarray(rays_a)
    indptr = np.concatenate([rays_a[:, 1], rays_a[-1:, 1] + rays_a[-1:, 2]])
    ts = np.asarray(ts, np.float32)
    gx = np.asarray(dL_dxyzs, np.float32)
    return segment_csr(gx, indptr), segment_csr(gx * ts[:, None] + np.asarray(dL_ddirs, np.float32), indptr)
