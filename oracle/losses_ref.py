"""ORACLE — test infrastructure only.  Never imported by the product path.

CPU restatement of the normal-clustering loss path:
  * `normals_from_depth`  — datasets/hypersim_src/utils.py:504-541 (_extract_normals_from_ray_batch)
  * `patch_triangles`     — datasets/base.py:35-66 (x1/x2/x3 local offsets of an 8x8 patch) and
                            losses.py:307-313 (get_patch_triang_idx)
  * `spherical_kmeans`    — the k-means behind losses.py:433-440 (faiss.Kmeans(3, k=20, niter=20,
                            spherical=True)).  faiss is not installed here and its version is unpinned
                            (not in README/requirements; imported at losses.py:8-9), so this is OUR
                            deterministic Lloyd spherical k-means (see `spherical_kmeans` doc) — PARITY
                            UNPINNED w.r.t. faiss.  The HIP kernel implements exactly this algorithm.
  * `cluster_select`      — losses.py:47-166 (_cluster_indices, _find_opposite, _normals_clustering),
                            pinned by golden vectors from the reference code (tests/golden).
  * `cluster_losses`      — losses.py:420-478 + the weight schedule losses.py:217 and the validity
                            filter losses.py:246-262, pinned by golden vectors from the reference code.
"""
import numpy as np
import torch
import torch.nn.functional as F

KM_K = 20
KM_NITER = 20


def patch_triangles(patch_size=8):
    """base.py:48-66 -> local (x1, x2, x3) offsets inside a patch_size^2 patch (row-major)."""
    loc = np.arange(patch_size * patch_size, dtype=np.int64).reshape(patch_size, patch_size)
    return loc[1:, 1:].reshape(-1), loc[:-1, 1:].reshape(-1), loc[1:, :-1].reshape(-1)


def patch_triangle_index(n_rays, patch_size=8):
    """losses.py:307-313: per-batch ray indices of every triangle's x1, x2, x3."""
    pa = patch_size * patch_size
    assert n_rays % pa == 0
    o1, o2, o3 = patch_triangles(patch_size)
    base = np.arange(n_rays // pa, dtype=np.int64)[:, None] * pa
    return ((base + o1[None]).reshape(-1), (base + o2[None]).reshape(-1), (base + o3[None]).reshape(-1))


def normals_from_depth(rays_o, rays_d, depth, x1, x2, x3):
    """hypersim_src/utils.py:504-541.  torch CPU, differentiable w.r.t. depth."""
    P = rays_o + rays_d * depth.unsqueeze(-1)
    P1, P2, P3 = P[x1], P[x2], P[x3]
    n = torch.cross(P2 - P1, P3 - P1, dim=-1)
    return F.normalize(n, p=2.0, dim=-1)


def valid_normals_mask(n):
    """losses.py:427-430: drop all-zero, NaN or Inf normals."""
    n = torch.as_tensor(n)
    inv = (torch.abs(n).sum(-1) == 0.0) | (torch.isnan(n).sum(-1) > 0) | (torch.isinf(n).sum(-1) > 0)
    return ~inv


def _mix32(x):
    x = (x ^ (x >> 16)) * 0x7FEB352D & 0xFFFFFFFF
    x = (x ^ (x >> 15)) * 0x846CA68B & 0xFFFFFFFF
    return (x ^ (x >> 16)) & 0xFFFFFFFF


def kmeans_init_indices(n, K, seed):
    """Stratified seeded init: one pick per stratum [k*n/K, (k+1)*n/K) (the HIP kernel uses the same)."""
    idx = []
    for k in range(K):
        lo = (k * n) // K
        hi = ((k + 1) * n) // K
        span = max(hi - lo, 1)
        idx.append(lo + _mix32((seed * 0x9E3779B1 + k * 0x85EBCA77 + 1) & 0xFFFFFFFF) % span)
    return np.array(idx, dtype=np.int64)


def spherical_kmeans(X, K=KM_K, niter=KM_NITER, seed=0):
    """Deterministic spherical Lloyd k-means (float32, numpy).

    init: X[kmeans_init_indices]; each of `niter` iterations: assign every point to the centroid of
    largest inner product (ties -> lowest index), centroid = mean of its members, empty clusters
    are split from the largest cluster with faiss's perturbation (+/- 1/1024 on alternating
    coordinates), then every centroid is L2-normalised (spherical).  The returned assignment is a
    final search against the final centroids, as losses.py:436 does with kmeans.index.search.
    Returns (centroids (K,3) f32, assign (n,) i64)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n = X.shape[0]
    C = X[kmeans_init_indices(n, K, seed)].copy()
    EPS = np.float32(1.0 / 1024.0)
    for _ in range(niter):
        a = np.argmax(X @ C.T, axis=1)
        cnt = np.bincount(a, minlength=K).astype(np.int64)
        S = np.zeros((K, 3), np.float64)
        np.add.at(S, a, X.astype(np.float64))
        newC = C.copy()
        for k in range(K):
            if cnt[k] > 0:
                newC[k] = (S[k] / cnt[k]).astype(np.float32)
        for k in range(K):  # split empty clusters from the (current) largest one
            if cnt[k] == 0:
                j = int(np.argmax(cnt))
                for dd in range(3):
                    if dd % 2 == 0:
                        newC[k, dd] = newC[j, dd] * (1 + EPS); newC[j, dd] = newC[j, dd] * (1 - EPS)
                    else:
                        newC[k, dd] = newC[j, dd] * (1 - EPS); newC[j, dd] = newC[j, dd] * (1 + EPS)
                cnt[k] = cnt[j] // 2
                cnt[j] = cnt[j] - cnt[k]
        nrm = np.sqrt((newC.astype(np.float64) ** 2).sum(1, keepdims=True))
        C = (newC / np.maximum(nrm, 1e-30)).astype(np.float32)
    a = np.argmax(X @ C.T, axis=1).astype(np.int64)
    return C, a


def _cluster_indices(sim_all, c_i, old_assign, t_merge):
    """losses.py:47-54 (merge=True)."""
    c_indices = np.nonzero(sim_all[c_i] > t_merge)[0]
    return np.isin(old_assign, c_indices)


def cluster_select(centrs, assign, t_similar):
    """losses.py:75-166 given k-means output.  Returns (labels in {0,+-1,+-2,+-3} (n,), centrs_new (3,3))."""
    centrs = np.asarray(centrs, np.float32)
    assign = np.asarray(assign, np.int64)
    new = np.zeros_like(assign)
    sim_all = centrs @ centrs.T
    sim_abs = np.abs(sim_all)
    sizes = np.bincount(assign)
    c1 = int(np.argmax(sizes))  # topk(sorted)[0]; ties -> lowest index
    new[_cluster_indices(sim_all, c1, assign, t_similar)] = 1
    crit = sim_abs[:, c1][:, None] + sim_abs[c1, :][None, :] + sim_abs
    mins = crit.min(axis=0)
    min_idxs = crit.argmin(axis=0)
    c2 = int(np.argmin(mins))
    c3 = int(min_idxs[c2])
    new[_cluster_indices(sim_all, c2, assign, t_similar)] = 2
    new[_cluster_indices(sim_all, c3, assign, t_similar)] = 3
    centrs_new = centrs[[c1, c2, c3]]
    for lab, ci in ((-1, c1), (-2, c2), (-3, c3)):  # losses.py:58-72, 139-163
        cand = sim_all[ci]
        co = int(np.argmin(cand))
        if -1.0 * cand[co] > t_similar:
            new[_cluster_indices(sim_all, co, assign, t_similar)] = lab
    return new, centrs_new


def w_sched(w, step, start=500, grow=2500):
    """losses.py:217"""
    return max(0, min(w, (step - start) * (w / grow)))


def cluster_losses(normals, labels):
    """losses.py:441-478 (ort / centr_dot / centr_L1 terms), torch, differentiable w.r.t. normals.
    `normals` are the VALID normals (after losses.py:427-430); `labels` from cluster_select."""
    labels = torch.as_tensor(labels)
    keep = labels != 0
    x = normals[keep]
    lab = labels[keep].clone()
    sgn = torch.where(lab < 0, -1.0, 1.0).to(x.dtype)
    x = x * sgn[:, None]  # losses.py:445-447 flip
    lab = lab.abs()
    cl = [x[lab == k] for k in (1, 2, 3)]
    c = [F.normalize(ck.mean(dim=0, keepdim=True), p=2.0, dim=-1) for ck in cl]
    ort = (torch.abs((c[0] * c[1]).sum()) + torch.abs((c[0] * c[2]).sum()) + torch.abs((c[1] * c[2]).sum())) / 3.0
    cdot = sum(1.0 - (cl[k] * c[k]).sum(dim=-1).mean() for k in range(3)) / 3.0
    cl1 = sum(torch.abs(cl[k] - c[k]).sum(dim=-1).mean() for k in range(3)) / 3.0
    return ort, cdot, cl1


def validity(loss):
    """losses.py:246-262: NaN/Inf (or non-scalar) terms are replaced by 0."""
    if loss.nelement() != 1 or torch.isnan(loss) or torch.isinf(loss):
        return torch.zeros((), dtype=loss.dtype)
    return loss


# ---- distortion loss (losses.py:16-44, models/csrc/losses.cu) -------------------------------------
def distortion_loss_fw(ws, deltas, ts, rays_a):
    """losses.cu:47-100 restated per ray with sequential f32 prefix sums (thrust's order):
    -> (loss (R) by ray_idx, ws_inclusive_scan (S), wts_inclusive_scan (S))."""
    ws = np.asarray(ws, np.float32); deltas = np.asarray(deltas, np.float32); ts = np.asarray(ts, np.float32)
    rays_a = np.asarray(rays_a, np.int64)
    S = ws.shape[0]
    wts = (ws * ts).astype(np.float32)
    wsi, wtsi = np.zeros(S, np.float32), np.zeros(S, np.float32)
    wse, wtse = np.zeros(S, np.float32), np.zeros(S, np.float32)
    loss = np.zeros(rays_a.shape[0], np.float32)
    for r, s0, n in rays_a:
        if n == 0:
            continue
        sl = slice(s0, s0 + n)
        wsi[sl] = np.cumsum(ws[sl], dtype=np.float32)
        wtsi[sl] = np.cumsum(wts[sl], dtype=np.float32)
        wse[sl] = wsi[sl] - ws[sl]
        wtse[sl] = wtsi[sl] - wts[sl]
    _loss = (np.float32(2) * (wtsi * wse - wsi * wtse) + np.float32(1.0 / 3) * ws * ws * deltas).astype(np.float32)
    for r, s0, n in rays_a:
        loss[r] = _loss[s0:s0 + n].sum(dtype=np.float32)
    return loss, wsi, wtsi


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    """losses.cu:103-140 -> dL_dws (S)."""
    wsi, wtsi = np.asarray(ws_inclusive_scan, np.float32), np.asarray(wts_inclusive_scan, np.float32)
    ws = np.asarray(ws, np.float32); deltas = np.asarray(deltas, np.float32); ts = np.asarray(ts, np.float32)
    g = np.asarray(dL_dloss, np.float32)
    out = np.zeros(ws.shape[0], np.float32)
    for r, s0, n in np.asarray(rays_a, np.int64):
        if n == 0:
            continue
        e = s0 + n - 1
        for s in range(s0, e + 1):
            before = np.float32(0) if s == s0 else ts[s] * wsi[s - 1] - wtsi[s - 1]
            v = g[r] * 2 * (before + (wtsi[e] - wtsi[s] - ts[s] * (wsi[e] - wsi[s])))
            out[s] = v + g[r] * np.float32(2.0 / 3) * ws[s] * deltas[s]
    return out


def distortion_loss_naive(ws, deltas, ts, rays_a):
    """The definition the O(N) form implements (Mip-NeRF 360 / DVGO-v2), float64 torch:
    sum_i sum_j w_i w_j |t_i - t_j| + 1/3 sum_i w_i^2 delta_i per ray (t ascending within a ray)."""
    out = []
    for r, s0, n in np.asarray(rays_a, np.int64):
        w, t, d = ws[s0:s0 + n], ts[s0:s0 + n], deltas[s0:s0 + n]
        out.append((w[:, None] * w[None, :] * (t[:, None] - t[None, :]).abs()).sum() + (w * w * d).sum() / 3)
    return torch.stack(out)
