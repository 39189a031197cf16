"""ORACLE — test infrastructure only.  Never imported by the product path.

CPU restatement of the normal-clustering loss path:
  * `normals_from_depth`  — datasets/hypersim_src/utils.py:504-541 (_extract_normals_from_ray_batch)
  * `patch_triangles`     — datasets/base.py:35-66 (x1/x2/x3 local offsets of an 8x8 patch) and
                            losses.py:307-313 (get_patch_triang_idx)
  * `spherical_kmeans`    — the k-means behind losses.py:86-89 (faiss.Kmeans(3, k=20, niter=20,
                            spherical=True) + index.search).  faiss is not installed here and its
                            version is unpinned (not in README/requirements; imported at
                            losses.py:8-9): this RESTATES faiss's published Clustering::train
                            (faiss/Clustering.cpp, utils/random.cpp of the 1.7 line) — subsampling
                            to k*max_points_per_centroid (256) points by rand_perm(seed 1234),
                            init = the first k points of rand_perm(seed 1235), search / centroid
                            mean / split_clusters (RandomGenerator(1234) per iteration) / L2
                            renormalisation per iteration, then a final search of all points —
                            with std::mt19937 restated below.  PARITY UNPINNED w.r.t. faiss itself
                            (no fixture of faiss output exists); float summation order differs
                            (faiss sums centroids in f32, the HIP kernel in exact fixed point).
                            The HIP kernel implements exactly this algorithm.
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


class Mt19937:
    """std::mt19937 (faiss RandomGenerator's engine: `mt((unsigned int)seed)`)."""

    def __init__(self, seed):
        mt = [0] * 624
        mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.mt, self.i = np.array(mt, np.uint64), 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (int(mt[i]) & 0x80000000) | (int(mt[(i + 1) % 624]) & 0x7FFFFFFF)
            v = int(mt[(i + 397) % 624]) ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            mt[i] = v
        self.i = 0

    def __call__(self):
        if self.i >= 624:
            self._twist()
        y = int(self.mt[self.i])
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    @staticmethod
    def _twist_np(mt):
        """The same twist, vectorised in the four ranges whose inputs are all old or all new."""
        mt = mt.copy()

        def f(i0, i1):
            i = np.arange(i0, i1)
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ np.where(y & 1, np.uint64(0x9908B0DF), np.uint64(0))
        for a, b in ((0, 227), (227, 454), (454, 623), (623, 624)):
            f(a, b)
        return mt

    def draws(self, count):
        """The next `count` outputs as a uint64 array (same sequence as `count` calls)."""
        out = []
        while count > 0:
            if self.i >= 624:
                self.mt, self.i = self._twist_np(self.mt), 0
            y = self.mt[self.i:self.i + count].copy()
            self.i += y.size
            count -= y.size
            y ^= y >> np.uint64(11)
            y ^= (y << np.uint64(7)) & np.uint64(0x9D2C5680)
            y ^= (y << np.uint64(15)) & np.uint64(0xEFC60000)
            y ^= y >> np.uint64(18)
            out.append(y & np.uint64(0xFFFFFFFF))
        return np.concatenate(out) if out else np.zeros(0, np.uint64)


def rand_perm_prefix(n, seed, m):
    """faiss rand_perm(perm, n, seed) (utils/random.cpp): Fisher-Yates with
    i2 = i + RandomGenerator::rand_int(n - i) = i + mt() % (n - i); only the first m steps (the
    first m entries are final after them)."""
    perm = np.arange(n, dtype=np.int64)
    rng = Mt19937(seed)
    for i in range(min(m, n - 1)):
        i2 = i + rng() % (n - i)
        perm[i], perm[i2] = perm[i2], perm[i]
    return perm[:m]


def rand_floats(seed, count):
    """RandomGenerator::rand_float() = mt() / float(mt.max()) in f32."""
    return (Mt19937(seed).draws(count).astype(np.float32) / np.float32(4294967295.0)).astype(np.float32)


MAX_POINTS_PER_CENTROID = 256  # faiss ClusteringParameters default
N_RAND = 4096


def faiss_training_set(nx, K, seed=1234):
    """(indices of the training points in subsample order, init picks as indices into the input)."""
    cap = K * MAX_POINTS_PER_CENTROID
    if nx > cap:
        sub = rand_perm_prefix(nx, seed, cap)  # subsample_training_set
    else:
        sub = np.arange(nx, dtype=np.int64)
    picks = rand_perm_prefix(len(sub), seed + 1, K)  # init (redo 0: seed + 1 + 0 * 15486557)
    return sub, sub[picks]


def plan_mask_row(nx, K, seed=1234):
    """Training-set membership bits (uint32 words, bit i = point i) of nx > K*256 points."""
    sub, _ = faiss_training_set(nx, K, seed)
    bits = np.zeros(((nx + 31) // 32) * 32, np.uint64)
    bits[sub] = 1
    return (bits.reshape(-1, 32) << np.arange(32, dtype=np.uint64)).sum(1).astype(np.uint32)


def _renorm(C):
    """faiss fvec_renorm_L2: x *= (float)(1.0 / sqrtf(|x|^2)) (a double division) when |x|^2 > 0;
    |x|^2 in f32 as ((x0 x0 + x1 x1) + x2 x2)."""
    C = C.astype(np.float32).copy()
    for k in range(C.shape[0]):
        nr = np.float32(np.float32(C[k, 0] * C[k, 0]) + np.float32(C[k, 1] * C[k, 1]))
        nr = np.float32(nr + np.float32(C[k, 2] * C[k, 2]))
        if nr > 0:
            C[k] = C[k] * np.float32(1.0 / float(np.sqrt(nr, dtype=np.float32)))
    return C


def _dots(X, C):
    """<x, c> in f32 without FMA as ((x0 c0 + x1 c1) + x2 c2): the HIP kernel's association (faiss
    itself uses BLAS sgemm: unpinned at the last bit)."""
    X = X.astype(np.float32)
    C = C.astype(np.float32)
    return (X[:, None, 0] * C[None, :, 0] + X[:, None, 1] * C[None, :, 1]) + X[:, None, 2] * C[None, :, 2]


KM_FXL = 2.0 ** 39


def _fixed_sum(X):
    """Sum of rows as the HIP kernel forms it: every coordinate rounded to 2^-39 (half to even),
    exact int64 sums, one rounding to f32 (faiss sums in f32 in point order: unpinned)."""
    q = np.rint(X.astype(np.float64) * KM_FXL).astype(np.int64).sum(0)
    return (q.astype(np.float64) * (1.0 / KM_FXL)).astype(np.float32)


def spherical_kmeans(X, K=KM_K, niter=KM_NITER, seed=1234, trace=None):
    """faiss.Kmeans(3, K, niter, spherical=True).train(X) + index.search(X, 1) (losses.py:86-89),
    restated (module doc) with the HIP kernel's arithmetic (_dots, _fixed_sum), so the device
    result is reproduced bit for bit.  Returns (centroids (K,3) f32, assign (n,) i64).
    trace (a list): appends the first training round whose assignment equals the previous round's
    (from there on the rounds are a fixed point), or niter if none does."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n = X.shape[0]
    sub, picks = faiss_training_set(n, K, seed)
    Xt = X[sub]
    nt = Xt.shape[0]
    if nt == K:  # faiss's nx == k corner case: the points are the centroids, no iteration
        C = X[:K].copy()
        return C, np.argmax(_dots(X, C), axis=1).astype(np.int64)
    C = _renorm(X[picks])
    EPS = 1.0 / 1024.0
    prev, fixed = None, None
    for it in range(niter):
        a = np.argmax(_dots(Xt, C), axis=1)  # IndexFlatIP search, ties -> lowest index
        if fixed is None and prev is not None and np.array_equal(a, prev):
            fixed = it
        prev = a
        cnt = np.bincount(a, minlength=K).astype(np.float32)  # hassign
        newC = np.zeros((K, 3), np.float32)
        for k in range(K):
            if cnt[k] > 0:
                newC[k] = _fixed_sum(Xt[a == k]) * (np.float32(1.0) / cnt[k])
        rng, r_i = rand_floats(1234, N_RAND), 0  # split_clusters: RandomGenerator rng(1234), per call
        for ci in range(K):
            if cnt[ci] == 0:
                cj = 0
                while True:
                    p = np.float32((float(cnt[cj]) - 1.0) / float(np.float32(nt - K)))
                    r = rng[r_i]
                    r_i += 1
                    if r < p:
                        break
                    cj = (cj + 1) % K
                newC[ci] = newC[cj]
                for dd in range(3):
                    if dd % 2 == 0:
                        newC[ci, dd] *= np.float32(1 + EPS); newC[cj, dd] *= np.float32(1 - EPS)
                    else:
                        newC[ci, dd] *= np.float32(1 - EPS); newC[cj, dd] *= np.float32(1 + EPS)
                cnt[ci] = cnt[cj] / np.float32(2)
                cnt[cj] -= cnt[ci]
        C = _renorm(newC)
    a = np.argmax(_dots(X, C), axis=1).astype(np.int64)  # kmeans.index.search(normals_np, 1)
    if trace is not None:
        trace.append(niter if fixed is None else fixed)
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


def cluster_losses(normals, labels, signs=None):
    """losses.py:441-478 (ort / centr_dot / centr_L1 terms), torch, differentiable w.r.t. normals.
    `normals` are the VALID normals (after losses.py:427-430); `labels` from cluster_select.
    signs (optional, test infrastructure): the branches of the terms' absolute values taken from
    another evaluation (kink_signs of it) — |v| is evaluated as s * v with s fixed, the same value
    wherever the two agree on the sign, and the gradient of the given branch; see kink_signs."""
    labels = torch.as_tensor(labels)
    keep = labels != 0
    x = normals[keep]
    lab = labels[keep].clone()
    sgn = torch.where(lab < 0, -1.0, 1.0).to(x.dtype)
    x = x * sgn[:, None]  # losses.py:445-447 flip
    lab = lab.abs()
    cl = [x[lab == k] for k in (1, 2, 3)]
    c = [F.normalize(ck.mean(dim=0, keepdim=True), p=2.0, dim=-1) for ck in cl]
    dots = [(c[0] * c[1]).sum(), (c[0] * c[2]).sum(), (c[1] * c[2]).sum()]
    if signs is None:
        ort = (torch.abs(dots[0]) + torch.abs(dots[1]) + torch.abs(dots[2])) / 3.0
        cl1 = sum(torch.abs(cl[k] - c[k]).sum(dim=-1).mean() for k in range(3)) / 3.0
    else:
        s_ort, s_l1 = signs
        ort = sum(float(s_ort[i]) * dots[i] for i in range(3)) / 3.0
        cl1 = sum(((cl[k] - c[k]) * torch.as_tensor(s_l1[k], dtype=x.dtype)).sum(dim=-1).mean() for k in range(3)) / 3.0
    cdot = sum(1.0 - (cl[k] * c[k]).sum(dim=-1).mean() for k in range(3)) / 3.0
    return ort, cdot, cl1


def kink_signs(normals, labels):
    """The sign branches cluster_losses' absolute values take on these VALID normals and labels:
    (signs of the three centroid dot products, per selected cluster the signs of (normal - centroid)
    per component), float64.  The ort and L1 terms are |.| of quantities that training drives to ~0
    (orthogonal Manhattan centroids, normals on their centroid), so at a trained state two correct
    evaluations whose normals differ by ~5e-4 rad take opposite branches for many of them, and the
    gradient flips there while the loss does not move: test infrastructure shares the branches as it
    shares the labels."""
    v_ort, v_l1, _ = kink_values(normals, labels)
    return np.sign(v_ort), [np.sign(v) for v in v_l1]


def kink_values(normals, labels):
    """The quantities whose absolute values cluster_losses takes (losses.py:461-478), float64:
    (the three centroid dot products c_i . c_j, per selected cluster (normal - centroid) per component
    (n_k, 3), the three unit centroids (3, 3)) — kink_signs' signs, and what a test checks them by."""
    n = np.asarray(normals, np.float64)
    lab = np.asarray(labels)
    keep = lab != 0
    x = n[keep] * np.where(lab[keep] < 0, -1.0, 1.0)[:, None]
    la = np.abs(lab[keep])
    cl = [x[la == k] for k in (1, 2, 3)]
    c = []
    for ck in cl:
        m = ck.mean(axis=0)
        c.append(m / max(np.linalg.norm(m), 1e-12))
    v_ort = np.array([c[0] @ c[1], c[0] @ c[2], c[1] @ c[2]])
    return v_ort, [cl[k] - c[k] for k in range(3)], np.stack(c)


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
