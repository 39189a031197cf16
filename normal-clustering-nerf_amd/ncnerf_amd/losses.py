"""NeRFMTLoss of the reference losses.py:169-587 for the training hot path.

Kept: the photometric MSE (losses.py:349-355), opacity entropy (:358-362), depth L2 (:372-385),
normals-from-depth vs GT normals L1/dot (:388-411), RegNeRF depth smoothness (:414-418) and the
normal-clustering block (:420-509) with its weight schedule (:217) and validity filter (:246-262).
The clustering block runs on the GPU end to end: `_extract_normals_from_ray_batch`
(hypersim_src/utils.py:504-541) is `ncn_normals_fwd/bwd`, and faiss k-means + the cluster selection
+ the three cluster losses + their gradient are ONE persistent launch (`ncn_cluster_loss`), so the
step no longer copies normals to the host (losses.py:434) or syncs on `.item()`s.

The k-means restates faiss's published `Clustering::train` as losses.py:86-89 calls it
(faiss.Kmeans(3, 20, niter=20, spherical=True)): the training set subsampled to 256*K points by
rand_perm(seed 1234) when larger, the initial centroids the first K of rand_perm(seed 1235), Lloyd
rounds with spherical renormalisation and faiss's split_clusters for empty clusters (its
RandomGenerator walk from a host-built std::mt19937 plan), then a final search over all points.
faiss itself is not available here: parity unpinned w.r.t. faiss, see DESIGN.md §3.

Not provided (weight 0 in every reference config, hyperparameters.py:33-49): semantic,
Manhattan-NeRF and the canonical-direction terms (raise if enabled).
"""
import einops
import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib, vren
from ._lib import F32, I32, I64, U32, call, check_input, ptr, stream

N_OUT = 11  # ncn_cluster_loss out_losses
_WS = {}


def _cluster_workspace(dev, K):
    """The clustering workspace of (device, K): zeroed once, reused by every call (ncn_cluster_loss
    leaves its grid-barrier words at zero).  Created on the first (eager) call, so a captured step
    reuses it.  Calls on one device are stream-ordered in this package (one training stream)."""
    key = (str(dev), K)
    ws = _WS.get(key)
    if ws is None:
        ws = torch.zeros(int(_lib.lib().ncn_cluster_workspace_words(I32(K))), dtype=torch.float32, device=dev)
        _WS[key] = ws
    return ws


_PLANS = {}


def kmeans_plan(dev, n_tri, K, seed=1234):
    """faiss's k-means draws for (n_tri, K, seed) (ncn_kmeans_plan_fill, built on the host once with
    std::mt19937 and kept on `dev`): subsample membership, init picks, split floats."""
    key = (str(dev), int(n_tri), int(K), int(seed))
    plan = _PLANS.get(key)
    if plan is None:
        words = int(_lib.lib().ncn_kmeans_plan_words(I32(n_tri), I32(K)))
        host = torch.zeros(words, dtype=torch.int32)
        rc = _lib.lib().ncn_kmeans_plan_fill(I32(n_tri), I32(K), U32(seed), ptr(host))
        if rc != 0:
            raise _lib.NcnError("ncn_kmeans_plan_fill failed: " + _lib.lib().ncn_last_error().decode())
        plan = host.to(dev)
        _PLANS[key] = plan
    return plan


def check_cluster_status(dev=None):
    """Raise if a clustering launch on any workspace (of `dev`, or all) hit its barrier/hand-off
    timeout (the kernel's sticky error word, ncn_cluster_status_offset): its losses and gradients
    were computed from incomplete partial sums.  One device read per workspace (host sync)."""
    for (d, K), ws in _WS.items():
        if dev is not None and d != str(dev):
            continue
        off = int(_lib.lib().ncn_cluster_status_offset(I32(K)))
        if int(ws.view(torch.int32)[off].item()) != 0:
            raise _lib.NcnError(f"ncn_cluster_loss on {d} (K={K}): a grid barrier / Lloyd hand-off timed out "
                                f"(its workgroups were not co-resident); cluster losses are invalid")


class _Normals(torch.autograd.Function):
    """hypersim_src/utils.py:504-541: n = normalize(cross(P2-P1, P3-P1)), P = rays_o + rays_d*depth."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, depth, x1, x2, x3):
        T = x1.shape[0]
        normals = torch.empty(T, 3, dtype=torch.float32, device=depth.device)
        call("ncn_normals_fwd", ptr(rays_o), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(T), ptr(normals),
             stream())
        ctx.save_for_backward(rays_o, rays_d, depth, x1, x2, x3)
        return normals

    @staticmethod
    def backward(ctx, dn):
        rays_o, rays_d, depth, x1, x2, x3 = ctx.saved_tensors
        ddepth = torch.zeros_like(depth)
        if dn is not None:
            call("ncn_normals_bwd", ptr(rays_o), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(x1.shape[0]),
                 ptr(dn.contiguous()), None, ptr(ddepth), stream())
        return None, None, ddepth, None, None, None


def extract_normals_from_ray_batch(rays_o, rays_d, depth, x123_idx):
    """Drop-in for datasets/hypersim_src/utils.py:_extract_normals_from_ray_batch (fp32)."""
    f = lambda t: t.float().contiguous()
    idx = lambda t: t.long().contiguous()
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (depth, "depth")):
        if not t.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")
    return _Normals.apply(f(rays_o), f(rays_d), f(depth), idx(x123_idx["x1"]), idx(x123_idx["x2"]),
                          idx(x123_idx["x3"]))


class _ClusterLoss(torch.autograd.Function):
    """losses.py:420-478 on the GPU.  Returns the three weighted terms (ort, centr_dot, centr_L1)
    and, as non-differentiable extras, the labels and the k-means centroids."""

    @staticmethod
    def forward(ctx, normals, K, niter, seed, t_sim, w):
        T = normals.shape[0]
        dev = normals.device
        out = torch.empty(N_OUT, dtype=torch.float32, device=dev)
        labels = torch.empty(T, dtype=torch.int32, device=dev)
        cents = torch.empty(K, 3, dtype=torch.float32, device=dev)
        dn = torch.empty(3, T, 3, dtype=torch.float32, device=dev)
        ws = _cluster_workspace(dev, K)
        hw, w_dev = _split_weights(w)
        call("ncn_cluster_loss", ptr(normals), I64(T), I32(K), I32(niter), ptr(kmeans_plan(dev, T, K, seed)), F32(t_sim), F32(hw[0]),
             F32(hw[1]), F32(hw[2]), ptr(w_dev), ptr(None), F32(0.0), F32(1.0), ptr(None), ptr(out), ptr(labels),
             ptr(cents), ptr(dn), ptr(ws), stream())
        ctx.save_for_backward(dn)
        terms = out[4:7].clone()
        ctx.mark_non_differentiable(labels, cents, out)
        return terms, labels, cents, out

    @staticmethod
    def backward(ctx, g, _g_labels, _g_cents, _g_out):
        (dn,) = ctx.saved_tensors
        if g is None:
            return None, None, None, None, None, None
        g = g.float()
        return g[0] * dn[0] + g[1] * dn[1] + g[2] * dn[2], None, None, None, None, None


def _split_weights(w):
    """(host weights, device weights or None): w is 3 floats or a device tensor of 3 (the
    step-dependent schedule evaluated on the device)."""
    if isinstance(w, torch.Tensor):
        return (0.0, 0.0, 0.0), w.float().contiguous()
    return tuple(float(x) for x in w), None


def _weights_arg(w):
    return w if isinstance(w, torch.Tensor) else tuple(float(x) for x in w)


def cluster_losses(norm_depth, K=20, niter=20, seed=1234, t_similar=0.99, w=(1.0, 1.0, 1.0)):
    """Weighted (ort, centr_dot, centr_L1) terms, labels (+-1..3, 0, -9 invalid), centroids, raw stats."""
    check_input(norm_depth, "norm_depth")
    return _ClusterLoss.apply(norm_depth, K, niter, seed, t_similar, _weights_arg(w))


class _NormalsClusterLoss(torch.autograd.Function):
    """`_Normals` followed by `_ClusterLoss` as one node, used when the depth normals feed only the
    clustering terms (every reference config).  The backward is one `ncn_normals_bwd` launch that
    combines the three per-term normal gradients with the upstream term gradients on the device,
    so no (T,3) normal gradient is materialised and nothing is reduced on the host."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, depth, x1, x2, x3, K, niter, seed, t_sim, w):
        T = x1.shape[0]
        dev = depth.device
        normals = torch.empty(T, 3, dtype=torch.float32, device=dev)
        call("ncn_normals_fwd", ptr(rays_o), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(T), ptr(normals),
             stream())
        out = torch.empty(N_OUT, dtype=torch.float32, device=dev)
        labels = torch.empty(T, dtype=torch.int32, device=dev)
        cents = torch.empty(K, 3, dtype=torch.float32, device=dev)
        dn = torch.empty(3, T, 3, dtype=torch.float32, device=dev)
        ws = _cluster_workspace(dev, K)
        hw, w_dev = _split_weights(w)
        call("ncn_cluster_loss", ptr(normals), I64(T), I32(K), I32(niter), ptr(kmeans_plan(dev, T, K, seed)), F32(t_sim), F32(hw[0]),
             F32(hw[1]), F32(hw[2]), ptr(w_dev), ptr(None), F32(0.0), F32(1.0), ptr(None), ptr(out), ptr(labels),
             ptr(cents), ptr(dn), ptr(ws), stream())
        ctx.save_for_backward(rays_o, rays_d, depth, x1, x2, x3, dn)
        terms = out[4:7].clone()
        ctx.mark_non_differentiable(normals, labels, cents, out)
        return terms, normals, labels, cents, out

    @staticmethod
    def backward(ctx, g, *_unused):
        rays_o, rays_d, depth, x1, x2, x3, dn = ctx.saved_tensors
        if g is None:
            return (None,) * 11
        ddepth = torch.zeros_like(depth)
        call("ncn_normals_bwd", ptr(rays_o), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(x1.shape[0]),
             ptr(dn), ptr(g.float().contiguous()), ptr(ddepth), stream())
        return None, None, ddepth, None, None, None, None, None, None, None, None


def normals_cluster_losses(rays_o, rays_d, depth, x123_idx, K=20, niter=20, seed=1234, t_similar=0.99,
                           w=(1.0, 1.0, 1.0)):
    """extract_normals_from_ray_batch + cluster_losses fused: (terms, normals, labels, centroids, raw)."""
    f = lambda t: t.float().contiguous()
    idx = lambda t: t.long().contiguous()
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (depth, "depth")):
        if not t.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")
    return _NormalsClusterLoss.apply(f(rays_o), f(rays_d), f(depth), idx(x123_idx["x1"]), idx(x123_idx["x2"]),
                                     idx(x123_idx["x3"]), K, niter, seed, t_similar, _weights_arg(w))


class _PhotoLoss(torch.autograd.Function):
    """losses.py:349-362 with the validity filter: (mean((rgb-gt)^2), w_op * mean(-o log o)) in one
    single-workgroup reduction; the backward is one elementwise launch."""

    @staticmethod
    def forward(ctx, rgb, rgb_gt, opacity, w_op):
        R = rgb.shape[0]
        loss = torch.empty(4, dtype=torch.float32, device=rgb.device)
        call("ncn_photo_loss_fwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(w_op), ptr(loss), stream())
        ctx.save_for_backward(rgb, rgb_gt, opacity, loss)
        ctx.w_op = w_op
        return loss[0], loss[1]

    @staticmethod
    def backward(ctx, g_rgb, g_op):
        rgb, rgb_gt, opacity, loss = ctx.saved_tensors
        dev = rgb.device
        g = torch.stack([torch.zeros((), device=dev) if g_rgb is None else g_rgb.float(),
                         torch.zeros((), device=dev) if g_op is None else g_op.float()])
        drgb, dop = torch.empty_like(rgb), torch.empty_like(opacity)
        call("ncn_photo_loss_bwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(rgb.shape[0]), F32(ctx.w_op), ptr(loss),
             ptr(g), ptr(drgb), ptr(dop), stream())
        return drgb, None, dop, None


def photo_losses(rgb, rgb_gt, opacity, w_opacity):
    """(rgb MSE, weighted opacity entropy), each 0 when non-finite (losses.py:246-262)."""
    f = lambda t: t.float().contiguous()
    check_input(rgb, "rgb")
    check_input(opacity, "opacity")
    if rgb.shape[0] != opacity.shape[0] or rgb_gt.shape != rgb.shape:
        raise ValueError("photo_losses: rgb, rgb_gt and opacity must cover the same rays")
    return _PhotoLoss.apply(f(rgb), f(rgb_gt), f(opacity), float(w_opacity))


class _NeRFLossFused(torch.autograd.Function):
    """NeRFMTLoss of the reference configuration (losses.py:169-587 with rgb + opacity +
    normal-clustering terms, `all_images_triang_patch` 8x8 patches) as ONE autograd node:
    forward = photometric reduction + normals + the clustering pipeline, whose last kernel also
    evaluates the weight schedule from the device step and the total; backward = ONE kernel
    (ncn_nerf_loss_bwd) writing dL/drgb, dL/dopacity and dL/ddepth (gathered per ray).
    Outputs: total, rgb, opacity, ort, centr_dot, centr_L1 (all differentiable, 0-d), then the
    non-differentiable labels, centroids and raw statistics."""

    @staticmethod
    def forward(ctx, rgb, opacity, depth, rays_o, rays_d, rgb_gt, x1, x2, x3, w_op, K, niter, seed, t_sim, w,
                step_dev, sched, count_job=None):
        R = rgb.shape[0]
        T = x1.shape[0]
        dev = rgb.device
        photo = torch.empty(4, dtype=torch.float32, device=dev)
        normals = torch.empty(T, 3, dtype=torch.float32, device=dev)
        cj = count_job  # (custom_functions.CountJob or None)
        tot = cj.total if cj is not None else None
        call("ncn_photo_normals_count_fwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(w_op), ptr(photo),
             ptr(rays_o), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(T), ptr(normals), ptr(tot),
             I64(tot.shape[0] if tot is not None else 0), ptr(cj.counter if cj else None),
             ptr(cj.out if cj else None), ptr(cj.acc if cj else None), stream())
        out = torch.empty(N_OUT, dtype=torch.float32, device=dev)
        labels = torch.empty(T, dtype=torch.int32, device=dev)
        cents = torch.empty(K, 3, dtype=torch.float32, device=dev)
        dn = torch.empty(3, T, 3, dtype=torch.float32, device=dev)
        ws = _cluster_workspace(dev, K)
        call("ncn_cluster_loss", ptr(normals), I64(T), I32(K), I32(niter), ptr(kmeans_plan(dev, T, K, seed)), F32(t_sim), F32(w[0]),
             F32(w[1]), F32(w[2]), ptr(None), ptr(step_dev), F32(sched[0]), F32(sched[1]), ptr(photo), ptr(out),
             ptr(labels), ptr(cents), ptr(dn), ptr(ws), stream())
        ctx.save_for_backward(rgb, opacity, depth, rays_o, rays_d, rgb_gt, photo, dn)
        ctx.w_op = w_op
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(labels, cents, out, normals)
        return out[10], photo[0], photo[1], out[4], out[5], out[6], labels, cents, out, normals

    @staticmethod
    def backward(ctx, g_total, g_rgb, g_op, g_ort, g_cdot, g_cl1, *_unused):
        rgb, opacity, depth, rays_o, rays_d, rgb_gt, photo, dn = ctx.saved_tensors
        dev = rgb.device
        terms = (g_rgb, g_op, g_ort, g_cdot, g_cl1)
        up_terms = None
        if any(g is not None for g in terms):  # a single term back-propagated on its own (rare)
            z = torch.zeros((), device=dev)
            up_terms = torch.stack([z if g is None else g.float().reshape(()) for g in terms]).contiguous()
        up_total = None if g_total is None else g_total.float().contiguous()
        R = rgb.shape[0]
        drgb, dop, ddepth = torch.empty_like(rgb), torch.empty_like(opacity), torch.empty_like(depth)
        call("ncn_nerf_loss_bwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(ctx.w_op), ptr(photo),
             ptr(rays_o), ptr(rays_d), ptr(depth), ptr(dn), ptr(up_total), ptr(up_terms), ptr(drgb), ptr(dop),
             ptr(ddepth), stream())
        return (drgb, dop, ddepth) + (None,) * 15


_STD_PATCH = np.arange(64).reshape(8, 8)
_STD_OFFSETS = (_STD_PATCH[1:, 1:].reshape(-1), _STD_PATCH[:-1, 1:].reshape(-1), _STD_PATCH[1:, :-1].reshape(-1))


def _standard_patch_offsets(patch_area, off):
    """True if the patch triangles are the reference's 8x8 ones (base.py:53-58), host arrays only."""
    if int(patch_area) != 64:
        return False
    for k, ref in zip(("x1", "x2", "x3"), _STD_OFFSETS):
        o = off[k]
        if isinstance(o, torch.Tensor) or not np.array_equal(np.asarray(o).reshape(-1), ref):
            return False
    return True


def _offsets_key(o):
    """Cache key of a host patch-offset array; None for tensors (indexed on the device, never read)."""
    if isinstance(o, torch.Tensor):
        return None
    return bytes(memoryview(np.ascontiguousarray(o, dtype=np.int64)))


class DistortionLoss(torch.autograd.Function):
    """losses.py:16-44: the Mip-NeRF 360 distortion loss in DVGO-v2's O(N) form
    (vren.distortion_loss_fw/bw -> ncn_distortion_loss_fw/bw).  ws, deltas, ts (S), rays_a (R,3)
    -> loss (R) by ray_idx."""

    @staticmethod
    def forward(ctx, ws, deltas, ts, rays_a):
        loss, ws_inclusive_scan, wts_inclusive_scan = vren.distortion_loss_fw(ws, deltas, ts, rays_a)
        ctx.save_for_backward(ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a)
        return loss

    @staticmethod
    def backward(ctx, dL_dloss):
        ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a = ctx.saved_tensors
        dL_dws = vren.distortion_loss_bw(dL_dloss.contiguous(), ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts,
                                         rays_a)
        return dL_dws, None, None, None


class NeRFMTLoss(nn.Module):
    """losses.py:169-587 (hot-path subset, see module docstring)."""

    def __init__(self, hparams_dict):
        super().__init__()
        h = hparams_dict
        self.opacity_w = h.get("loss_opacity_w", 0)
        self.distortion_w = h.get("loss_distortion_w", 0)
        self.depth_w = h.get("loss_depth_w", 0)
        self.sem_w = h.get("loss_sem_w", 0)
        self.manhattan_nerf_w = h.get("loss_manhattan_nerf_w", 0)
        self.norm_DEpth_L1_w = h.get("loss_norm_depth_L1_w", 0)
        self.norm_DEpth_dot_w = h.get("loss_norm_depth_dot_w", 0)
        self.norm_CAN_tres = h.get("loss_norm_can_tres", 0)
        self.norm_D_C_ort_dot_w = h.get("loss_norm_D_C_ort_dot_w", 0)
        self.norm_D_C_centr_dot_w = h.get("loss_norm_D_C_centr_dot_w", 0)
        self.norm_D_C_centr_L1_w = h.get("loss_norm_D_C_centr_L1_w", 0)
        self.norm_D_C_can_dot_w = h.get("loss_norm_D_C_can_dot_w", 0)
        self.norm_D_C_can_L1_w = h.get("loss_norm_D_C_can_L1_w", 0)
        self.reg_depth_w = h.get("loss_reg_depth_w", 0)
        self.ray_sampling_strategy = h.get("ray_sampling_strategy", None)
        self.random_tr_poses = h.get("random_tr_poses", False)
        self.pred_norm_depth = h.get("pred_norm_depth", False)
        self.kmeans_seed = h.get("kmeans_seed", 1234)
        for name in ("sem_w", "manhattan_nerf_w", "norm_D_C_can_dot_w", "norm_D_C_can_L1_w"):
            if getattr(self, name) > 0:
                raise NotImplementedError(f"loss term {name} is not part of the ported hot path (0 in all configs)")
        if self.norm_DEpth_L1_w > 0 or self.norm_DEpth_dot_w > 0:
            self.norm_GT = "normals_depth" if h.get("loss_norm_GT_depth", False) else "normals"
        start = h.get("loss_norm_can_start", 0)
        self.can_sched_start = start
        self.can_sched_end = h.get("loss_norm_can_end", -1)
        grow = h.get("loss_norm_can_grow", 1)
        self.w_sched = lambda w, step: max(0, min(w, (step - start) * (w / grow)))  # losses.py:217
        self._grow = grow
        self.L1_norm = lambda x, y: ((torch.abs(x - y)).sum(-1)).mean()
        self.dot_prod = lambda x, y: (1.0 - torch.nn.CosineSimilarity(dim=-1)(x, y)).mean()
        if self.pred_norm_depth:
            assert self.ray_sampling_strategy in ["all_images_triang", "all_images_triang_val", "same_image_triang",
                                                  "all_images_triang_patch", "same_image_triang_patch"]
        self.last_cluster = None  # (labels, centroids, raw stats) of the last step, for logging/tests
        self.last_normals = None  # (fused path) the normals the clustering saw, for tests
        self._idx_cache = {}
        self._wt = {}

    @staticmethod
    def _validity(loss, dev):
        """losses.py:246-262 without host syncs: non-finite -> 0."""
        if loss.nelement() != 1:
            return torch.tensor(0.0, device=dev)
        return torch.where(torch.isfinite(loss), loss, torch.zeros_like(loss))

    def _fused(self, pred_w_gt, target_gt, pred_unsup, kwargs):
        """The reference configuration in one autograd node (_NeRFLossFused)."""
        f = lambda t: t.float().contiguous()
        step = kwargs["global_step"]
        base = (self.norm_D_C_ort_dot_w, self.norm_D_C_centr_dot_w, self.norm_D_C_centr_L1_w)
        if isinstance(step, torch.Tensor):  # schedule evaluated on the device (graph-captured step)
            step_dev, w = step.to(torch.int64).reshape(()), base
            if not step_dev.is_contiguous():
                step_dev = step_dev.contiguous()
        else:
            if self.can_sched_end != -1 and step > self.can_sched_end:
                w = (0.0, 0.0, 0.0)
            else:
                w = tuple(self.w_sched(x, step) for x in base)
            step_dev = None
        x = pred_unsup["x123_idx"]
        for t, n in ((pred_w_gt["rgb"], "rgb"), (pred_unsup["depth"], "depth")):
            if not t.is_cuda:
                raise RuntimeError(f"{n} must be a CUDA tensor")
        total, l_rgb, l_op, ort, cdot, cl1, labels, cents, raw, normals = _NeRFLossFused.apply(
            f(pred_w_gt["rgb"]), f(pred_unsup["opacity"]), f(pred_unsup["depth"]), f(pred_unsup["rays_o"]),
            f(pred_unsup["rays_d"]), f(target_gt["rgb"]), x["x1"], x["x2"], x["x3"], float(self.opacity_w), 20, 20,
            self.kmeans_seed, 1.0 - self.norm_CAN_tres, w, step_dev, (float(self.can_sched_start), float(self._grow)),
            kwargs.get("count_job"))
        self.last_cluster = (labels, cents, raw)
        self.last_normals = normals  # the patch triangles' normals (zero / invalid ones included)
        return {"rgb": l_rgb, "opacity": l_op, "norm_D_C_ort_dot": ort, "norm_D_C_centr_dot": cdot,
                "norm_D_C_centr_L1": cl1, "total": total}

    def forward(self, pred_raw, target_raw, **kwargs):
        pred_w_gt, target_gt, pred_unsup = {}, {}, {}
        gt_l = target_raw["rgb"].shape[0]
        for k in ("rgb", "depth", "normals", "normals_depth"):
            if k in target_raw:
                target_gt[k] = target_raw[k]
        # slices that cover the whole tensor are skipped: an autograd slice node would cost a
        # zero-fill + copy in the backward for nothing
        head = lambda t: t if t.shape[0] == gt_l else t[:gt_l]
        pred_w_gt["rgb"] = head(pred_raw["rgb"])
        pred_w_gt["depth"] = head(pred_raw["depth"])
        pred_w_gt["rays_o"] = head(pred_raw["rays_o"])
        pred_w_gt["rays_d"] = head(pred_raw["rays_d"])
        unsup_start = gt_l if self.random_tr_poses else 0
        tail = lambda t: t if unsup_start == 0 else t[unsup_start:]
        pred_unsup["opacity"] = pred_raw["opacity"]
        pred_unsup["depth"] = tail(pred_raw["depth"])
        pred_unsup["rays_o"] = tail(pred_raw["rays_o"])
        pred_unsup["rays_d"] = tail(pred_raw["rays_d"])
        dev = pred_raw["rgb"].device

        def get_triang_idx(seq_len):
            pix = einops.rearrange(torch.arange(0, seq_len, device=dev), "(n s) -> n s", s=3)
            return {"x1": pix[:, 0], "x2": pix[:, 1], "x3": pix[:, 2]}

        def get_patch_triang_idx(seq_len, patch_s, off):
            # constant for a given (batch, patch, offsets): cached so the step issues no H2D copies
            key = (seq_len, int(patch_s), str(dev)) + tuple(_offsets_key(off[k]) for k in ("x1", "x2", "x3"))
            hit = None if None in key else self._idx_cache.get(key)
            if hit is None:
                pix = einops.rearrange(torch.arange(0, seq_len, device=dev), "(n s) -> n s", s=patch_s)
                hit = {k: einops.rearrange(pix[:, torch.as_tensor(off[k], device=dev)], "n s -> (n s)").contiguous()
                       for k in ("x1", "x2", "x3")}
                if None not in key:
                    if len(self._idx_cache) > 16:
                        self._idx_cache.clear()
                    self._idx_cache[key] = hit
            return hit

        n_unsup, n_w_gt = pred_unsup["depth"].shape[0], pred_w_gt["rgb"].shape[0]
        if self.ray_sampling_strategy in ["all_images_triang", "same_image_triang"]:
            pred_w_gt["x123_idx"] = get_triang_idx(n_w_gt)
            pred_unsup["x123_idx"] = get_triang_idx(n_unsup)
        elif self.ray_sampling_strategy in ["all_images_triang_patch", "same_image_triang_patch"]:
            off = {"x1": target_raw["x1_offsets_local"], "x2": target_raw["x2_offsets_local"],
                   "x3": target_raw["x3_offsets_local"]}
            pred_w_gt["x123_idx"] = get_patch_triang_idx(n_w_gt, target_raw["patch_area"], off)
            pred_unsup["x123_idx"] = get_patch_triang_idx(n_unsup, target_raw["patch_area"], off)
        clustering = self.norm_D_C_ort_dot_w > 0 or self.norm_D_C_centr_dot_w > 0 or self.norm_D_C_centr_L1_w > 0
        if (clustering and self.pred_norm_depth and unsup_start == 0 and self.opacity_w > 0 and self.distortion_w == 0
                and self.ray_sampling_strategy in ("all_images_triang_patch", "same_image_triang_patch")
                and self.depth_w == 0 and self.norm_DEpth_L1_w == 0 and self.norm_DEpth_dot_w == 0
                and self.reg_depth_w == 0 and n_w_gt == pred_unsup["opacity"].shape[0] and n_w_gt % 64 == 0
                and n_w_gt > 0 and _standard_patch_offsets(target_raw["patch_area"], off)):
            return self._fused(pred_w_gt, target_gt, pred_unsup, dict(kwargs, count_job=pred_raw.get("_count_job")))
        job = pred_raw.get("_count_job")
        if job is not None:  # render left its sample count to the fused node, not used in this configuration
            call("ncn_count_samples", ptr(job.total), I64(job.total.shape[0]), ptr(job.counter), ptr(job.out),
                 ptr(job.acc), stream())
        fuse_normals = (clustering and self.pred_norm_depth and unsup_start == 0 and self.norm_DEpth_L1_w == 0
                        and self.norm_DEpth_dot_w == 0)
        if self.pred_norm_depth and not fuse_normals:
            pred_w_gt["norm_depth"] = extract_normals_from_ray_batch(pred_w_gt["rays_o"], pred_w_gt["rays_d"],
                                                                     pred_w_gt["depth"], pred_w_gt["x123_idx"])
            if unsup_start == 0:
                pred_unsup["norm_depth"] = pred_w_gt["norm_depth"]
            else:
                pred_unsup["norm_depth"] = extract_normals_from_ray_batch(pred_unsup["rays_o"], pred_unsup["rays_d"],
                                                                          pred_unsup["depth"], pred_unsup["x123_idx"])
        loss_d = {}
        if self.opacity_w > 0 and pred_w_gt["rgb"].shape[0] == pred_unsup["opacity"].shape[0]:
            loss_d["rgb"], loss_d["opacity"] = photo_losses(pred_w_gt["rgb"], target_gt["rgb"], pred_unsup["opacity"],
                                                            self.opacity_w)
        else:
            rgb_loss = ((pred_w_gt["rgb"] - target_gt["rgb"]) ** 2).mean()
            loss_d["rgb"] = self._validity(rgb_loss, dev)
        if self.opacity_w > 0 and "opacity" not in loss_d:
            o = pred_unsup["opacity"] + 1e-10
            loss_d["opacity"] = self._validity(self.opacity_w * (-o * torch.log(o)).mean(), dev)
        if self.distortion_w > 0:  # losses.py:365-369 with quirk q5: ws := ts (losses.py:290)
            ts = pred_raw["ts"].float().contiguous()
            dist = DistortionLoss.apply(ts, pred_raw["deltas"].float().contiguous(), ts, pred_raw["rays_a"].contiguous())
            loss_d["distortion"] = self._validity(self.distortion_w * dist.mean(), dev)
        if self.depth_w > 0:
            d_pred, d_tgt = pred_w_gt["depth"], target_gt["depth"]
            valid = d_tgt > 0
            loss_d["depth"] = self._validity(self.depth_w * ((d_pred[valid] - d_tgt[valid]) ** 2).mean(), dev)
        if self.norm_DEpth_L1_w > 0 or self.norm_DEpth_dot_w > 0:
            nd = pred_w_gt["norm_depth"]
            tgt = target_gt[self.norm_GT][pred_w_gt["x123_idx"]["x1"]]
            valid = tgt.abs().sum(-1) > 0
            if self.norm_DEpth_L1_w > 0:
                loss_d["norm_D_L1"] = self._validity(self.norm_DEpth_L1_w * self.L1_norm(nd[valid], tgt[valid]), dev)
            if self.norm_DEpth_dot_w > 0:
                loss_d["norm_D_dot"] = self._validity(self.norm_DEpth_dot_w * self.dot_prod(nd[valid], tgt[valid]),
                                                      dev)
        step_t = isinstance(kwargs.get("global_step"), torch.Tensor)
        if step_t and (self.reg_depth_w > 0 or self.can_sched_end != -1):
            raise NotImplementedError("a device global_step needs step-independent control flow "
                                      "(loss_reg_depth_w == 0 and loss_norm_can_end == -1)")
        if self.reg_depth_w > 0 and kwargs["global_step"] > self.can_sched_start:
            d_pred, x = pred_unsup["depth"], pred_unsup["x123_idx"]
            reg = ((d_pred[x["x1"]] - d_pred[x["x2"]]) ** 2 + (d_pred[x["x1"]] - d_pred[x["x3"]]) ** 2).mean()
            loss_d["reg_depth"] = self._validity(reg, dev)
        if clustering:
            step = kwargs["global_step"]
            if step_t or step <= self.can_sched_end or self.can_sched_end == -1:
                if step_t:  # the schedule on the device (graph-captured step): clamp((s-start)*w/grow, 0, w)
                    wt = self._wt.get(dev)
                    if wt is None:  # created once, before any capture (no H2D copy inside a graph)
                        wt = torch.tensor([self.norm_D_C_ort_dot_w, self.norm_D_C_centr_dot_w,
                                           self.norm_D_C_centr_L1_w], dtype=torch.float32, device=dev)
                        self._wt[dev] = wt
                    ramp = (step.float() - float(self.can_sched_start)) * (wt / float(self._grow))
                    w = torch.minimum(torch.clamp_min(ramp, 0.0), wt)
                else:
                    w = (self.w_sched(self.norm_D_C_ort_dot_w, step), self.w_sched(self.norm_D_C_centr_dot_w, step),
                         self.w_sched(self.norm_D_C_centr_L1_w, step))
                if fuse_normals:
                    terms, _normals, labels, cents, raw = normals_cluster_losses(
                        pred_unsup["rays_o"], pred_unsup["rays_d"], pred_unsup["depth"], pred_unsup["x123_idx"], K=20,
                        niter=20, seed=self.kmeans_seed, t_similar=1.0 - self.norm_CAN_tres, w=w)
                else:
                    terms, labels, cents, raw = cluster_losses(pred_unsup["norm_depth"], K=20, niter=20,
                                                               seed=self.kmeans_seed,
                                                               t_similar=1.0 - self.norm_CAN_tres, w=w)
                loss_d["norm_D_C_ort_dot"] = terms[0]
                loss_d["norm_D_C_centr_dot"] = terms[1]
                loss_d["norm_D_C_centr_L1"] = terms[2]
                self.last_cluster = (labels, cents, raw)
        loss_d["total"] = sum(lo for lo in loss_d.values())
        return loss_d
