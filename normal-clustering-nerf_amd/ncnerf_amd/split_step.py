"""The reference configuration's training step as an explicit kernel sequence with the backward
split by the gradient's source (Trainer's graph step, `split_backward`).

Same computation as render() -> NeRFMTLoss -> backward (train_nerf.py:165-358 with the loss terms
of the reference configuration, losses.py:349-362 + 420-478): the same kernels on the same inputs,
so the losses are bit-identical and the gradients agree up to f32 summation order.  What changes is
the order: the autograd backward can only start once the whole loss node (photometric + normals +
the normal clustering, ~90 us of latency-bound k-means in 16 workgroups) has finished, while the
photometric gradient does not depend on the clustering at all.  Here the photometric part is
back-propagated on a side stream while the clustering runs:

  main:  march -> field fwd -> composite fw -> photo+normals fwd -+-> cluster loss (k-means)
                                                                   |   -> loss bwd (depth)
  side:                                                            +-> loss bwd (rgb, opacity)
                                                                       -> composite bw (rgb)
                                                                       -> field MLP bwd, rgb part
  main (after the join): composite bw (all terms) -> field MLP bwd, sigma part -> table scatter
                         (+ the dW slab reduction in the same launch)

The rgb_net's input gradient dL/draws = w * dL/drgb needs only the photometric term, so the first
composite backward yields it exactly as the joint one would; dL/dsigma mixes all three upstream
terms and comes from the second (joint) composite backward after the clustering.
ncn_field_bwd_mlp_part's rgb pass takes the rgb_net weight gradients and the rgb part of dL/dh
(stashed in fp32); the sigma pass adds TruncExp'(h0) dL/dsigma and finishes the sigma_net and
encoding gradients.  Every per-sample value is therefore bit-identical to the autograd step's;
only the float-atomic flush order of the table gradient differs, as between any two runs.  The rgb
pass uses at most SPLIT_BLOCKS workgroups so the clustering's 16 co-resident workgroups keep CUs
of their own (an rgb-pass workgroup takes a whole CU's LDS); the sigma pass keeps only the
sigma_net's fragments and exchange tiles in LDS and runs two workgroups per CU.  Only the
fused-loss configuration takes this path (split_eligible), and only on a device that can hold the
clustering beside the rgb pass (SplitStep refuses otherwise); anything else falls back to the
autograd step."""
import ctypes

import torch

from . import _lib, vren
from ._lib import F32, I32, I64, call, ptr, stream
from .losses import N_OUT, _cluster_workspace, _standard_patch_offsets, kmeans_plan
from .ngp_mt import N_W
from .rendering import march_train_fused

SPLIT_BLOCKS = 240  # MLP-backward workgroups of each split pass at most: 256 CUs - the clustering's 16
K_CLUSTERS, K_ITERS = 20, 20  # NeRFMTLoss._fused (losses.py:86-89: faiss.Kmeans(3, 20, niter=20))
KM_BLOCKS = 16  # the clustering kernel's co-resident workgroups (csrc/loss.hip KM_BLOCKS)


def split_rgb_blocks(cus, per_cu, cap=SPLIT_BLOCKS):
    """The rgb pass's workgroups on a device of `cus` CUs where `per_cu` clustering workgroups fit
    per CU: every CU but the ceil(KM_BLOCKS / per_cu) the clustering needs, at most `cap` (240 on
    MI355X's 256 CUs).  0 when the device cannot hold the clustering at all."""
    if cus <= 0 or per_cu <= 0:
        return 0
    return max(0, min(cap, cus - -(-KM_BLOCKS // per_cu)))


def device_rgb_blocks():
    """split_rgb_blocks for the current device (ncn_cluster_coresidency with no busy CUs reports
    cus x per_cu)."""
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    cap = ctypes.c_int(0)
    _lib.lib().ncn_cluster_coresidency(I32(K_CLUSTERS), I32(0), ctypes.byref(cap))  # rc != 0 leaves cap < 16
    return split_rgb_blocks(cus, cap.value // max(cus, 1))


def split_eligible(trainer, batch):
    """True when the step is the reference configuration the fused loss node serves (the condition
    of NeRFMTLoss.forward's fused branch) on the static-shape white-background render."""
    L, m, kw = trainer.loss, trainer.model, trainer.render_kwargs
    R = batch["rays_o"].shape[0]
    clustering = L.norm_D_C_ort_dot_w > 0 or L.norm_D_C_centr_dot_w > 0 or L.norm_D_C_centr_L1_w > 0
    off = {k: batch.get(k + "_offsets_local") for k in ("x1", "x2", "x3")}
    return (clustering and L.pred_norm_depth and not L.random_tr_poses and L.opacity_w > 0 and L.distortion_w == 0
            and L.ray_sampling_strategy in ("all_images_triang_patch", "same_image_triang_patch")
            and L.depth_w == 0 and L.norm_DEpth_L1_w == 0 and L.norm_DEpth_dot_w == 0 and L.reg_depth_w == 0
            and R > 0 and R % 64 == 0 and R <= 16384 and batch["rgb"].shape[0] == R
            and all(v is not None for v in off.values()) and _standard_patch_offsets(batch.get("patch_area", 0), off)
            and not m.pred_norm and not m.pred_sem and getattr(m, "_aabb", None) is not None
            and kw.get("exp_step_factor", 0.0) == 0 and kw.get("anneal_strategy", "none") == "none"
            and not kw.get("random_bg", False)
            and not any(isinstance(v, torch.Tensor) for k, v in kw.items() if k != "count_acc"))


class SplitStep:
    """One training step (forward + split backward) of `trainer`'s model; run() is graph-capturable
    (no host reads).  Buffers that depend only on the batch size are allocated once."""

    def __init__(self, trainer, rgb_blocks=None):
        """rgb_blocks: the rgb pass's workgroups (one per CU), which run beside the clustering; by
        default sized from the device (device_rgb_blocks: 240 on MI355X, fewer on a smaller part).
        The clustering's workgroups meet at grid barriers, so they must all stay resident on the CUs
        the rgb pass leaves: checked here (ncn_cluster_coresidency), before the step is captured — a
        configuration where they cannot is refused (NcnError) instead of spinning into the barrier
        timeout, and Trainer then runs the autograd step.  (At N > 1
        nothing else shares the step: the all-reduce of step k is stream-ordered before graph k+1,
        and RCCL's channels run beside the deferred coarse-level scatter, which leaves them 32 CUs,
        distributed.DP_SCATTER_BLOCKS.)"""
        self.tr = trainer
        self._tri = None
        self.rgb_blocks = device_rgb_blocks() if rgb_blocks is None else int(rgb_blocks)
        if self.rgb_blocks < 1:
            raise _lib.NcnError("SplitStep: the device cannot hold the clustering's workgroups beside an rgb pass")
        cap = ctypes.c_int(0)
        call("ncn_cluster_coresidency", I32(K_CLUSTERS), I32(self.rgb_blocks), ctypes.byref(cap))
        self.cluster_capacity = cap.value

    def _triangles(self, R, dev):
        # the 8x8 patch triangles of losses.py:307-313 (x1/x2/x3 = the standard patch offsets)
        if self._tri is None or self._tri[0] != R or self._tri[1] != dev:
            pix = torch.arange(R, device=dev).view(-1, 64)
            from .losses import _STD_OFFSETS
            tri = tuple(pix[:, torch.as_tensor(o, device=dev)].reshape(-1).contiguous() for o in _STD_OFFSETS)
            self._tri = (R, dev, tri)
        return self._tri[2]

    def run(self, batch, step_dev, premarched=None):
        tr, m, L = self.tr, self.tr.model, self.tr.loss
        kw = tr.render_kwargs
        rays_o, rays_d = batch["rays_o"].contiguous().float(), batch["rays_d"].contiguous().float()
        R, dev = rays_o.shape[0], rays_o.device
        # ---- render (rendering.py:152-242 via render_rays_train's static-shape path) ----
        pm = premarched
        if pm is None:
            if not getattr(m, "_packed_fresh", False):
                m.prepare_weights()
            pm = march_train_fused(m, rays_o, rays_d, kw["near_distance"], kw["max_samples"], batch.get("march_noise"),
                                   None if "march_noise" in batch else (tr._rng_seed, step_dev))
        rays_a, xyzs, dirs, deltas, ts = pm["rays_a"], pm["xyzs"], pm["dirs"], pm["deltas"], pm["ts"]
        T_thr = kw.get("T_threshold", 1e-4)  # render_rays_train's default (rendering.py:170)
        n_dev = pm["counter"][0]
        n = xyzs.shape[0]
        sigmas, rgbs, enc, packed, order = m._field_fwd(xyzs, dirs, n_dev, 0, True)
        total_s, opacity, depth, rend, ws, rgb = vren.composite_train_multi_fw(sigmas, rgbs, deltas, ts, rays_a,
                                                                              T_thr, bg=1.0)
        # ---- NeRFMTLoss forward (_NeRFLossFused.forward) ----
        x1, x2, x3 = self._triangles(R, dev)
        T = x1.shape[0]
        photo = torch.empty(4, dtype=torch.float32, device=dev)
        normals = torch.empty(T, 3, dtype=torch.float32, device=dev)
        cnt = torch.empty((), dtype=torch.int64, device=dev)
        acc = kw.get("count_acc")
        rgb_gt = batch["rgb"].contiguous().float()
        # (the normals use results["rays_o"] = rays_d, rendering.py:227 quirk q1)
        call("ncn_photo_normals_count_fwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(L.opacity_w), ptr(photo),
             ptr(rays_d), ptr(rays_d), ptr(depth), ptr(x1), ptr(x2), ptr(x3), I64(T), ptr(normals), ptr(total_s),
             I64(R), ptr(n_dev if acc is not None else None), ptr(cnt), ptr(acc), stream())
        out = torch.empty(N_OUT, dtype=torch.float32, device=dev)
        labels = torch.empty(T, dtype=torch.int32, device=dev)
        cents = torch.empty(K_CLUSTERS, 3, dtype=torch.float32, device=dev)
        dn = torch.empty(3, T, 3, dtype=torch.float32, device=dev)
        cws = _cluster_workspace(dev, K_CLUSTERS)
        plan = kmeans_plan(dev, T, K_CLUSTERS, L.kmeans_seed)
        w = (L.norm_D_C_ort_dot_w, L.norm_D_C_centr_dot_w, L.norm_D_C_centr_L1_w)
        one = tr._unit(dev)
        lib = _lib.lib()
        nb = (min(self.rgb_blocks, int(lib.ncn_field_bwd_part_blocks(I64(n), I32(1)))),
              int(lib.ncn_field_bwd_part_blocks(I64(n), I32(2))))  # (the sigma pass: two workgroups per CU)
        drgb, dop, ddepth = torch.empty_like(rgb), torch.empty_like(opacity), torch.empty_like(depth)
        slab = torch.empty(max(nb) * N_W, dtype=torch.float32, device=dev)
        dE_ws = torch.empty(int(lib.ncn_field_bwd_dE_floats(I64(n))), dtype=torch.float32, device=dev)
        stash = torch.empty(int(lib.ncn_field_bwd_stash_floats(I64(n))), dtype=torch.float32, device=dev)
        lmax = m._level_max()
        scale = m._bwd_loss_scale()
        g_table, g_w = m._grad_views()

        def mlp_part(part, dsig, drw):
            call("ncn_field_bwd_mlp_part", ptr(xyzs), ptr(dirs), I64(n), ptr(n_dev), ptr(order), ptr(packed), I32(m._prec),
                 ptr(enc), ptr(dsig), ptr(None), ptr(drw), ptr(scale), I32(part), I32(nb[part - 1]), ptr(slab),
                 ptr(dE_ws),
                 ptr(lmax), ptr(stash), stream())

        # the photometric backward on a side stream (its first launch waits for the fork; the
        # clustering, issued first on this stream, takes its CUs before the rgb pass fills the rest)
        cur = torch.cuda.current_stream(dev)
        side = tr._side_stream()
        side.wait_stream(cur)
        call("ncn_cluster_loss", ptr(normals), I64(T), I32(K_CLUSTERS), I32(K_ITERS), ptr(plan),
             F32(1.0 - L.norm_CAN_tres), F32(w[0]), F32(w[1]), F32(w[2]), ptr(None), ptr(step_dev),
             F32(float(L.can_sched_start)), F32(float(L._grow)), ptr(photo), ptr(out), ptr(labels), ptr(cents),
             ptr(dn), ptr(cws), stream())
        with torch.cuda.stream(side):
            # ---- photometric backward: loss -> composite -> field MLP (rgb part) ----
            call("ncn_nerf_loss_bwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(L.opacity_w), ptr(photo),
                 ptr(rays_d), ptr(rays_d), ptr(depth), ptr(None), ptr(one), ptr(None), ptr(drgb), ptr(dop),
                 ptr(None), stream())
            # dL/draws = w * dL/drgb: the photometric gradient alone, bit for bit the joint backward's
            _, draws = vren.composite_train_multi_bw(dop, None, drgb, None, sigmas, rgbs, ws, deltas, ts, rays_a,
                                                     opacity, depth, rend, T_thr, bg=1.0)
            mlp_part(1, None, draws)
        # ---- clustering backward: loss (depth) -> composite (all terms) -> field MLP (sigma part) ----
        call("ncn_nerf_loss_bwd", ptr(rgb), ptr(rgb_gt), ptr(opacity), I64(R), F32(L.opacity_w), ptr(photo),
             ptr(rays_d), ptr(rays_d), ptr(depth), ptr(dn), ptr(one), ptr(None), ptr(None), ptr(None), ptr(ddepth),
             stream())
        cur.wait_stream(side)
        # dL/dsigma from all three upstream terms in one expression, as the autograd step's backward
        dsig, _ = vren.composite_train_multi_bw(dop, ddepth, drgb, None, sigmas, rgbs, ws, deltas, ts, rays_a,
                                                opacity, depth, rend, T_thr, bg=1.0)
        mlp_part(2, dsig, None)
        m._scatter(xyzs, n, n_dev, order, dE_ws, lmax, g_table, wgrad=(slab, nb[1], nb[0], g_w))
        L.last_cluster = (labels, cents, out)
        L.last_normals = normals
        results = {"rays_a": rays_a, "deltas": deltas, "ts": ts, "rm_samples": n_dev, "vr_samples": cnt,
                   "opacity": opacity, "depth": depth, "ws": ws, "rgb": rgb, "rays_d": rays_d, "rays_o": rays_d,
                   "total_samples": total_s}
        loss_d = {"rgb": photo[0], "opacity": photo[1], "norm_D_C_ort_dot": out[4], "norm_D_C_centr_dot": out[5],
                  "norm_D_C_centr_L1": out[6], "total": out[10]}
        return results, loss_d
