"""autograd.Functions of the reference models/custom_functions.py:8-173, backed by the HIP `vren`.

Same class names, `apply` signatures, outputs and `custom_fwd(cast_inputs=float32)` behaviour.
"""
import torch
from torch.amp import custom_bwd, custom_fwd

from . import vren


class RayAABBIntersector(torch.autograd.Function):
    """custom_functions.py:8-29 -> (hits_cnt (R), hits_t (R,max_hits,2), hits_voxel_idx (R,max_hits))"""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, center, half_size, max_hits):
        return tuple(vren.ray_aabb_intersect(rays_o, rays_d, center, half_size, max_hits))


class RayMarcher(torch.autograd.Function):
    """custom_functions.py:55-112.

    forward -> (rays_a, xyzs, dirs, deltas, ts, total_samples).  `noise` is drawn on device as in
    the reference (custom_functions.py:83); tests may pass an explicit `noise` tensor (quirk q8).
    backward (:102-112): the reference's torch_scatter.segment_csr over indptr = [rays_a[:, 1],
    rays_a[-1, 1] + rays_a[-1, 2]] — row i of dL/drays_o is the sum of dL/dxyzs over samples
    [indptr[i], indptr[i+1]), row i of dL/drays_d the same sum of dL/dxyzs * t + dL/ddirs — as one
    HIP launch (ncn_segment_csr: a wave per row, fixed summation order, no atomics).  Rows map
    to ray rows by position (the reference's rows are ray-ordered, rays_a[i, 0] == i, and so are
    this marcher's, with starts in ray order, so every segment is exactly ray i's samples)."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, grid_size,
                max_samples, noise=None, static_capacity=False):
        if noise is None:
            noise = torch.rand_like(rays_o[:, 0])
        rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
            rays_o, rays_d, hits_t.contiguous(), density_bitfield, cascades, scale, exp_step_factor, noise.contiguous(),
            grid_size, max_samples, static_capacity=static_capacity)
        total_samples = counter[0]  # with static_capacity: THE device count (n_samples_dev) of the arrays
        ctx.save_for_backward(rays_a, ts)
        ctx.n_rays = rays_o.shape[0]
        ctx.static_capacity = static_capacity
        return rays_a, xyzs, dirs, deltas, ts, total_samples

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_drays_a, dL_dxyzs, dL_ddirs, dL_ddeltas, dL_dts, dL_dtotal_samples):
        rays_a, ts = ctx.saved_tensors
        if ctx.static_capacity:
            raise NotImplementedError("ray gradients are not available on the static-capacity (graph) path")
        c = lambda t: None if t is None else t.contiguous().float()  # noqa: E731
        dL_drays_o, dL_drays_d = vren.raymarching_train_backward(c(dL_dxyzs), c(dL_ddirs), ts, rays_a)
        return dL_drays_o, dL_drays_d, None, None, None, None, None, None, None, None, None


class VolumeRenderer(torch.autograd.Function):
    """custom_functions.py:115-159 -> (total_samples (scalar), opacity, depth, rend, ws).

    Unused output gradients arrive as None (set_materialize_grads(False)) and are passed to the
    kernel as NULL instead of zero tensors — numerically identical to the reference, which
    receives materialised zeros."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, sigmas, raws, deltas, ts, rays_a, T_threshold):
        sigmas = sigmas.contiguous(); raws = raws.contiguous()
        total_samples, opacity, depth, rend, ws = vren.composite_train_multi_fw(sigmas, raws, deltas, ts, rays_a,
                                                                                  T_threshold)
        ctx.save_for_backward(sigmas, raws, deltas, ts, rays_a, opacity, depth, rend, ws)
        ctx.T_threshold = T_threshold
        ctx.set_materialize_grads(False)
        return vren.count_samples(total_samples), opacity, depth, rend, ws

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_dtotal_samples, dL_dopacity, dL_ddepth, dL_drend, dL_dws):
        sigmas, raws, deltas, ts, rays_a, opacity, depth, rend, ws = ctx.saved_tensors
        c = lambda t: None if t is None else t.contiguous().float()
        dL_dsigmas, dL_draws = vren.composite_train_multi_bw(c(dL_dopacity), c(dL_ddepth), c(dL_drend), c(dL_dws),
                                                             sigmas, raws, ws, deltas, ts, rays_a, opacity, depth,
                                                             rend, ctx.T_threshold)
        return dL_dsigmas, dL_draws, None, None, None, None


class CountJob:
    """The render's sample count handed to the loss node (Trainer's graph step): a plain object, not
    a dict or tuple, so autocast's input casting of the autograd Function passes it through as is."""
    __slots__ = ("total", "counter", "acc", "out")

    def __init__(self):
        self.total = self.counter = self.acc = self.out = None


class VolumeRendererBg(torch.autograd.Function):
    """VolumeRenderer followed by render()'s background blend (rendering.py:232-240) as one node:
    -> (total_samples, opacity, depth, rgb = rend + bg * (1 - opacity), ws).  Same kernels with the
    blend in the forward's epilogue and its opacity gradient in the backward (no torch glue)."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, sigmas, raws, deltas, ts, rays_a, T_threshold, bg, count=None):
        sigmas = sigmas.contiguous(); raws = raws.contiguous()
        total_samples, opacity, depth, rend, ws, rgb = vren.composite_train_multi_fw(sigmas, raws, deltas, ts, rays_a,
                                                                                       T_threshold, bg=bg)
        ctx.save_for_backward(sigmas, raws, deltas, ts, rays_a, opacity, depth, rend, ws)
        ctx.T_threshold, ctx.bg = T_threshold, bg
        ctx.set_materialize_grads(False)
        # count = (the marcher's device counter, a float64 (2,) accumulator[, job]) or None
        # (ncn_count_samples); with a job dict the count is left to the loss node's first launch
        # (ncn_photo_normals_count_fwd): cnt is filled there, the caller must run that loss
        if count is not None and len(count) > 2 and count[2] is not None:
            cnt = torch.empty((), dtype=torch.int64, device=sigmas.device)
            job = count[2]
            job.total, job.counter, job.acc, job.out = total_samples, count[0], count[1], cnt
        else:
            cnt = vren.count_samples(total_samples, *(count[:2] if count is not None else ()))
        return cnt, opacity, depth, rgb, ws

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_dtotal_samples, dL_dopacity, dL_ddepth, dL_drgb, dL_dws):
        sigmas, raws, deltas, ts, rays_a, opacity, depth, rend, ws = ctx.saved_tensors
        c = lambda t: None if t is None else t.contiguous().float()
        dL_dsigmas, dL_draws = vren.composite_train_multi_bw(c(dL_dopacity), c(dL_ddepth), c(dL_drgb), c(dL_dws),
                                                             sigmas, raws, ws, deltas, ts, rays_a, opacity, depth,
                                                             rend, ctx.T_threshold, bg=ctx.bg)
        return dL_dsigmas, dL_draws, None, None, None, None, None, None, None


class TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173 (the field kernel fuses this; kept for API parity)."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_dout):
        x = ctx.saved_tensors[0]
        return dL_dout * torch.exp(x.clamp(-15, 15))
