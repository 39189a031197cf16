"""ORACLE — test infrastructure only: the pure-PyTorch/C CPU training step used as bench.py's
`cpu_baseline` leg (kind "port") and as the CPU side of the end-to-end tests.

Same step as ncnerf_amd/trainer.py, built only from the oracle restatements:
  ray/AABB + near clamp (rendering.py:24-28) -> train marcher (oracle C) -> field (oracle torch,
  fp32) -> composite fw/bw (oracle C inside an autograd.Function, custom_functions.py:115-159) ->
  white background (rendering.py:232-240) -> rgb MSE + opacity + normals-from-depth + clustering
  losses (losses_ref) -> backward -> global-norm clip 0.05 + AdamW(eps 1e-15) (train_nerf.py:262-285).
"""
import math

import numpy as np
import torch

from . import field_ref, losses_ref, vren_ref


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigmas, raws, deltas, ts, rays_a, thr):
        tot, op, de, rend, ws = vren_ref.composite_train_multi_fw(sigmas, raws, deltas, ts, rays_a, thr)
        T = lambda a: torch.from_numpy(a)
        ctx.save_for_backward(sigmas.detach(), raws.detach(), deltas, ts, rays_a, T(op), T(de), T(rend), T(ws))
        ctx.thr = thr
        return torch.tensor(float(tot.sum())), T(op), T(de), T(rend), T(ws)

    @staticmethod
    def backward(ctx, _g_tot, dO, dD, dR, dW):
        sig, raws, deltas, ts, rays_a, op, de, rend, ws = ctx.saved_tensors
        z = lambda g, like: torch.zeros_like(like) if g is None else g
        ds, dr = vren_ref.composite_train_multi_bw(z(dO, op), z(dD, de), z(dR, rend), None if dW is None else dW, sig,
                                                   raws, ws, deltas, ts, rays_a, op, de, rend, ctx.thr)
        return torch.from_numpy(ds), torch.from_numpy(dr), None, None, None, None


def render_train_ref(P, levels, rays_o, rays_d, bitfield, noise, near=0.01, max_samples=1024, T_thr=1e-4,
                     impl="torch", emulate=None):
    """rendering.py:9-42 + 152-242 (train path, exp_step_factor 0) on the oracle: returns the
    differentiable rgb (with white background), depth, opacity and the marcher/compositor outputs."""
    o, d = np.ascontiguousarray(rays_o, np.float32), np.ascontiguousarray(rays_d, np.float32)
    _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
    ht = ht[:, 0].copy()
    nearm = (ht[:, 0] >= 0) & (ht[:, 0] < near)
    ht[nearm, 0] = near
    rays_a, xyzs, dirs, deltas, ts, counter = vren_ref.raymarching_train(o, d, ht, bitfield, 1, 0.5, 0.0, noise, 128,
                                                                         max_samples)
    sig, rgb, _ = field_ref.field_forward_autograd(torch.from_numpy(xyzs), torch.from_numpy(dirs), P, levels,
                                                   impl=impl, emulate=emulate)
    vr, opacity, depth, rend, ws = _Composite.apply(sig, rgb, torch.from_numpy(deltas), torch.from_numpy(ts),
                                                    torch.from_numpy(rays_a), T_thr)
    return dict(rgb=rend + 1.0 * (1 - opacity)[:, None], depth=depth, opacity=opacity, ws=ws, rays_a=rays_a,
                deltas=deltas, ts=ts, rm_samples=int(counter[0]), vr_samples=int(vr))


class CPUTrainer:
    """Hypersim config: scale 0.5, G 128, max_samples 1024, near 0.01, loss weights as the trainer."""

    def __init__(self, bitfield, seed=0, lr=1e-2, w_cluster=2e-3, opacity_w=1e-3, num_epochs=None, epoch_steps=1000,
                 encode_impl="torch", emulate=None, emulate_bwd=False):
        """encode_impl: "torch" (field_ref.hash_encode, the pure-PyTorch path of config #1) or "c"
        (its C restatement, oracle/hashgrid_ref.c: the same algorithm ~10x faster, for the PSNR
        seed ensembles).
        emulate_bwd (with emulate): the field backward's gradients rounded as the HIP kernel's
        loss-scaled fp16 chain rounds them (field_ref.field_forward_autograd bwd_scale = 128 x S),
        with the GradScaler that S comes from (torch.cuda.amp.GradScaler defaults, as the HIP
        optimizer's: init 2^16, a non-finite gradient skips the step and halves S, 2000 finite steps
        in a row double it)."""
        self.encode_impl = encode_impl
        self.emulate = emulate  # "fp16": the MLP operands rounded as tcnn's / the HIP kernel's (field_ref)
        self.emulate_bwd = bool(emulate_bwd) and emulate is not None
        self.amp_S, self.amp_tracker, self.amp_skips = 65536.0, 0, 0
        P, self.levels = field_ref.init_params(seed=seed)
        self.params = [t.requires_grad_(True) for t in P.tensors()]
        self.P = field_ref.FieldParams(*self.params)
        self.bitfield = np.ascontiguousarray(bitfield, np.uint8)
        self.opt = torch.optim.AdamW([{"params": self.params[:1], "weight_decay": 0.0},
                                      {"params": self.params[1:], "weight_decay": 1e-6}], lr=lr, eps=1e-15)
        self.w_cluster, self.opacity_w = w_cluster, opacity_w
        # CosineAnnealingLR(T_max=num_epochs) stepped per epoch of `epoch_steps` steps
        # (train_nerf.py:286-288; base.py:78-81); None keeps lr constant
        self.base_lr, self.num_epochs, self.epoch_steps = lr, num_epochs, epoch_steps

    def set_lr_for_step(self, global_step):
        if not self.num_epochs:
            return
        e = global_step // self.epoch_steps
        lr = 0.5 * self.base_lr * (1 + math.cos(math.pi * e / self.num_epochs))
        for g in self.opt.param_groups:
            g["lr"] = lr

    def load_state(self, flat_params, exp_avg, exp_avg_sq, adam_step, amp_scale=None, amp_tracker=0, bitfield=None):
        """Continue from another trainer's state (a HIP training snapshot): the flat fp32 parameter
        buffer [table | W1 | W2 | W3 | W4 | W5] (ncnerf_amd NGPMT.flat_params order), Adam's flat first
        and second moments and its step count (AdamW's per-parameter `step`, identical for every
        parameter), the GradScaler's scale / growth tracker, the occupancy bitfield."""
        flat = [torch.as_tensor(np.asarray(a, np.float32)).reshape(-1) for a in (flat_params, exp_avg, exp_avg_sq)]
        off = 0
        with torch.no_grad():
            for p in self.params:
                n = p.numel()
                p.copy_(flat[0][off:off + n].view_as(p))
                self.opt.state[p] = {"step": torch.tensor(float(adam_step)),
                                     "exp_avg": flat[1][off:off + n].view_as(p).clone(),
                                     "exp_avg_sq": flat[2][off:off + n].view_as(p).clone()}
                off += n
        assert off == flat[0].numel(), (off, flat[0].numel())
        if amp_scale is not None:
            self.amp_S, self.amp_tracker = float(amp_scale), int(amp_tracker)
        if bitfield is not None:
            self.bitfield = np.ascontiguousarray(bitfield, np.uint8)

    def step(self, batch, global_step=3000, noise=None, record=None, force_labels=None, force_signs=None):
        """One training step; `noise` (R,) injects the marcher's perturbation (default torch.rand).
        record (a dict, optional) receives the step's intermediate values: the loss terms (as
        NeRFMTLoss names them, weighted), the unweighted cluster terms, the valid-normal mask and the
        cluster labels of the valid normals, the gradient of every parameter before the clip (the
        unscaled gradient the optimizer receives) and whether the GradScaler skipped the step.
        force_labels (int array over the valid normals, optional): the cluster losses use these labels
        (e.g. the HIP step's) instead of this step's own k-means — whose labels are still computed and
        recorded — so that what follows the clustering is compared on identical clusters.
        force_signs (optional, with force_labels): the branches of the cluster terms' absolute values
        (losses_ref.kink_signs of the other side's normals); the record then counts how many of this
        step's own branches differ from them (`sign_mismatch`)."""
        o, d = batch["rays_o"], batch["rays_d"]
        R = o.shape[0]
        _, ht, _ = vren_ref.ray_aabb_intersect(o, d, np.zeros((1, 3), np.float32), np.full((1, 3), 0.5, np.float32), 1)
        ht = ht[:, 0].copy()
        near = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
        ht[near, 0] = 0.01
        noise = torch.rand(R).numpy() if noise is None else np.ascontiguousarray(noise, np.float32)
        self.set_lr_for_step(global_step)
        rays_a, xyzs, dirs, deltas, ts, counter = vren_ref.raymarching_train(o, d, ht, self.bitfield, 1, 0.5, 0.0,
                                                                             noise, 128, 1024)
        self.opt.zero_grad()
        # the kernel's backward chain scale: fp16 at tcnn's 128 x the GradScaler's S; bf16 unscaled (no
        # GradScaler: PL's bf16 mode, tcnn's non-fp16 modules)
        K = (128.0 * self.amp_S if self.emulate == "fp16" else 1.0) if self.emulate_bwd else None
        sig, rgb, _ = field_ref.field_forward_autograd(torch.from_numpy(xyzs), torch.from_numpy(dirs), self.P,
                                                       self.levels, impl=self.encode_impl, emulate=self.emulate,
                                                       bwd_scale=K)
        _, opacity, depth, rend, _ = _Composite.apply(sig, rgb, torch.from_numpy(deltas), torch.from_numpy(ts),
                                                      torch.from_numpy(rays_a), 1e-4)
        out_rgb = rend + 1.0 * (1 - opacity)[:, None]
        l_rgb = ((out_rgb - torch.from_numpy(batch["rgb"])) ** 2).mean()
        oo = opacity + 1e-10
        l_op = self.opacity_w * (-oo * torch.log(oo)).mean()
        loss = l_rgb + l_op
        rec = {} if record is None else record
        rec.update(rgb=float(l_rgb.detach()), opacity=float(l_op.detach()), samples=int(counter[0]))
        x1, x2, x3 = losses_ref.patch_triangle_index(R)
        dt = torch.from_numpy(d)
        n = losses_ref.normals_from_depth(dt, dt, depth, x1, x2, x3)  # rays_o := rays_d (quirk q1)
        valid = losses_ref.valid_normals_mask(n.detach())
        nv = n[valid]
        rec["valid"] = valid.numpy().copy()
        rec["normals"] = n.detach().numpy().copy()
        if nv.shape[0] >= 20:
            C, a = losses_ref.spherical_kmeans(nv.detach().numpy(), K=20, niter=20, seed=1234)
            lab, _ = losses_ref.cluster_select(C, a, 0.99)
            rec["labels_own"] = np.asarray(lab).copy()
            if force_labels is not None:
                lab = np.asarray(force_labels).astype(np.asarray(lab).dtype)
                assert lab.shape == rec["labels_own"].shape, (lab.shape, rec["labels_own"].shape)
            if force_signs is not None:
                own = losses_ref.kink_signs(nv.detach().numpy(), lab)
                rec["sign_mismatch"] = {"ort": int((own[0] != force_signs[0]).sum()),
                                        "l1": int(sum((a != b).sum() for a, b in zip(own[1], force_signs[1]))),
                                        "l1_total": int(sum(a.size for a in own[1]))}
            ort, cdot, cl1 = losses_ref.cluster_losses(nv, torch.from_numpy(lab), signs=force_signs)
            w = losses_ref.w_sched(self.w_cluster, global_step)
            terms = [losses_ref.validity(t) for t in (ort, cdot, cl1)]
            rec.update(labels=np.asarray(lab).copy(), w_cluster=float(w),
                       norm_D_C_ort_dot=float(w * terms[0].detach()), norm_D_C_centr_dot=float(w * terms[1].detach()),
                       norm_D_C_centr_L1=float(w * terms[2].detach()), raw_cluster=[float(t.detach()) for t in terms])
            loss = loss + w * (terms[0] + terms[1] + terms[2])
        rec["total"] = float(loss.detach())
        loss.backward()
        if record is not None:
            rec["grads"] = [p.grad.detach().clone() for p in self.params]
        if self.emulate_bwd and self.emulate == "fp16":  # GradScaler.step / update (torch defaults)
            if not all(bool(torch.isfinite(p.grad).all()) for p in self.params):
                self.opt.zero_grad()
                self.amp_S *= 0.5
                self.amp_tracker = 0
                self.amp_skips += 1
                rec["skipped"] = True
                return float(loss.detach()), int(counter[0])
            self.amp_tracker += 1
            if self.amp_tracker >= 2000:
                self.amp_S *= 2.0
                self.amp_tracker = 0
        rec["skipped"] = False
        torch.nn.utils.clip_grad_norm_(self.params, 0.05)
        self.opt.step()
        return float(loss.detach()), int(counter[0])
