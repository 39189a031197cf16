"""Optimizer step of the reference training loop on the flat parameter buffer.

Reference: apex FusedAdam (AdamW mode, eps 1e-15) with two groups — hash-grid features (weight
decay 0) and MLP weights (weight decay 1e-6) — (train_nerf.py:262-285), gradient clipping by global
L2 norm 0.05 (train_nerf.py:955), CosineAnnealingLR(T_max=num_epochs, eta_min=0) stepped once per
epoch (:286-288; `set_epoch`).  Two launches per step (ncn_adam_step: sum of squares whose last
workgroup forms the clip factor and step scalars, then Adam of both groups); the clip factor never
leaves the device.  With `zero_grad_on_step` the Adam pass also zeroes the gradient it consumed, so
the next step needs no zero_grad fill (PL's zero_grad before every backward, folded in).
"""
import math

import torch

from . import _lib
from ._lib import F32, I32, I64, call, ptr, stream


class FlatAdam:
    def __init__(self, model, lr=1e-2, betas=(0.9, 0.999), eps=1e-15, weight_decay=(0.0, 1e-6), max_norm=0.05,
                 num_epochs=None, zero_grad_on_step=False):
        self.model = model
        self.base_lr = self.lr = lr
        self.betas, self.eps, self.wd, self.max_norm = betas, eps, weight_decay, max_norm
        flat = model.flat_params()
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.part = torch.empty(1024, dtype=torch.float32, device=flat.device)
        self.work = torch.zeros(int(_lib.lib().ncn_adam_step_work_floats()), dtype=torch.float32, device=flat.device)
        self.step_count = 0
        # device-side step counter and learning rate: the step kernels read them, so the optimizer
        # step can sit inside a captured HIP graph (the counter is bumped by the sum-of-squares kernel)
        self.step_dev = torch.zeros((), dtype=torch.int32, device=flat.device)
        self.lr_dev = torch.full((), float(lr), dtype=torch.float32, device=flat.device)
        self.num_epochs = num_epochs
        self.n_table = model._n_table
        self.zero_grad_on_step = zero_grad_on_step
        self.epoch = 0
        # gate of a deferred step inside a captured graph (Trainer(defer_optimizer=True)): 0 = no
        # gradient pending, the step is skipped
        self.gate = torch.ones((), dtype=torch.int32, device=flat.device)
        # refresh the model's packed MLP fragments inside the Adam pass (models with pack_target)
        self.pack_fused = hasattr(model, "pack_target")
        if self.pack_fused:
            model.pack_target()  # (the map is built here, eagerly: a later first call may be inside a capture)

    def zero_grad(self):
        self.model.flat_grad().zero_()

    def set_epoch(self, epoch):
        """CosineAnnealingLR(T_max=num_epochs, eta_min=0) stepped per epoch (train_nerf.py:286-288):
        lr(e) = base_lr * (1 + cos(pi * e / T_max)) / 2.  Writes the device lr the step kernels read
        (also inside a captured graph); a no-op when the epoch is unchanged."""
        if self.num_epochs and epoch != self.epoch:
            self.epoch = epoch
            self.lr = 0.5 * self.base_lr * (1 + math.cos(math.pi * epoch / self.num_epochs))
            self.lr_dev.fill_(self.lr)

    def step(self, grad_scale=1.0, gated=False):
        """grad_scale: the gradient used is flat_grad * grad_scale (1/world after an all-reduce SUM).
        gated: the step runs only if the device gate is 1 (a deferred step in a captured graph)."""
        self.step_count += 1
        p = self.model.flat_params()
        g = self.model.flat_grad()
        b1, b2 = self.betas
        args = [ptr(p), ptr(g), ptr(self.m), ptr(self.v), I64(p.numel()), I64(self.n_table), F32(grad_scale),
                F32(self.max_norm), F32(self.lr), _lib.F64(b1), _lib.F64(b2), F32(self.eps), F32(self.wd[0]),
                F32(self.wd[1]), ptr(self.lr_dev), ptr(self.step_dev), ptr(self.work),
                I32(1 if self.zero_grad_on_step else 0), ptr(getattr(self.model, "amp_state", None)),
                ptr(self.gate if gated else None)]
        if self.pack_fused:
            # the field's packed MLP fragments refreshed by the Adam pass itself (ncn_adam_step_packed):
            # afterwards they match the parameters whether the step applied or was skipped
            inv, off, packed, prec = self.model.pack_target()
            call("ncn_adam_step_packed", *args, ptr(inv), I64(off), ptr(packed), I32(prec), stream())
            self.model._packed_fresh = True
        else:
            call("ncn_adam_step", *args, stream())

    def state_tensors(self):
        """Every tensor the step mutates (parameters, moments, device counters)."""
        st = [self.model.flat_params(), self.m, self.v, self.step_dev, self.lr_dev]
        amp = getattr(self.model, "amp_state", None)
        return st + ([amp] if amp is not None else [])
