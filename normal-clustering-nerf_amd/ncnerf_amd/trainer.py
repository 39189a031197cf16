"""One training step of the reference NeRFSystem (train_nerf.py:165-358) on the HIP hot path:
render (intersect -> march -> field -> composite) -> NeRFMTLoss (rgb + opacity + normal
clustering) -> backward -> [RCCL gradient all-reduce] -> clip + Adam, plus the occupancy-grid
refresh every 16 steps (train_nerf.py:314-320) when `update_grid` is on, and the per-epoch cosine
learning rate (CosineAnnealingLR(T_max=num_epochs), train_nerf.py:286-288; an epoch is the
training set's 1000 items, base.py:78-81, split over the ranks by DDP's DistributedSampler).

Hyper-parameters default to the Hypersim config (experiments/hypersim/hyperparameters.py);
preset="scannet_manhattan" selects config #5's (experiments/scannet_man/hyperparameters.py)."""
import math
import warnings

import torch

from . import _lib, distributed
from .losses import NeRFMTLoss, check_cluster_status
from .optim import FlatAdam
from .rendering import march_train_fused, render

HYPERSIM_HPARAMS = dict(
    scale=0.5, grid_size=128, rend_max_samples=1024, rend_near_dist=0.01, density_tresh_decay=1.0,
    loss_opacity_w=1e-3, loss_distortion_w=0, loss_depth_w=0, loss_norm_depth_dot_w=0, loss_norm_depth_L1_w=0,
    loss_reg_depth_w=0, loss_sem_w=0, loss_manhattan_nerf_w=0,
    loss_norm_D_C_ort_dot_w=2e-3, loss_norm_D_C_centr_dot_w=2e-3, loss_norm_D_C_centr_L1_w=2e-3,
    loss_norm_D_C_can_dot_w=0, loss_norm_D_C_can_L1_w=0, loss_norm_can_tres=0.01, loss_norm_can_start=500,
    loss_norm_can_end=-1, loss_norm_can_grow=2500, lr=1e-2, num_epochs=30, batch_size=8192,
    ray_sampling_strategy="all_images_triang_patch", grad_clip=0.05, pred_norm_depth=True)

# config #5 (experiments/scannet_man/hyperparameters.py): the Hypersim settings with the three
# normal-clustering weights at 1e-2 (:45-47); scale, grid, samples, lr, batch and clip are equal (:21-24)
SCANNET_HPARAMS = dict(HYPERSIM_HPARAMS, loss_norm_D_C_ort_dot_w=1e-2, loss_norm_D_C_centr_dot_w=1e-2,
                       loss_norm_D_C_centr_L1_w=1e-2)

PRESETS = {"hypersim": HYPERSIM_HPARAMS, "scannet_manhattan": SCANNET_HPARAMS}


def hparams_for(preset):
    """The hyper-parameter dict of a dataset preset (train_nerf.py --dataset_name)."""
    if preset not in PRESETS:
        raise ValueError(f"unknown preset {preset!r}; one of {sorted(PRESETS)}")
    return dict(PRESETS[preset])


class Trainer:
    warmup_steps = 256
    update_interval = 16

    epoch_items = 1000  # base.py:78-81 (training "epoch" = 1000 batches)

    def __init__(self, model, hparams=None, update_grid=False, use_graph=False, scatter_split=None,
                 defer_optimizer=False, preset="hypersim", split_backward=True):
        """hparams: overrides of the preset's hyper-parameters (PRESETS: "hypersim" = configs #1-#4,
        "scannet_manhattan" = config #5).  split_backward (graph step; taken when the loss is the
        reference configuration, split_step.split_eligible): the step runs as split_step.SplitStep —
        the photometric backward overlaps the normal clustering, every per-sample value as the
        autograd backward computes it — instead of render -> loss -> autograd backward."""
        self.h = dict(hparams_for(preset), **(hparams or {}))
        self.model = model
        self.loss = NeRFMTLoss(self.h)
        # the Adam pass zeroes the gradient it consumed: no zero_grad fill in the step
        self.opt = FlatAdam(model, lr=self.h["lr"], max_norm=self.h["grad_clip"], num_epochs=self.h["num_epochs"],
                            zero_grad_on_step=True)
        self.world = distributed.world_size()
        self.steps_per_epoch = math.ceil(self.epoch_items / self.world)  # DistributedSampler split
        # data-parallel step: all-reduce the gradient in two buckets, the table levels
        # [scatter_split, 16) + MLP weights while the levels [0, scatter_split) are scattered
        if self.world > 1:
            model.scatter_split = distributed.DEFAULT_SCATTER_SPLIT if scatter_split is None else scatter_split
        self.update_grid = update_grid
        self.render_kwargs = dict(near_distance=self.h["rend_near_dist"], max_samples=self.h["rend_max_samples"],
                                  test_time=False, random_bg=False, anneal_strategy="none", anneal_steps=0)
        self.use_graph = use_graph
        self.split_backward = bool(split_backward) and use_graph
        self._split = None  # the SplitStep of the captured graph (split_backward and split_eligible)
        self.graph = None
        # defer_optimizer (graph step): the optimizer step of step k runs inside graph k+1 on a side
        # stream, concurrently with step k+1's marcher (which reads no parameter), and joins before
        # the field forward; a refresh of the occupancy grid, or flush_optimizer(), applies a pending
        # step first.  Parameters read between steps are one step behind until flush_optimizer() is
        # called.  N > 1: the gradient all-reduce of step k (eager, after graph k) is ordered before
        # graph k+1 on the same stream, so the deferred step reads the reduced gradient; DDP's
        # 1/world goes in as the step's grad_scale on the fp32 wire (the fp16 wire divides before
        # the sum, as DDP does: grad_scale 1).
        self.defer = bool(defer_optimizer) and use_graph
        self._grad_scale = distributed.grad_scale_after_reduce(model, self.world)
        self._pending = False
        self._rng_seed = int(torch.randint(0, 2 ** 62, (1,)).item())  # marcher jitter stream (CPU generator)
        # optional seed of each grid refresh (global_step -> int); default: drawn from torch's CPU generator
        self.grid_seed = None

    def flush_optimizer(self):
        """Apply the deferred optimizer step (defer_optimizer) now, if one is pending."""
        if self._pending:
            self.opt.step(grad_scale=self._grad_scale)
            self._pending = False

    def _maybe_update_grid(self, global_step):
        m = self.model
        if self.update_grid and global_step % self.update_interval == 0:
            thr = 0.01 * self.h["rend_max_samples"] / 3 ** 0.5 * self.h["density_tresh_decay"]
            seed = self.grid_seed(global_step) if self.grid_seed is not None else None
            # the pending optimizer step first (the density pass reads the parameters), issued beside
            # the refresh's cell sampling, which reads only the density grid
            m.update_density_grid(thr, warmup=global_step < self.warmup_steps, seed=seed, beside=self.flush_optimizer)
            distributed.broadcast_occupancy(m)

    # -- graph-captured step ---------------------------------------------------------------------
    # The whole step (zero_grad, render with static shapes, losses, backward, [optimizer]) is one
    # HIP graph: the marcher's sample count stays on the device (static_shapes), the loss-weight
    # schedule and Adam's step/lr are device scalars, so nothing in the step reads the host.  A
    # replay costs one launch instead of ~150 Python-driven ones.  Inputs are copied into the
    # graph's static batch buffers; the occupancy-grid refresh and the RCCL all-reduce (N > 1)
    # run eagerly around it.
    def _body(self, batch, step_dev, with_opt):
        m = self.model
        kw = dict(self.render_kwargs, global_step=0, static_shapes=True)
        kw["count_in_loss"] = True  # vr_samples summed by the loss node's first launch (no launch of its own)
        if "march_noise" in batch:
            kw["march_noise"] = batch["march_noise"]
        else:  # jitter drawn on the device from the step counter: no torch RNG node in the graph
            kw["march_rng"] = (self._rng_seed, step_dev)
        if self.defer:
            # the previous step's optimizer (gated: skipped when nothing is pending) beside this step's
            # marcher; joined before the field forward reads the parameters
            cur = torch.cuda.current_stream()
            side = self._side_stream()
            side.wait_stream(cur)

            def optimizer():
                self.opt.step(gated=True, grad_scale=self._grad_scale)
                if not self.opt.pack_fused:
                    m._pack_weights()  # the MLP's fp16 fragments of the updated weights, also beside the marcher
                m._packed_fresh = True  # (pack_fused: the Adam pass has written them)

            def marcher(out=None):
                return march_train_fused(m, batch["rays_o"], batch["rays_d"], kw["near_distance"], kw["max_samples"],
                                         kw.get("march_noise"), kw.get("march_rng"), out=out)

            # (the optimizer on the main stream and the marcher on the side one measured the same:
            # DESIGN.md §7, rounds 4 and 6)
            with torch.cuda.stream(side):
                optimizer()
            kw["premarched"] = marcher()
            cur.wait_stream(side)
        if self._split is not None:
            results, loss_d = self._split.run(batch, step_dev, premarched=kw.get("premarched"))
        else:
            results = render(m, batch["rays_o"], batch["rays_d"], **kw)
            loss_d = self.loss(results, batch, global_step=step_dev)
            # (a constant upstream gradient: no ones_like fill node per step)
            torch.autograd.backward(loss_d["total"], grad_tensors=self._unit(loss_d["total"].device))
        if with_opt and not self.defer:
            self.opt.step()
        return results, loss_d

    def _unit(self, dev):
        """A device fp32 1.0: the upstream gradient of the total loss."""
        if getattr(self, "_one", None) is None or self._one.device != dev:
            self._one = torch.ones((), dtype=torch.float32, device=dev)
        return self._one

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.model.flat_params().device)
        return self._side

    def _capture(self, batch):
        import torch
        dev = batch["rays_o"].device
        if self.render_kwargs.get("anneal_steps", 0) > 0:
            raise NotImplementedError("ray-range annealing is step-dependent host control flow")
        self._static = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}
        from .split_step import SplitStep, split_eligible
        self._split = None
        if self.split_backward and split_eligible(self, self._static):
            try:
                self._split = SplitStep(self)
            except _lib.NcnError as e:  # the clustering cannot stay resident beside the rgb pass
                warnings.warn(f"split backward unavailable on this device, using the autograd step: {e}")
        self._step_dev = torch.zeros((), dtype=torch.int64, device=dev)
        # the optimizer is in the graph unless the gradient is reduced (or its scatter finished) outside
        self._with_opt = not distributed.is_distributed() and self.model.scatter_split is None
        state = self.opt.state_tensors()
        saved = [t.clone() for t in state]  # warm-up steps must not advance training
        saved_count = self.opt.step_count
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                self._body(self._static, self._step_dev, self._with_opt)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.model._deferred = []  # (the warm-ups' deferred scatters are dropped with their gradients)
        # the warm-ups' optimizer steps also refreshed the packed MLP fragments (FlatAdam.pack_fused):
        # the captured forward packs for itself unless the deferred optimizer in the body does it
        self.model._packed_fresh = False
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._out = self._body(self._static, self._step_dev, self._with_opt)
        # the captured backward's deferred scatter names the graph's static buffers: every replay's
        # reduce_gradients(graph=True) runs that same entry; eager backwards keep their own list
        self.model._deferred_graph = self.model._deferred
        self.model._deferred = []
        for t, v in zip(state, saved):
            t.copy_(v)
        if hasattr(self.model, "prepare_weights"):
            self.model.prepare_weights()  # (the fragments of the restored parameters)
        self.opt.step_count = saved_count
        self.model.flat_grad().zero_()  # (the warm-ups without the optimizer left gradients behind)

    def _graph_step(self, batch, global_step):
        if self.graph is None:
            self._capture(batch)
        dst, src = [], []
        for k, v in batch.items():
            if k in self._static and hasattr(v, "copy_") and v is not self._static[k]:
                dst.append(self._static[k])
                src.append(v)
        fast = len(dst) <= 8 and all(
            s.is_cuda and s.is_contiguous() and d.is_contiguous() and s.dtype == d.dtype and s.shape == d.shape
            for s, d in zip(src, dst))
        gate = 1 if self._pending else 0  # (defer: the previous step's gradient awaits its optimizer step)
        if fast:  # the batch copies, the device step counter and the gate in one launch (ncn_step_inputs)
            _lib.step_inputs(src, dst, self._step_dev, global_step, self.opt.gate if self.defer else None, gate)
        else:
            if dst:
                torch._foreach_copy_(dst, src, non_blocking=True)  # one launch for the whole batch
            self._step_dev.fill_(global_step)
            if self.defer:
                self.opt.gate.fill_(gate)
        self.graph.replay()
        scale = distributed.reduce_gradients(self.model, graph=True) if not self._with_opt else 1.0
        if self.defer:  # (the next graph's side stream applies it, after the reduction above)
            self.opt.step_count += gate
            self._pending = True
        elif not self._with_opt:
            self.opt.step(grad_scale=scale)
        else:
            self.opt.step_count += 1
        return self._out

    status_interval = 100  # steps between reads of the clustering kernel's error word

    def step(self, batch, global_step):
        m = self.model
        if global_step % self.status_interval == 0:
            check_cluster_status(m.flat_params().device)  # (raises if an earlier launch timed out)
        self._maybe_update_grid(global_step)
        epoch = global_step // self.steps_per_epoch
        if epoch != self.opt.epoch:
            self.flush_optimizer()  # (a pending step belongs to the previous epoch's learning rate)
        self.opt.set_epoch(epoch)
        if self.use_graph:
            return self._graph_step(batch, global_step)
        kw = dict(self.render_kwargs, global_step=global_step)
        if "march_noise" in batch:
            kw["march_noise"] = batch["march_noise"]
        results = render(m, batch["rays_o"], batch["rays_d"], **kw)
        loss_d = self.loss(results, batch, global_step=global_step)
        loss_d["total"].backward()
        self.opt.step(grad_scale=distributed.reduce_gradients(m))
        return results, loss_d
