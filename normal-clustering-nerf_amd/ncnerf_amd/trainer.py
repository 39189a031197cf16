"""One training step of the reference NeRFSystem (train_nerf.py:165-358) on the HIP hot path:
render (intersect -> march -> field -> composite) -> NeRFMTLoss (rgb + opacity + normal
clustering) -> backward -> [RCCL gradient all-reduce] -> clip + Adam, plus the occupancy-grid
refresh every 16 steps (train_nerf.py:314-320) when `update_grid` is on.

Hyper-parameters default to the Hypersim config (experiments/hypersim/hyperparameters.py)."""
import torch

from . import distributed
from .losses import NeRFMTLoss
from .optim import FlatAdam
from .rendering import render

HYPERSIM_HPARAMS = dict(
    scale=0.5, grid_size=128, rend_max_samples=1024, rend_near_dist=0.01, density_tresh_decay=1.0,
    loss_opacity_w=1e-3, loss_distortion_w=0, loss_depth_w=0, loss_norm_depth_dot_w=0, loss_norm_depth_L1_w=0,
    loss_reg_depth_w=0, loss_sem_w=0, loss_manhattan_nerf_w=0,
    loss_norm_D_C_ort_dot_w=2e-3, loss_norm_D_C_centr_dot_w=2e-3, loss_norm_D_C_centr_L1_w=2e-3,
    loss_norm_D_C_can_dot_w=0, loss_norm_D_C_can_L1_w=0, loss_norm_can_tres=0.01, loss_norm_can_start=500,
    loss_norm_can_end=-1, loss_norm_can_grow=2500, lr=1e-2, num_epochs=30, batch_size=8192,
    ray_sampling_strategy="all_images_triang_patch", grad_clip=0.05, pred_norm_depth=True)


class Trainer:
    warmup_steps = 256
    update_interval = 16

    def __init__(self, model, hparams=None, update_grid=False):
        self.h = dict(HYPERSIM_HPARAMS, **(hparams or {}))
        self.model = model
        self.loss = NeRFMTLoss(self.h)
        self.opt = FlatAdam(model, lr=self.h["lr"], max_norm=self.h["grad_clip"], num_epochs=self.h["num_epochs"])
        self.update_grid = update_grid
        self.render_kwargs = dict(near_distance=self.h["rend_near_dist"], max_samples=self.h["rend_max_samples"],
                                  test_time=False, random_bg=False, anneal_strategy="none", anneal_steps=0)

    def step(self, batch, global_step):
        m = self.model
        if self.update_grid and global_step % self.update_interval == 0:
            thr = 0.01 * self.h["rend_max_samples"] / 3 ** 0.5 * self.h["density_tresh_decay"]
            m.update_density_grid(thr, warmup=global_step < self.warmup_steps)
            distributed.broadcast_occupancy(m)
        self.opt.zero_grad()
        kw = dict(self.render_kwargs, global_step=global_step)
        if "march_noise" in batch:
            kw["march_noise"] = batch["march_noise"]
        results = render(m, batch["rays_o"], batch["rays_d"], **kw)
        loss_d = self.loss(results, batch, global_step=global_step)
        loss_d["total"].backward()
        distributed.allreduce_grads(m.flat_grad())
        self.opt.step()
        return results, loss_d
