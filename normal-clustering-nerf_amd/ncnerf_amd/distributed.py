"""Data parallelism of the reference (PL DDPPlugin, train_nerf.py:944-952) on torch.distributed.

One process per GPU; backend "nccl" is RCCL on ROCm (xGMI).  Every rank draws its own ray batch
(weak scaling, 8192 rays per rank as in the reference, base.py:94-171); the only data-path exchange
is the all-reduce (SUM) of the flat gradient buffer (hash table + MLPs, ~45.8 MB fp32) per step,
the 1/world of DDP's average folded into the optimizer.  `reduce_gradients` issues it as two
buckets so that most of it overlaps the table scatter: the backward scatters the fine table levels
[split, 16) first; their bucket (plus the MLP weights, contiguous behind them) is all-reduced
asynchronously while the coarse levels [0, split) are scattered, then the coarse bucket follows.
The occupancy grid is kept identical on every rank by broadcasting rank 0's density grid +
bitfield after each refresh (the reference relies on DDP buffer broadcast).
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from RANK/WORLD_SIZE/MASTER_* (torchrun) if present."""
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) <= 1:
        return 0, 1
    if not dist.is_initialized():
        if backend is None:  # NCN_DIST_BACKEND=gloo: rehearse the N>1 path with several ranks on one GPU
            backend = os.environ.get("NCN_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


# table levels [0, 10) (~21.8 MB, run-aggregated in the scatter) are scattered while levels
# [10, 16) + the MLP weights (~24 MB) are all-reduced
DEFAULT_SCATTER_SPLIT = 10
# workgroups of the deferred (overlapped) scatter: one per CU would leave no CU to RCCL's kernels
DP_SCATTER_BLOCKS = int(os.environ.get("NCN_DP_SCATTER_BLOCKS", "224"))


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_distributed():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_grads(flat_grad, average=True):
    """Sum the flat gradient over ranks (single bucket: the buffer is contiguous).  Returns the scale
    that turns the sum into DDP's average (1/world): with average=False the caller folds it into the
    optimizer (FlatAdam.step(grad_scale)) instead of a separate division pass over the buffer."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)
        if average:
            flat_grad.div_(dist.get_world_size())
            return 1.0
        return 1.0 / dist.get_world_size()
    return 1.0


def reduce_gradients(model):
    """DDP's gradient all-reduce of one step (sum over ranks; returns the 1/world scale for the
    optimizer).  With model.scatter_split set, the backward left the coarse table levels unscattered:
    bucket A (fine levels + MLP weights) is reduced asynchronously while the deferred scatter runs on
    the current stream, then bucket B; both are waited on (current stream) before returning.
    Single process: runs the deferred scatter, returns 1."""
    split = getattr(model, "scatter_split", None)
    if not is_distributed():
        if split is not None and model._deferred:
            model.run_deferred_scatter()
        return 1.0
    if split is None:
        dist.all_reduce(model.flat_grad(), op=dist.ReduceOp.SUM)
    else:
        a, b = model.grad_buckets(split)
        wa = dist.all_reduce(a, op=dist.ReduceOp.SUM, async_op=True)
        model.run_deferred_scatter(max_blocks=DP_SCATTER_BLOCKS)
        wb = dist.all_reduce(b, op=dist.ReduceOp.SUM, async_op=True)
        wa.wait()
        wb.wait()
    return 1.0 / dist.get_world_size()


def broadcast_occupancy(model, src=0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if hasattr(model, "density_grid"):
            dist.broadcast(model.density_grid, src)
        dist.broadcast(model.density_bitfield, src)


def shard_patches(n_patches_global, rank, world):
    """Patch-granular shard [lo, hi) of a global batch (never splits an 8x8 patch)."""
    per = n_patches_global // world
    return rank * per, (rank + 1) * per
