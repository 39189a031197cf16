"""Data parallelism of the reference (PL DDPPlugin, train_nerf.py:944-952) on torch.distributed.

One process per GPU; backend "nccl" is RCCL on ROCm (xGMI).  Every rank draws its own ray batch
(weak scaling, 8192 rays per rank as in the reference, base.py:94-171); the only data-path exchange
is the all-reduce (SUM) of the flat gradient buffer (hash table + MLPs, 11.5 M values) per step —
as fp16 values fp16(S * g) / world (22.9 MB: the reference's own DDP wire — tcnn's fp16 gradients at
the GradScaler's scale, divided by the world size BEFORE the sum as torch DDP's default hook does)
when the model runs the fp16 AMP, else fp32 (45.8 MB) with the 1/world of DDP's average folded into
the optimizer (exact for a power-of-two world).  `reduce_gradients` issues it as two
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


# Gradient wire format of the all-reduce.  "auto": fp16 values fp16(S * g) / world when the model runs
# the fp16 AMP (it has the GradScaler state amp_state) — what the reference's DDP moves: tcnn keeps
# fp16 parameters, so its gradient buckets are fp16 at PL's loss scale S, and DDP's default hook
# divides each bucket by the world size before the all-reduce SUM (torch
# ddp_comm_hooks/default_hooks.py, _allreduce_fut: "Apply the division first to avoid overflow,
# especially for FP16") — half the bytes of fp32 on xGMI; "fp32": the unscaled fp32 gradient (the
# bf16 / fp32 models always use it: no scale), summed, the 1/world applied by the optimizer.
DP_WIRE = os.environ.get("NCN_DP_WIRE", "auto")


def wire_of(model):
    """"fp16" or "fp32": the format reduce_gradients moves the model's gradient in."""
    if DP_WIRE == "fp32" or getattr(model, "amp_state", None) is None:
        return "fp32"
    return "fp16"


def grad_scale_after_reduce(model, world=None):
    """The factor the optimizer applies to the reduced gradient to form DDP's average: 1 on the fp16
    wire (divided by the world before the sum), 1/world on the fp32 wire (a plain SUM)."""
    world = world_size() if world is None else world
    return 1.0 if world <= 1 or wire_of(model) == "fp16" else 1.0 / world


class _Bucket:
    """One all-reduce bucket: a view of the flat gradient, moved as is (fp32) or packed to the fp16
    wire (ncn_grad_pack_f16: x S, then / world as DDP divides) and unpacked (/ S) into the same view
    after the collective."""

    def __init__(self, model, view):
        self.view = view
        self.scale = None
        self.wire = None
        if wire_of(model) == "fp16":
            fg = model.flat_grad()
            if getattr(model, "_wire_buf", None) is None or model._wire_buf.numel() != fg.numel() \
                    or model._wire_buf.device != fg.device:
                model._wire_buf = torch.empty(fg.numel(), dtype=torch.float16, device=fg.device)
            off = (view.data_ptr() - fg.data_ptr()) // 4
            self.wire = model._wire_buf[off:off + view.numel()]
            self.scale = model.amp_state

    def start(self):
        from . import _lib
        t = self.view
        if self.wire is not None:
            _lib.call("ncn_grad_pack_f16", _lib.ptr(self.view), _lib.I64(self.view.numel()), _lib.ptr(self.scale),
                      _lib.I32(dist.get_world_size()), _lib.ptr(self.wire), _lib.stream())
            t = self.wire
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)

    def finish(self, work):
        from . import _lib
        work.wait()
        if self.wire is not None:
            _lib.call("ncn_grad_unpack_f16", _lib.ptr(self.wire), _lib.I64(self.view.numel()), _lib.ptr(self.scale),
                      _lib.ptr(self.view), _lib.stream())


def reduce_gradients(model, graph=False):
    """DDP's gradient all-reduce of one step, in the format wire_of(model) names; returns the scale
    that turns the result into DDP's average (grad_scale_after_reduce: 1 on the pre-divided fp16
    wire, 1/world on the fp32 SUM) for the optimizer.  With model.scatter_split set, the backward left
    the coarse table levels unscattered: bucket A (fine levels + MLP weights) is reduced
    asynchronously while the deferred scatter runs on the current stream, then bucket B; both are
    waited on (current stream) before returning.  Single process: runs the deferred scatter,
    returns 1.  graph: the gradient is a replayed captured step's (its deferred scatter is the
    captured one, NGPMT.run_deferred_scatter(graph=True))."""
    split = getattr(model, "scatter_split", None)
    if not is_distributed():
        if split is not None and (model._deferred_graph if graph else model._deferred):
            model.run_deferred_scatter(graph=graph)
        return 1.0
    if split is None:
        bk = _Bucket(model, model.flat_grad())
        bk.finish(bk.start())
    else:
        a, b = model.grad_buckets(split)
        ba, bb = _Bucket(model, a), _Bucket(model, b)
        wa = ba.start()
        model.run_deferred_scatter(max_blocks=DP_SCATTER_BLOCKS, graph=graph)
        wb = bb.start()
        ba.finish(wa)
        bb.finish(wb)
    return grad_scale_after_reduce(model)


def broadcast_occupancy(model, src=0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if hasattr(model, "density_grid"):
            dist.broadcast(model.density_grid, src)
        dist.broadcast(model.density_bitfield, src)


def shard_patches(n_patches_global, rank, world):
    """Patch-granular shard [lo, hi) of a global batch (never splits an 8x8 patch)."""
    per = n_patches_global // world
    return rank * per, (rank + 1) * per
