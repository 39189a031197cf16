"""Worker of tests/test_gpu_ddp.py (not a test module).

`run` — under torchrun every rank trains the model through Trainer(use_graph=True) on ITS OWN
batches (seeded by rank and step): the N>1 path — graph-captured step without the optimizer, the
two-bucket gradient all-reduce (SUM) overlapped with the deferred coarse-level table scatter, Adam
with grad_scale = 1/world (argv[3] == "defer": inside the next step's graph, beside its marcher) —
and rank 0 saves the parameters.

`run_reference` — one process, the eager step: for every step the gradients of all ranks' batches
are accumulated into the flat gradient (one backward per batch, no optimizer in between), then one
Adam step with grad_scale = 1/world, i.e. DDP's average computed without any collective.  With the
fp16 gradient wire (distributed.wire_of: the fp16 AMP model) each rank's gradient is rounded as
DDP's bucket holds it and divides it — fp16(fp16(S g) / world) — the ranks' values are summed in
rank order with fp16 rounding (the collective's own order may differ: `wire_sum` below), / S, and
Adam takes grad_scale 1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]

import torch  # noqa: E402

N_RAYS = 1024


def _setup(device):
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.synthetic import SyntheticScene
    scene = SyntheticScene()
    torch.manual_seed(0)
    model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(device))
    model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(device))
    return scene, model


# GLOBAL: config #4's layout — ONE global batch per step (65 536 rays), each rank taking its
# shard_patches slice (8192 rays of whole 8x8 patches); otherwise every rank draws its own batch
GLOBAL = os.environ.get("DDP_GLOBAL_RAYS")


def _batch(scene, rank, k, device, world=1):
    if GLOBAL:
        from ncnerf_amd import distributed
        n = int(GLOBAL)
        full = scene.batch(n, seed=50_000 + k)
        lo, hi = distributed.shard_patches(n // 64, rank, world)
        g = torch.Generator().manual_seed(60_000 + k)
        noise = torch.rand(n, generator=g)[lo * 64:hi * 64]
        batch = {}
        for kk, v in full.items():
            if hasattr(v, "shape") and not kk.endswith("_offsets_local") and v.shape[:1] == (n,):
                batch[kk] = torch.from_numpy(v[lo * 64:hi * 64].copy()).to(device)
            else:
                batch[kk] = v
        batch["march_noise"] = noise.to(device)
        return batch
    batch = scene.torch_batch(N_RAYS, seed=1000 * rank + 10 + k, device=device)
    g = torch.Generator().manual_seed(1000 * rank + k)
    batch["march_noise"] = torch.rand(N_RAYS, generator=g).to(device)
    return batch


def run(steps, device, out=None, rank=0, defer=False, world=1, split=False):
    from ncnerf_amd.trainer import Trainer
    scene, model = _setup(device)
    tr = Trainer(model, use_graph=True, defer_optimizer=defer, split_backward=split)
    for k in range(steps):
        tr.step(_batch(scene, rank, k, device, world), global_step=3000 + k)
    tr.flush_optimizer()  # (defer: the last step's optimizer is still pending)
    torch.cuda.synchronize()
    flat = model.flat_params().detach().cpu().clone()
    if out:
        torch.save(flat, out)
    return flat


def wire_value(g, S, world):
    """One rank's fp16 wire value: DDP's bucket fp16(S g), divided in place by the world (fp16)."""
    return ((g * S).half().float() / world).half()


def wire_sum(per_rank, S, world):
    """The fp16 wire's all-reduce SUM in rank order with fp16 rounding of every partial sum (float)."""
    tot = wire_value(per_rank[0], S, world)
    for g in per_rank[1:]:
        tot = (tot.float() + wire_value(g, S, world).float()).half()
    return tot.float()


AMBIGUOUS = [None]  # run_reference, fp16 wire: union over the steps of the order-ambiguous entries


def run_reference(steps, device, world):
    AMBIGUOUS[0] = None
    from ncnerf_amd.rendering import render
    from ncnerf_amd.trainer import Trainer
    scene, model = _setup(device)
    tr = Trainer(model, use_graph=False)
    from ncnerf_amd import distributed
    fp16_wire = distributed.wire_of(model) == "fp16"
    for k in range(steps):
        tr.opt.set_epoch((3000 + k) // -(-tr.epoch_items // world))  # the ranks' epoch (DistributedSampler)
        per_rank = []
        for r in range(world):
            batch = _batch(scene, r, k, device, world)
            # the graph step's kernels (fused marcher, sample-order compositor) on the eager path
            kw = dict(tr.render_kwargs, global_step=3000 + k, march_noise=batch["march_noise"], static_shapes=True)
            results = render(model, batch["rays_o"], batch["rays_d"], **kw)
            tr.loss(results, batch, global_step=3000 + k)["total"].backward()
            if fp16_wire:  # each rank's gradient on its own (the wire rounds them separately)
                per_rank.append(model.flat_grad().clone())
                model.flat_grad().zero_()
        if fp16_wire:
            S = float(model.amp_state[0])
            model.flat_grad().copy_(wire_sum(per_rank, S, world) / S)
            # entries whose reduced sum may round to another side of zero (or to zero) in another
            # summation order: |exact sum| within the order-independent bound of an fp16 sum
            h = torch.stack([wire_value(g, S, world).double() for g in per_rank])
            bound = (world - 1) * (2.0 ** -11 * h.abs().sum(0) + 2.0 ** -25)
            amb = ((h.sum(0).abs() <= bound) & (h != 0).any(0)).cpu()  # (all-zero terms: exactly 0 in any order)
            AMBIGUOUS[0] = amb if AMBIGUOUS[0] is None else (AMBIGUOUS[0] | amb)
        tr.opt.step(grad_scale=distributed.grad_scale_after_reduce(model, world))
    torch.cuda.synchronize()
    return model.flat_params().detach().cpu().clone()


if __name__ == "__main__":
    from ncnerf_amd import distributed
    rank, world = distributed.init_from_env(backend=os.environ.get("DDP_BACKEND", "gloo"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    run(int(sys.argv[2]), torch.device("cuda", torch.cuda.current_device()), sys.argv[1] if rank == 0 else None,
        rank=rank, defer="defer" in sys.argv[3:], world=world, split="split" in sys.argv[3:])
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
