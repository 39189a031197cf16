"""Multi-rank logic on CPU with gloo (world_size 2): gradient averaging of the flat buffer, the
two-bucket reduction overlapped with the deferred table scatter, patch sharding, occupancy
broadcast."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Model:
    def __init__(self, rank):
        self.density_grid = torch.full((1, 64), float(rank))
        self.density_bitfield = torch.full((8,), rank, dtype=torch.uint8)


class _SplitModel:
    """Stands in for NGPMT in reduce_gradients: a flat gradient [coarse levels | fine levels + W],
    a split, and a deferred scatter that adds into the coarse bucket (it must land before that
    bucket is reduced, and the fine bucket must not see it)."""

    def __init__(self, rank):
        self.scatter_split = 3
        self.g = torch.arange(12, dtype=torch.float32) + 100 * rank
        self._deferred = True
        self.calls = []

    def flat_grad(self):
        return self.g

    def grad_buckets(self, split):
        cut = 2 * split  # (2 floats per level in this stand-in)
        return self.g[cut:], self.g[:cut]

    def run_deferred_scatter(self, max_blocks=0, graph=False):
        self.calls.append(max_blocks)
        self.g[: 2 * self.scatter_split] += 1000.0


class _AmpStandIn:
    amp_state = object()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ncnerf_amd import distributed
    r, w = distributed.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    distributed.allreduce_grads(g)
    g2 = torch.ones(4) * (rank + 1)
    scale = distributed.allreduce_grads(g2, average=False)  # sum; the 1/world goes to the optimizer
    assert scale == 0.5 and g2.tolist() == [3.0] * 4
    sm = _SplitModel(rank)
    assert distributed.reduce_gradients(sm) == 0.5
    # DDP's average: the fp16 wire (an AMP model) divides before the sum, the fp32 wire after it
    assert distributed.grad_scale_after_reduce(_AmpStandIn()) == 1.0
    assert distributed.grad_scale_after_reduce(sm) == 0.5
    assert sm.calls == [distributed.DP_SCATTER_BLOCKS]
    base = torch.arange(12, dtype=torch.float32) * 2 + 100  # sum over ranks 0, 1 of arange + 100 r
    want_split = base.clone()
    want_split[:6] += 2000.0
    assert torch.equal(sm.g, want_split), sm.g
    m = _Model(rank)
    distributed.broadcast_occupancy(m)
    lo, hi = distributed.shard_patches(1024, rank, world)
    q.put((rank, g.tolist(), float(m.density_grid.sum()), int(m.density_bitfield.sum()), lo, hi))
    dist.destroy_process_group()


def test_gloo_two_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [1.5 * i for i in range(10)]  # mean of i*1 and i*2
    for rank, g, grid_sum, bf_sum, lo, hi in res:
        assert g == want
        assert grid_sum == 0.0 and bf_sum == 0  # rank 0's occupancy everywhere
        assert (lo, hi) == (rank * 512, (rank + 1) * 512)
