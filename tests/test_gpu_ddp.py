"""The multi-rank training path (Trainer with world_size 2: graph without the optimizer, two-bucket
all-reduce SUM of the flat gradient overlapped with the deferred coarse-level scatter, Adam on DDP's
average — grad_scale 1/world on the fp32 wire, 1 on the fp16 wire, which divides before the sum) on
the one GPU of the test box: two torchrun ranks share cuda:0 over gloo, each trains on ITS OWN batches, and the parameters must equal a single-process run that accumulates the
gradients of both ranks' batches and steps once with grad_scale 1/2 (DDP's average without a
collective).  So a skipped or doubled all-reduce, a lost 1/world or a missing deferred scatter all
fail.  The table gradient's float-atomic summation order differs run to run (and Adam turns the sign
of a near-zero gradient into a full lr step), so the bound is the run-to-run floor of two
single-process runs: entries off by > 1e-4 at most 3x the floor + 1e-6 of all, and at most 0.1 %
off by more than 1e-6."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("defer,split", [(False, False), (True, False), (True, True)])
def test_two_rank_step_matches_single_process(dev, tmp_path, defer, split):
    """defer: the optimizer of step k inside graph k+1 (Trainer(defer_optimizer=True), the bench's
    default) after the eager all-reduce of step k; 3 steps so that two deferred steps run in-graph.
    split: the bench's split backward (Trainer(split_backward=True)), whose deferred coarse-level
    scatter the all-reduce overlaps as the autograd step's."""
    out = str(tmp_path / "flat.pt")
    steps = 3 if defer else 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "_ddp_step_worker.py"), out, str(steps)]
    if defer:
        cmd.append("defer")
    if split:
        cmd.append("split")
    env = dict(os.environ, DDP_BACKEND="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    dist_flat = torch.load(out, weights_only=True)
    sys.path.insert(0, HERE)
    from _ddp_step_worker import run_reference
    single = run_reference(steps, dev, world=2)
    single2 = run_reference(steps, dev, world=2)
    assert torch.isfinite(single).all()
    floor = int(((single2 - single).abs() > 1e-4).sum())
    d = (dist_flat - single).abs()
    assert int((d > 1e-4).sum()) <= 3 * floor + 1e-6 * d.numel(), (int((d > 1e-4).sum()), floor)
    assert float((d > 1e-6).float().mean()) <= 1e-3


@pytest.mark.parametrize("wire", ["fp32", "fp16"])
def test_config4_sharded_global_batch_8_ranks(dev, tmp_path, monkeypatch, wire):
    """Config #4's workload: ONE 65 536-ray global batch per step, sharded over 8 ranks by
    shard_patches (8192 rays of whole 8x8 patches each), the data-parallel Trainer step (graph,
    two-bucket all-reduce overlapped with the coarse scatter, deferred optimizer) on 8 gloo ranks
    sharing this GPU, against one process that accumulates the 8 shards' gradients and forms DDP's
    average.  wire="fp16" is the bench's wire for the fp16 AMP model: every rank's bucket is
    fp16(fp16(S g) / 8) (DDP divides before the SUM), and the emulation sums the 8 ranks in rank
    order with fp16 rounding — the collective's order may differ by a few fp16 ulps per entry (the
    bound of test_fp16_wire_8_ranks), which Adam's sign-like first steps absorb except where a sum
    is near zero, the same entries the float-atomic floor moves."""
    from ncnerf_amd import distributed
    monkeypatch.setattr(distributed, "DP_WIRE", wire if wire == "fp32" else "auto")
    out = str(tmp_path / "flat8.pt")
    # fp16: ONE step (applied by flush_optimizer), so that every entry the collective's order can move
    # is known from the emulation; a second step's forward would see the first step's order-moved
    # entries (full lr steps) and spread the difference.  The in-graph deferred optimizer at 8 ranks
    # is the fp32 case's (2 steps); the wire format does not enter it.
    steps, world = (2 if wire == "fp32" else 1), 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "_ddp_step_worker.py"), out, str(steps),
           "defer"]
    env = dict(os.environ, DDP_BACKEND="gloo", OMP_NUM_THREADS="2", DDP_GLOBAL_RAYS="65536",
               NCN_DP_WIRE=wire if wire == "fp32" else "auto")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    dist_flat = torch.load(out, weights_only=True)
    sys.path.insert(0, HERE)
    import _ddp_step_worker as w
    monkeypatch.setattr(w, "GLOBAL", "65536")
    single = w.run_reference(steps, dev, world=world)
    single2 = w.run_reference(steps, dev, world=world)
    assert torch.isfinite(single).all()
    floor = int(((single2 - single).abs() > 1e-4).sum())
    d = (dist_flat - single).abs()
    off = d > 1e-4
    # fp16: an entry whose 8-way sum lies within the fp16 sum's order bound of zero can round to
    # zero or to the other sign in the collective's order, which Adam's first steps turn into a full
    # lr difference; every other entry must agree as the fp32 wire's do
    amb = w.AMBIGUOUS[0] if wire == "fp16" else torch.zeros_like(off)
    unexplained = int((off & ~amb).sum())
    # the fp16 sum's order also moves a reduced value by ~2^-11 relative, i.e. an Adam update by
    # ~lr 2^-11 = 5e-6 once the moments differ: the small-difference threshold is lr 2^-9 there
    small = 1e-6 if wire == "fp32" else 1e-2 * 2.0 ** -9
    print(f"8 ranks ({wire} wire) vs single process: {int(off.sum())} entries off by > 1e-4 (floor {floor}; "
          f"{int((off & amb).sum())} of them order-ambiguous of {int(amb.sum())} such entries), "
          f"{float((d > small).float().mean()):.2e} off by > {small:.1e}")
    assert unexplained <= 3 * floor + 1e-6 * d.numel(), (unexplained, floor)
    assert float((d > small).float().mean()) <= 1e-3


def test_fp16_wire_8_ranks(tmp_path):
    """The fp16 gradient wire at 8 ranks (gloo on this GPU): ncn_grad_pack_f16 -> all-reduce SUM ->
    ncn_grad_unpack_f16 through distributed.reduce_gradients, against DDP's arithmetic emulated in
    one process: h_r = fp16(fp16(S g_r) / 8), summed.  The collective's summation order is its own,
    so the bound is the order-independent one of an fp16 sum of 8 terms: every partial sum is
    rounded once (<= 2^-11 of its magnitude, or half a subnormal step 2^-25), so
    |sum_got - sum_exact| <= 7 (2^-11 sum_r |h_r| + 2^-25).  Elements [0, 256) are S g = +-16 384 on
    every rank: finite per rank, an undivided 8-way sum (131 072) would overflow fp16 — the divided
    wire must give exactly +-16 384 / S (its partial sums are exact in any order).  The returned optimizer scale is 1 (already the average)."""
    out = str(tmp_path / "wire8.pt")
    world = 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "_ddp_wire_worker.py"), out]
    env = dict(os.environ, DDP_BACKEND="gloo", OMP_NUM_THREADS="1", NCN_DP_WIRE="auto")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = torch.load(out, weights_only=True)
    assert int(res["world"]) == world and float(res["scale"]) == 1.0
    sys.path.insert(0, HERE)
    import _ddp_wire_worker as ww
    from _ddp_step_worker import wire_sum, wire_value
    per_rank = [ww.rank_grad(r) for r in range(world)]
    S = ww.S
    h = torch.stack([wire_value(g, S, world).double() for g in per_rank])  # the ranks' wire values
    exact = h.sum(0)
    bound = (world - 1) * (2.0 ** -11 * h.abs().sum(0) + 2.0 ** -25)
    got = res["grad"].double() * S
    assert torch.isfinite(got).all()
    err = (got - exact).abs()
    assert bool((err <= bound).all()), (float((err - bound).max()), int((err > bound).sum()))
    # the overflow case: finite, and exactly the average of the ranks' equal values
    sign = torch.sign(per_rank[0][:ww.N_BIG].double())
    assert torch.equal(got[:ww.N_BIG], ww.BIG * sign)
    undivided = torch.stack([(g * S).half().double() for g in per_rank]).sum(0)
    assert bool((undivided[:ww.N_BIG].abs() > 65504).all())  # (the old wire's fp16 sum: inf)
    # and most entries agree with the rank-order emulation bit for bit
    rank_order = wire_sum(per_rank, S, world).double()
    same = float((got == rank_order).double().mean())
    print(f"fp16 wire, 8 ranks: max err / bound {float((err / bound).max()):.3f}, "
          f"{same:.4f} of the entries equal to the rank-order fp16 sum")
