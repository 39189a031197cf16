"""The multi-rank training path (Trainer with world_size 2: graph without the optimizer, RCCL-style
all-reduce SUM of the flat gradient, Adam with grad_scale 1/world) on the one GPU of the test box:
two torchrun ranks share cuda:0 over gloo, both train on the same batches, and the parameters must
equal a single-process run of the same steps (identical gradients: sum * 1/2 is exact).
Tolerance: 1e-6 absolute on the parameters (expected bit-equal)."""
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


def test_two_rank_step_matches_single_process(dev, tmp_path):
    out = str(tmp_path / "flat.pt")
    steps = 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "_ddp_step_worker.py"), out, str(steps)]
    env = dict(os.environ, DDP_BACKEND="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    dist_flat = torch.load(out, weights_only=True)
    sys.path.insert(0, HERE)
    from _ddp_step_worker import run
    single = run(steps, dev)
    assert torch.isfinite(single).all()
    assert (dist_flat - single).abs().max().item() <= 1e-6
