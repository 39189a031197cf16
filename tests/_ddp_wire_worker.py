"""Worker of tests/test_gpu_ddp.py::test_fp16_wire_8_ranks (not a test module).

Every rank builds its own flat fp32 gradient on cuda:0 (seeded by rank), hands it to
distributed.reduce_gradients through a stand-in of the fp16 AMP model (amp_state = [S, 0]), i.e.
ncn_grad_pack_f16 (fp16(S g), then DDP's division by the world size, fp16 again) -> all-reduce SUM
-> ncn_grad_unpack_f16 (/ S), and rank 0 saves the reduced gradient and the returned optimizer scale.

`rank_grad` is also what the test's single-process emulation reads, so both sides see the same
values.  Element classes (by index):
  [0, n_big): S * g = +-16 384, the same on every rank — finite per rank (fp16 max 65 504), but an
              undivided 8-way sum (131 072) overflows, while DDP's divided sum (8 x 2 048) does not;
  [n_big, 2 n_big): S * g near fp16's subnormal range after the division (DDP's second rounding
              flushes / rounds them);
  the rest: S * g log-uniform over 1e-3 .. 1e3 with random signs (ordinary gradient values).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]

import torch  # noqa: E402

N = (1 << 16) + 5  # (a scalar tail past the kernels' 8-element chunks)
N_BIG = 256
S = 65536.0
BIG = 16384.0  # (every partial sum of 8 x BIG / 8 is a multiple of 2048: exact in fp16 in any order)


def rank_grad(rank):
    g = torch.Generator().manual_seed(7000 + rank)
    mag = 10.0 ** (torch.rand(N, generator=g, dtype=torch.float64) * 6 - 3)
    sign = torch.where(torch.rand(N, generator=g) < 0.5, -1.0, 1.0).double()
    sg = mag * sign
    big_sign = torch.where(torch.rand(N_BIG, generator=torch.Generator().manual_seed(6999)) < 0.5, -1.0, 1.0)
    sg[:N_BIG] = BIG * big_sign.double()  # (the same value on every rank)
    sg[N_BIG:2 * N_BIG] = 2.0 ** -21 * (1 + torch.rand(N_BIG, generator=g, dtype=torch.float64)) * sign[N_BIG:2 * N_BIG]
    return (sg / S).float()


class _AmpModel:
    """Stands in for the fp16 AMP NGPMT in reduce_gradients: one flat gradient, the GradScaler
    state, no deferred scatter."""

    def __init__(self, grad):
        self.g = grad
        self.amp_state = torch.tensor([S, 0.0], device=grad.device)
        self.scatter_split = None

    def flat_grad(self):
        return self.g


if __name__ == "__main__":
    from ncnerf_amd import distributed
    rank, world = distributed.init_from_env(backend=os.environ.get("DDP_BACKEND", "gloo"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    model = _AmpModel(rank_grad(rank).to(dev))
    assert distributed.wire_of(model) == "fp16"
    scale = distributed.reduce_gradients(model)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"grad": model.g.cpu(), "scale": torch.tensor(scale), "world": torch.tensor(world)},
                   sys.argv[1])
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
