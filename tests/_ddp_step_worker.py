"""Worker of tests/test_gpu_ddp.py (not a test module): under torchrun, every rank trains the same
model on the SAME batch through Trainer(use_graph=True) — the N>1 path: graph-captured step
without the optimizer, all-reduce SUM of the flat gradient, Adam with grad_scale = 1/world — and
rank 0 saves the parameters.  With identical batches the averaged gradient equals the
single-process gradient, so the result must match a 1-process run of the same steps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "normal-clustering-nerf_amd"), ROOT]

import torch  # noqa: E402


def run(steps, device, out=None):
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    scene = SyntheticScene()
    torch.manual_seed(0)
    model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(device))
    model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(device))
    tr = Trainer(model, use_graph=True)
    for k in range(steps):
        batch = scene.torch_batch(1024, seed=10 + k, device=device)
        batch["march_noise"] = torch.rand(1024, generator=torch.Generator().manual_seed(k)).to(device)
        tr.step(batch, global_step=3000 + k)
    torch.cuda.synchronize()
    flat = model.flat_params().detach().cpu().clone()
    if out:
        torch.save(flat, out)
    return flat


if __name__ == "__main__":
    from ncnerf_amd import distributed
    rank, world = distributed.init_from_env(backend=os.environ.get("DDP_BACKEND", "gloo"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    run(int(sys.argv[2]), torch.device("cuda", torch.cuda.current_device()), sys.argv[1] if rank == 0 else None)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
