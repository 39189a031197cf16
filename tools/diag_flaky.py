"""Diagnostic: which step of a graph-replayed run first departs from run 0 (the 15.7k-entry event)."""
import sys

import torch

sys.path.insert(0, "normal-clustering-nerf_amd")
from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers  # noqa: E402
from ncnerf_amd.synthetic import SyntheticScene  # noqa: E402
from ncnerf_amd.trainer import Trainer  # noqa: E402

dev = torch.device("cuda", 0)
scene = SyntheticScene()
split = len(sys.argv) > 1 and sys.argv[1] == "split"
NRUNS = int(sys.argv[2]) if len(sys.argv) > 2 else 6


def model():
    torch.manual_seed(7)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    with torch.no_grad():
        m.flat_params()[: m._n_table].uniform_(-1e-2, 1e-2)
        m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    return m


batches = []
for k in range(3):
    b = scene.torch_batch(4096, seed=90 + k, device=dev)
    b["march_noise"] = torch.rand(4096, device=dev, generator=torch.Generator(device=dev).manual_seed(90 + k))
    batches.append(b)
runs = []
for run in range(NRUNS):
    m = model()
    tr = Trainer(m, update_grid=False, use_graph=True, split_backward=split)
    rec = []
    for k in range(6):
        res, ld = tr.step(batches[k % 3], global_step=1000 + 300 * k)
        torch.cuda.synchronize()
        labels, cents, raw = tr.loss.last_cluster
        rec.append(dict(params=m.flat_params().detach().clone(), amp=m.amp_state.clone(),
                        loss={kk: float(v) for kk, v in ld.items()}, labels=labels.clone(), cents=cents.clone(),
                        raw=raw.clone(), vr=int(res["vr_samples"]), rm=int(res["rm_samples"]),
                        allloss=[float(v) for v in ld.values()]))
    runs.append(rec)
    nt = m._n_table
    print("run", run, "done", flush=True)
for run in range(1, NRUNS):
    for k in range(6):
        a, b = runs[0][k], runs[run][k]
        d = (a["params"][:nt] - b["params"][:nt]).abs()
        big = int((d > 1e-4).sum())
        print(f"run {run} step {k}: big {big} frac6 {float((d > 1e-6).float().mean()):.2e} "
              f"labels_diff {int((a['labels'] != b['labels']).sum())} cents {float((a['cents'] - b['cents']).abs().max()):.2e} "
              f"raw {float((a['raw'] - b['raw']).abs().max()):.2e} amp {a['amp'].tolist()} {b['amp'].tolist()} "
              f"loss {a['loss']['total']:.8f} {b['loss']['total']:.8f} vr {a['vr']} {b['vr']} rm {a['rm']} {b['rm']} "
              f"lossdiff {max(abs(x - y) for x, y in zip(a['allloss'], b['allloss'])):.2e}")
