"""Diagnostic: FlatAdam (apex arithmetic) vs torch.optim.AdamW on REAL gradient magnitudes."""
import sys, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'normal-clustering-nerf_amd')
import test_gpu_amp_external as T
from ncnerf_amd.losses import NeRFMTLoss
from ncnerf_amd.trainer import HYPERSIM_HPARAMS
from ncnerf_amd.optim import FlatAdam
dev = torch.device("cuda:0")
loss_fn = NeRFMTLoss(dict(HYPERSIM_HPARAMS))
scene, m = T._setup(dev, "internal")
grads = []
for k in range(3):
    b = T._batch(scene, k, dev)
    m.flat_grad().zero_()
    T._loss(m, b, k, loss_fn).backward()
    grads.append(m.flat_grad().clone())
p0 = m.flat_params().clone()
nt = m._n_table
class F:
    def __init__(s, p): s._p, s._g, s._n_table = p, torch.zeros_like(p), nt
    def flat_params(s): return s._p
    def flat_grad(s): return s._g
f = F(p0.clone()); opt = FlatAdam(f, lr=1e-2, max_norm=0.05, zero_grad_on_step=True)
a = p0[:nt].clone().requires_grad_(True); bb = p0[nt:].clone().requires_grad_(True)
topt = torch.optim.AdamW([{"params": [a], "weight_decay": 0.0}, {"params": [bb], "weight_decay": 1e-6}], lr=1e-2, eps=1e-15, foreach=False)
for g in grads:
    f._g.copy_(g); opt.step()
    a.grad, bb.grad = g[:nt].clone(), g[nt:].clone()
    print("norm", float(g.norm()))
    torch.nn.utils.clip_grad_norm_([a, bb], 0.05); topt.step()
    pt = torch.cat([a.detach(), bb.detach()])
    err = (f._p - pt).abs(); bad = err > 2e-6 * pt.abs() + 5e-7
    print("beyond:", int(bad[:nt].sum()), int(bad[nt:].sum()), "max", float(err.max()))
    idx = torch.nonzero(bad)[:8, 0]
    print([(int(i), float(f._p[i]), float(pt[i]), [float(gg[i]) for gg in grads]) for i in idx])
