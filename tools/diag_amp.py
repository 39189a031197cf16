import sys, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'normal-clustering-nerf_amd')
import test_gpu_amp_external as T
dev = torch.device("cuda:0")
from ncnerf_amd.losses import NeRFMTLoss
from ncnerf_amd.trainer import HYPERSIM_HPARAMS
loss_fn = NeRFMTLoss(dict(HYPERSIM_HPARAMS))
scene, mi = T._setup(dev, "internal"); _, mi2 = T._setup(dev, "internal"); _, me = T._setup(dev, "external")
b = T._batch(scene, 0, dev)
T._loss(mi, b, 0, loss_fn).backward(); T._loss(mi2, b, 0, loss_fn).backward()
S = 65536.0
(T._loss(me, b, 0, loss_fn) * S).backward()
g1, g2, ge = mi.flat_grad(), mi2.flat_grad(), me.flat_grad() / S
nt = mi._n_table
for name, a, c in (("int-int", g1, g2), ("ext-int", ge, g1)):
    d = (a - c).abs()
    nz = d > 0
    print(name, "differ:", int(nz[:nt].sum()), int(nz[nt:].sum()), "max", float(d[:nt].max()), float(d[nt:].max()))
    idx = torch.nonzero(nz[:nt])[:10, 0]
    print("  samples", [(int(i), float(a[i]), float(c[i])) for i in idx])
    zz = ((a == 0) != (c == 0))
    print("  zero-pattern differs:", int(zz.sum()))
# gradient magnitude distribution of table
gt = g1[:nt]; nzv = gt[gt != 0].abs()
print("table |g| quantiles", [float(torch.quantile(nzv[:1000000], q)) for q in (0.0, 0.001, 0.01, 0.5, 0.99)])
