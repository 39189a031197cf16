"""Diagnostic: per-step gradients/params of the internal (Trainer) and external (GradScaler+AdamW) loops."""
import sys, torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'normal-clustering-nerf_amd')
import test_gpu_amp_external as T
from ncnerf_amd.losses import NeRFMTLoss
from ncnerf_amd.trainer import HYPERSIM_HPARAMS, Trainer
dev = torch.device("cuda:0")
steps = 3
scene, mi = T._setup(dev, "internal"); tr = Trainer(mi)
_, me = T._setup(dev, "external")
loss_fn = NeRFMTLoss(dict(HYPERSIM_HPARAMS))
groups = [{"params": [me.xyz_encoder.params], "weight_decay": 0.0}, {"params": [me.sigma_net.params, me.rgb_net.params], "weight_decay": 1e-6}]
opt = torch.optim.AdamW(groups, lr=1e-2, betas=(0.9, 0.999), eps=1e-15, foreach=False)
scaler = torch.amp.GradScaler("cuda")
nt = mi._n_table
orig_step = tr.opt.step
gi = []
def cap_step(*a, **k):
    gi.append(mi.flat_grad().clone()); return orig_step(*a, **k)
tr.opt.step = cap_step
for k in range(steps):
    b = T._batch(scene, k, dev)
    r, ld = tr.step(b, global_step=T.STEP0 + k)
    opt.zero_grad(set_to_none=False)
    le = T._loss(me, b, k, loss_fn)
    scaler.scale(le).backward(); scaler.unscale_(opt)
    ge = me.flat_grad().clone()
    torch.nn.utils.clip_grad_norm_(list(me.parameters()), 0.05); scaler.step(opt); scaler.update()
    d = (gi[-1] - ge).abs()
    print(k, "loss", float(ld["total"]), float(le), "grad differ", int((d > 1e-6 * ge.abs().max()).sum()), "zero-pattern", int(((gi[-1]==0)!=(ge==0)).sum()))
    pd = (mi.flat_params() - me.flat_params()).abs(); bad = pd > 2e-6 * me.flat_params().abs() + 5e-7
    print("   params beyond", int(bad[:nt].sum()), int(bad[nt:].sum()), "max", float(pd.max()))
    idx = torch.nonzero(bad)[:6, 0]
    print("   ", [(int(i), float(mi.flat_params()[i]), float(me.flat_params()[i]), [float(g[i]) for g in gi], float(ge[i])) for i in idx])
