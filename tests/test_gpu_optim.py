"""ncn_adam_step (FlatAdam) element-wise against (a) apex FusedAdam's AdamW arithmetic (the reference
optimizer, train_nerf.py:285; multi_tensor_adam's ADAM_MODE_1 restated in torch f32: moments with
the f32 betas, bias corrections 1 - beta**step formed in double on the host), tolerance 2e-6
relative + 1e-8; (b) torch.optim.AdamW, which forms (1 - beta) in double where apex uses f32
(1 - 0.999f is 1.3e-5 off 0.001), so the two optimizers' updates differ by up to ~1e-5 of lr:
tolerance 2e-6 relative + 5e-7.  Both after clip_grad_norm_(max_norm) on the scaled gradient and
with the reference's two groups (hash grid wd 0, nets wd 1e-6, eps 1e-15; train_nerf.py:262-285,
955).
Covers grad_scale != 1 (DDP's 1/world), an odd n (scalar tail), an odd group boundary, clipped and
unclipped norms, n beyond one grid-stride of the Adam launch, and the zero_grad fold."""
import math

import pytest
import torch

from ncnerf_amd.optim import FlatAdam

pytestmark = pytest.mark.gpu


class _Flat:
    def __init__(self, p, n_table):
        self._p, self._g, self._n_table = p, torch.zeros_like(p), n_table

    def flat_params(self):
        return self._p

    def flat_grad(self):
        return self._g


def _apex_reference(p0, grads, n0, scale, lr, max_norm, wd=(0.0, 1e-6), b1=0.9, b2=0.999, eps=1e-15):
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    wdv = torch.full_like(p0, wd[1])
    wdv[:n0] = wd[0]
    fb1, fb2 = torch.tensor(b1, dtype=torch.float32), torch.tensor(b2, dtype=torch.float32)
    for st, g in enumerate(grads, 1):
        gs = g * scale
        norm = float(gs.double().norm())
        gi = gs * min(1.0, max_norm / (norm + 1e-6))
        m = fb1 * m + (1 - fb1) * gi
        v = fb2 * v + (1 - fb2) * gi * gi
        bc1, bc2 = 1 - b1 ** st, 1 - b2 ** st
        upd = (m / bc1) / (torch.sqrt(v / bc2) + eps) + wdv * p
        p = p - lr * upd
    return p


def _torch_reference(p0, grads, n0, scale, lr, max_norm, wd=(0.0, 1e-6)):
    a = p0[:n0].clone().requires_grad_(True)
    b = p0[n0:].clone().requires_grad_(True)
    opt = torch.optim.AdamW([{"params": [a], "weight_decay": wd[0]}, {"params": [b], "weight_decay": wd[1]}],
                            lr=lr, betas=(0.9, 0.999), eps=1e-15, foreach=False)
    for g in grads:
        gs = g * scale
        a.grad, b.grad = gs[:n0].clone(), gs[n0:].clone()
        torch.nn.utils.clip_grad_norm_([a, b], max_norm)
        opt.step()
    return torch.cat([a.detach(), b.detach()])


@pytest.mark.parametrize("n,n0,scale,gmag,steps", [
    (100003, 70001, 0.5, 1e-2, 3),       # clipped (norm >> 0.05), odd sizes, DDP scale
    (100003, 70001, 1.0, 1e-5, 3),       # unclipped
    (4096, 4096, 0.25, 1.0, 3),          # one group only
    (34_000_003, 22_000_001, 0.5, 1e-3, 1),  # beyond 16384 workgroups x 2048 elements
])
def test_adam_step_matches_torch_adamw(dev, n, n0, scale, gmag, steps):
    g = torch.Generator(device=dev).manual_seed(n)
    p0 = torch.randn(n, device=dev, generator=g) * 0.1
    grads = [torch.randn(n, device=dev, generator=g) * gmag for _ in range(steps)]
    m = _Flat(p0.clone(), n0)
    opt = FlatAdam(m, lr=1e-2, max_norm=0.05, zero_grad_on_step=True)
    for gr in grads:
        m.flat_grad().copy_(gr)
        opt.step(grad_scale=scale)
        assert int(m.flat_grad().count_nonzero()) == 0  # gradient consumed and zeroed
    got = m.flat_params()
    for ref, atol in ((_apex_reference(p0, grads, n0, scale, 1e-2, 0.05), 1e-8),
                      (_torch_reference(p0, grads, n0, scale, 1e-2, 0.05), 5e-7)):
        err = (got - ref).abs()
        bad = int((err > 2e-6 * ref.abs() + atol).sum())
        assert bad == 0, (atol, bad, float(err.max()))
    assert int(opt.step_dev.item()) == steps


def test_adam_step_keeps_grad_without_fold(dev):
    m = _Flat(torch.zeros(1000, device=dev), 500)
    opt = FlatAdam(m, lr=1e-2, max_norm=0.05)
    m.flat_grad().fill_(1.0)
    opt.step()
    assert bool((m.flat_grad() == 1.0).all())


def test_trainer_sets_cosine_epoch_lr(dev):
    """Trainer.step applies CosineAnnealingLR(T_max=30) per 1000-step epoch (train_nerf.py:286-288)."""
    from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
    from ncnerf_amd.synthetic import SyntheticScene
    from ncnerf_amd.trainer import Trainer
    scene = SyntheticScene()
    model = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    model.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    tr = Trainer(model)
    batch = scene.torch_batch(256, seed=0, device=dev)
    for step, epoch in ((999, 0), (1000, 1), (14999, 14), (15000, 15)):
        tr.step(batch, global_step=step)
        want = 0.5 * 1e-2 * (1 + math.cos(math.pi * epoch / 30))
        assert abs(tr.opt.lr - want) < 1e-12 and abs(float(tr.opt.lr_dev.item()) - want) < 1e-9


def test_amp_grad_scaler_semantics(dev):
    """amp_state (torch GradScaler of the reference's fp16 run): a non-finite gradient skips the
    step (parameters, moments and the device step counter unchanged; the gradient still zeroed)
    and halves the scale; finite steps count up and the 2000th doubles the scale."""
    n = 4099
    p = torch.randn(n, device=dev)
    f = _Flat(p, 1001)
    f.amp_state = torch.tensor([65536.0, 0.0], device=dev)
    opt = FlatAdam(f, lr=1e-2, max_norm=0.05, zero_grad_on_step=True)
    f._g.copy_(torch.randn(n, device=dev))
    opt.step()
    torch.cuda.synchronize()
    assert f.amp_state.tolist() == [65536.0, 1.0] and int(opt.step_dev) == 1
    p1, m1, v1 = p.clone(), opt.m.clone(), opt.v.clone()
    f._g.copy_(torch.randn(n, device=dev))
    f._g[17] = float("inf")
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(p, p1) and torch.equal(opt.m, m1) and torch.equal(opt.v, v1)
    assert int(opt.step_dev) == 1 and f.amp_state.tolist() == [32768.0, 0.0]
    assert float(f._g.abs().max()) == 0.0
    f.amp_state[1] = 1999.0
    f._g.copy_(torch.randn(n, device=dev))
    opt.step()
    torch.cuda.synchronize()
    assert f.amp_state.tolist() == [65536.0, 0.0] and int(opt.step_dev) == 2
    assert not torch.equal(p, p1)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_adam_step_packed_matches_pack_weights(dev, precision):
    """ncn_adam_step_packed (FlatAdam on an NGPMT): the packed MLP fragments the Adam pass writes are
    bit-identical to ncn_field_pack_weights of the updated parameters — after a normal step, a
    clipped step, an AMP-skipped step (non-finite gradient: weights unchanged, fragments rewritten
    from them even if the buffer was stale) and a gated-off deferred step; and the parameters equal
    those of ncn_adam_step without the fold."""
    from ncnerf_amd import _lib
    from ncnerf_amd._lib import I32, ptr, stream
    from ncnerf_amd.ngp_mt import NGPMT, N_PACKED_HALVES
    torch.manual_seed(0)
    m = NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev)
    flat = m.flat_params()
    with torch.no_grad():
        flat.copy_(torch.randn_like(flat) * 0.05)
    ref = _Flat(flat.clone(), m._n_table)
    if m.amp_state is None:  # (bf16: a GradScaler state all the same, for the skipped step)
        m.amp_state = torch.tensor([65536.0, 0.0], device=dev)
    ref.amp_state = m.amp_state.clone()
    opt = FlatAdam(m, lr=1e-2, max_norm=0.05, zero_grad_on_step=True)
    opt_ref = FlatAdam(ref, lr=1e-2, max_norm=0.05, zero_grad_on_step=True)
    assert opt.pack_fused and not opt_ref.pack_fused

    def expected():
        out = torch.empty(N_PACKED_HALVES, dtype=torch.float16, device=dev)
        assert _lib.lib().ncn_field_pack_weights(ptr(flat[m._n_table:]), ptr(out), I32(m._prec), stream()) == 0
        return out

    g = torch.Generator(device=dev).manual_seed(3)
    for k, mag in enumerate((1e-4, 10.0, "inf", "gate", 1e-3)):
        gr = torch.randn(flat.numel(), device=dev, generator=g) * (1e-3 if isinstance(mag, str) else mag)
        if mag == "inf":
            gr[flat.numel() - 5] = float("inf")
        m.flat_grad().copy_(gr)
        ref.flat_grad().copy_(gr)
        m._packed.fill_(0)  # stale: the pass must rewrite every fragment
        gated = mag == "gate"
        opt.gate.fill_(0 if gated else 1)
        opt_ref.gate.fill_(0 if gated else 1)
        opt.step(gated=gated)
        opt_ref.step(gated=gated)
        torch.cuda.synchronize()
        assert torch.equal(flat, ref.flat_params()), k
        assert torch.equal(m._packed, expected()), k
    assert torch.equal(m.amp_state, ref.amp_state) and float(m.amp_state[0]) == 32768.0
