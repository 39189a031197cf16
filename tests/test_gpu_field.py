"""Parity of the fused hash-grid + MLP field (ncn_field_fwd/bwd) with the torch CPU oracle
(oracle/field_ref.py, tiny-cuda-nn semantics restated; parity unpinned w.r.t. tcnn itself).

Forward tolerance: vs the fp16-emulating oracle, |Δsigma| <= 2e-3*|sigma| + 1e-5 and
|Δrgb| <= 2e-3 (fp16 operands, fp32 accumulation, different summation order).
Backward tolerance: relative L2 error of each parameter-gradient block <= 2e-2 vs torch autograd
through the fp16-emulating oracle forward (same ReLU masks; fp16 MFMA operands in the backward)."""
import numpy as np
import pytest
import torch

from oracle import field_ref
from ncnerf_amd.ngp_mt import NGPMT, grid_levels

pytestmark = pytest.mark.gpu


def _model_from_oracle(P, dev):
    m = NGPMT(scale=0.5, grid_size=128).to(dev)
    flat = m.flat_params()
    n_table = m._n_table
    with torch.no_grad():
        flat[:n_table].copy_(P.table.reshape(-1))
        off = n_table
        for W in (P.W1, P.W2, P.W3, P.W4, P.W5):
            flat[off:off + W.numel()].copy_(W.reshape(-1))
            off += W.numel()
    return m


def _inputs(n, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(n, 3, generator=g) - 0.5) * 0.999
    d = torch.randn(n, 3, generator=g)
    d = d / d.norm(dim=1, keepdim=True)
    return x, d


def test_level_table_matches_oracle():
    lv, n = grid_levels(0.5)
    lo, no = field_ref.grid_levels(0.5)
    assert n == no  # same geometry as the oracle
    for a, b in zip(lv, lo):
        assert (a["scale"], a["res"], a["params"], a["offset"]) == (b["scale"], b["res"], b["params"], b["offset"])


@pytest.mark.parametrize("n", [1, 17, 4099])
def test_field_forward(dev, n):
    P, levels = field_ref.init_params(seed=3, table_init=0.5)  # large table values exercise the encoding
    m = _model_from_oracle(P, dev)
    x, d = _inputs(n, 1)
    with torch.no_grad():
        out = m(x.to(dev), d.to(dev))
        sig_d = m.density(x.to(dev))
    sig, rgb, _ = field_ref.field_forward(x, d, P, levels, emulate_f16=True)
    np.testing.assert_allclose(out["sigmas"].cpu().numpy(), sig.numpy(), rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(out["rgbs"].cpu().numpy(), rgb.numpy(), atol=2e-3)
    np.testing.assert_allclose(sig_d.cpu().numpy(), sig.numpy(), rtol=2e-3, atol=1e-5)


def test_field_backward(dev):
    n = 3000
    P, levels = field_ref.init_params(seed=5, table_init=0.5)
    m = _model_from_oracle(P, dev)
    x, d = _inputs(n, 2)
    g = torch.Generator().manual_seed(9)
    gs = torch.randn(n, generator=g)
    gr = torch.randn(n, 3, generator=g)
    out = m(x.to(dev), d.to(dev))
    (out["sigmas"] * gs.to(dev)).sum().add_((out["rgbs"] * gr.to(dev)).sum()).backward()
    gflat = m.flat_grad().cpu()
    Pt = field_ref.FieldParams(*[t.clone().requires_grad_(True) for t in P.tensors()])
    sig, rgb, _ = field_ref.field_forward_autograd(x, d, Pt, levels, emulate_f16=True)
    ((sig * gs).sum() + (rgb * gr).sum()).backward()
    off, errs = 0, {}
    for name, t in zip(("table", "W1", "W2", "W3", "W4", "W5"), Pt.tensors()):
        k = t.numel()
        got, ref = gflat[off:off + k].reshape(t.shape), t.grad
        errs[name] = float((got - ref).norm() / ref.norm().clamp_min(1e-12))
        off += k
    print("field backward rel errors:", errs)
    assert all(e < 2e-2 for e in errs.values()), errs


def test_field_backward_accumulates(dev):
    """Two backward passes accumulate into param.grad (views of the flat gradient buffer)."""
    P, levels = field_ref.init_params(seed=6, table_init=0.5)
    m = _model_from_oracle(P, dev)
    x, d = _inputs(512, 4)
    for _ in range(2):
        out = m(x.to(dev), d.to(dev))
        out["rgbs"].sum().backward()
    g2 = m.flat_grad().clone()
    m.flat_grad().zero_()
    out = m(x.to(dev), d.to(dev))
    out["rgbs"].sum().backward()
    assert torch.allclose(g2, 2 * m.flat_grad(), rtol=1e-4, atol=1e-7)
    assert m.xyz_encoder.params.grad.data_ptr() == m.flat_grad().data_ptr()
