"""Parity of the fused hash-grid + MLP field (ncn_field_fwd/bwd) with the torch CPU oracle
(oracle/field_ref.py, tiny-cuda-nn semantics restated; parity unpinned w.r.t. tcnn itself).

The model is tcnn's padded form (rgb_net input padded to 32 with 1.0: W3 (64,32); output padded to
16 rows: W5 (16,64)), in both MFMA operand precisions:
Forward tolerance: vs the oracle emulating the same operand rounding, fp16: |Δsigma| <= 2e-3*|sigma|
+ 1e-5 and |Δrgb| <= 2e-3; bf16 (8-bit mantissa: one operand rounding flip moves a value by up to
0.8 %): 2e-2*|sigma| + 1e-4 and 1e-2.  (fp32 accumulation in a different summation order.)
Backward tolerance: relative L2 error of each parameter-gradient block vs torch autograd through
the emulating oracle forward (same ReLU masks): <= 2e-2 (fp16), <= 5e-2 (bf16).  The padded
rows 3..15 of W5 get exactly zero gradient."""
import numpy as np
import pytest
import torch

from oracle import field_ref
from ncnerf_amd.ngp_mt import NGPMT, grid_levels

pytestmark = pytest.mark.gpu


TOL = {"fp16": dict(rtol=2e-3, atol=1e-5, rgb=2e-3, bwd=2e-2), "bf16": dict(rtol=2e-2, atol=1e-4, rgb=1e-2, bwd=5e-2)}


def _model_from_oracle(P, dev, precision="fp16", loss_scale=1.0):
    """loss_scale: the AMP scale of the fp16 backward (NGPMT.amp_state; the training default is
    GradScaler's 2^16, sized for a real step's ~1e-5 upstream gradients).  These tests drive the
    backward with upstream gradients of order 1, which that scale would overflow (GradScaler then
    skips the step and backs off), so they run it at 1 unless a test asks otherwise."""
    m = NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev)
    if loss_scale is not None and m.amp_state is not None:
        m.amp_state[0] = loss_scale
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


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("n", [1, 17, 4099])
def test_field_forward(dev, n, precision):
    P, levels = field_ref.init_params(seed=3, table_init=0.5)  # large table values exercise the encoding
    m = _model_from_oracle(P, dev, precision)
    x, d = _inputs(n, 1)
    with torch.no_grad():
        out = m(x.to(dev), d.to(dev))
        sig_d = m.density(x.to(dev))
    sig, rgb, _ = field_ref.field_forward(x, d, P, levels, emulate=precision)
    t = TOL[precision]
    np.testing.assert_allclose(out["sigmas"].cpu().numpy(), sig.numpy(), rtol=t["rtol"], atol=t["atol"])
    np.testing.assert_allclose(out["rgbs"].cpu().numpy(), rgb.numpy(), atol=t["rgb"])
    np.testing.assert_allclose(sig_d.cpu().numpy(), sig.numpy(), rtol=t["rtol"], atol=t["atol"])


def test_padded_rgb_input_is_a_bias(dev):
    """tcnn's constant-1 padding columns of W3 act as a bias: adding c to column 19+j of W3 equals
    adding c to the first rgb layer's pre-activation (checked against the oracle's padded form),
    and changes the output (the columns are live parameters)."""
    P, levels = field_ref.init_params(seed=4, table_init=0.5)
    x, d = _inputs(256, 3)
    m0 = _model_from_oracle(P, dev)
    with torch.no_grad():
        r0 = m0(x.to(dev), d.to(dev))["rgbs"].cpu()
    P.W3[:, 19:] += 0.05
    m1 = _model_from_oracle(P, dev)
    with torch.no_grad():
        r1 = m1(x.to(dev), d.to(dev))["rgbs"].cpu()
    _, rgb1, _ = field_ref.field_forward(x, d, P, levels, emulate_f16=True)
    assert float((r1 - r0).abs().max()) > 1e-3
    np.testing.assert_allclose(r1.numpy(), rgb1.numpy(), atol=2e-3)
    assert m1.rgb_net.params.numel() == 7168 and m1.sigma_net.params.numel() == 3072  # tcnn's counts


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("n", [3000, 4097, 12289])  # (scatter units of 4096 / 2048: partial last units, dynamic grabs)
def test_field_backward(dev, precision, n):
    P, levels = field_ref.init_params(seed=5, table_init=0.5)
    m = _model_from_oracle(P, dev, precision)
    x, d = _inputs(n, 2)
    g = torch.Generator().manual_seed(9)
    gs = torch.randn(n, generator=g)
    gr = torch.randn(n, 3, generator=g)
    out = m(x.to(dev), d.to(dev))
    (out["sigmas"] * gs.to(dev)).sum().add_((out["rgbs"] * gr.to(dev)).sum()).backward()
    gflat = m.flat_grad().cpu()
    Pt = field_ref.FieldParams(*[t.clone().requires_grad_(True) for t in P.tensors()])
    sig, rgb, _ = field_ref.field_forward_autograd(x, d, Pt, levels, emulate=precision)
    ((sig * gs).sum() + (rgb * gr).sum()).backward()
    off, errs = 0, {}
    for name, t in zip(("table", "W1", "W2", "W3", "W4", "W5"), Pt.tensors()):
        k = t.numel()
        got, ref = gflat[off:off + k].reshape(t.shape), t.grad
        errs[name] = float((got - ref).norm() / ref.norm().clamp_min(1e-12))
        off += k
    print("field backward rel errors:", precision, errs)
    assert all(e < TOL[precision]["bwd"] for e in errs.values()), errs
    w5 = gflat[-16 * 64:].reshape(16, 64)
    assert float(w5[3:].abs().max()) == 0.0  # padded output rows: no gradient


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_field_backward_tcnn_init(dev, precision):
    """The backward at tcnn's initialisation (table U(-1e-4, 1e-4)) with upstream gradients of a real
    step's size (~1e-5: MSE over 8192 rays): in fp16 the MLP chain underflows unless the loss is
    scaled, as the reference's AMP GradScaler does (train_nerf.py:954) — NGPMT.amp_state carries
    that scale (2^16).  Relative L2 per block as test_field_backward, and the table entries the
    oracle gives a gradient also get one (<= 0.1 % lost to fp16 range)."""
    n = 3000
    P, levels = field_ref.init_params(seed=5)
    m = _model_from_oracle(P, dev, precision, loss_scale=None)  # (the training default)
    x, d = _inputs(n, 2)
    g = torch.Generator().manual_seed(9)
    gs = torch.randn(n, generator=g) * 1e-5
    gr = torch.randn(n, 3, generator=g) * 1e-5
    out = m(x.to(dev), d.to(dev))
    (out["sigmas"] * gs.to(dev)).sum().add_((out["rgbs"] * gr.to(dev)).sum()).backward()
    gflat = m.flat_grad().cpu()
    Pt = field_ref.FieldParams(*[t.clone().requires_grad_(True) for t in P.tensors()])
    sig, rgb, _ = field_ref.field_forward_autograd(x, d, Pt, levels, emulate=precision)
    ((sig * gs).sum() + (rgb * gr).sum()).backward()
    off, errs = 0, {}
    for name, t in zip(("table", "W1", "W2", "W3", "W4", "W5"), Pt.tensors()):
        k = t.numel()
        got, ref = gflat[off:off + k].reshape(t.shape), t.grad
        errs[name] = float((got - ref).norm() / ref.norm().clamp_min(1e-30))
        if name == "table":
            nz_ref = ref.reshape(-1) != 0
            lost = int((nz_ref & (got.reshape(-1) == 0)).sum())
            assert lost <= 1e-3 * int(nz_ref.sum()), (lost, int(nz_ref.sum()))
        off += k
    print("field backward (tcnn init) rel errors:", precision, errs)
    # (at this init the encodings are ~1e-4, partly fp16 subnormals in the kernel's encoding cache:
    # W1's gradient, their outer product with dD1, carries that rounding)
    assert all(e < 2.5 * TOL[precision]["bwd"] for e in errs.values()), errs


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


@pytest.mark.parametrize("n", [8192, 13000])
def test_field_morton_window_order(dev, n):
    """ncn_field_sort_windows: `order` is a permutation of every 4096-sample window sorted by the
    Morton code of the positions (checked on the host), and the field evaluated in that processing
    order gives the same outputs (bitwise: each sample's arithmetic does not depend on its position)
    and the same gradients as in sample order up to summation order and the table scatter's
    fixed-point rounding (its addends are per-lane runs of samples sharing a cell, and which samples
    form a run depends on the processing order: 32-bit sums at 2^-(30 - log2(unit) - e) of the
    level's max |dE|, so relative L2 <= 2e-4 for the table block, 1e-5 for the MLP weights)."""
    from ncnerf_amd import _lib
    from ncnerf_amd._lib import F32, I64, ptr, stream
    P, _ = field_ref.init_params(seed=5, table_init=0.5)
    m = _model_from_oracle(P, dev)
    x, d = _inputs(n, 3)
    x, d = x.to(dev), d.to(dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    assert _lib.lib().ncn_field_sort_windows(ptr(x), I64(n), ptr(None), F32(m._xyz_min), F32(m._xyz_extent),
                                             ptr(order), stream()) == 0
    o = order.cpu().numpy().astype(np.int64)
    xc = x.cpu().numpy()
    q = np.clip(((xc - m._xyz_min) / m._xyz_extent * 1024).astype(np.int64), 0, 1023)

    def spread(v):
        r = np.zeros_like(v)
        for b in range(10):
            r |= ((v >> b) & 1) << (3 * b)
        return r
    code = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    for w0 in range(0, n, 4096):
        win = o[w0:w0 + 4096]
        assert np.array_equal(np.sort(win), np.arange(w0, min(n, w0 + 4096)))
        key = code[win] * 4096 + (win - w0)
        assert np.all(np.diff(key) > 0)

    def run(sort):
        m.sort_samples = sort
        m.flat_grad().zero_()
        xs, ds = x.clone(), d.clone()
        out = m(xs, ds)
        (out["sigmas"] * 0.01 + (out["rgbs"] * torch.linspace(-1, 1, 3, device=dev)).sum(1)).sum().backward()
        return out["sigmas"].detach().clone(), out["rgbs"].detach().clone(), m.flat_grad().clone()

    s0, r0, g0 = run(False)
    s1, r1, g1 = run(True)
    m.sort_samples = False
    assert torch.equal(s0, s1) and torch.equal(r0, r1)
    nt = m._n_table
    for (a, b), tol in (((g0[:nt], g1[:nt]), 2e-4), ((g0[nt:], g1[nt:]), 1e-5)):
        assert float((a - b).norm() / a.norm()) < tol


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_density_level_split_mode_bitexact(dev, precision):
    """ncn_field_fwd mode 2 (the grid refresh's density pass: encoding split by level over the
    XCDs into a scratch, then sigma_net) == mode 1 (sample-major) bit for bit, with a device count
    below the capacity (points past it untouched) and a count that is not a multiple of 16."""
    from ncnerf_amd import _lib
    from ncnerf_amd._lib import F32, I32, I64, ptr, stream
    from ncnerf_amd import vren
    m = NGPMT(scale=0.5, grid_size=128, precision=precision).to(dev)
    with torch.no_grad():
        m.flat_params()[: m._n_table].uniform_(-0.5, 0.5, generator=torch.Generator(device=dev).manual_seed(3))
    cap = 1 << 18
    cells = vren.morton3D_invert(torch.arange(0, 2 * cap, 2, dtype=torch.int32, device=dev))
    g = torch.Generator(device=dev).manual_seed(4)
    pts = ((cells.float() + torch.rand(cells.shape, device=dev, generator=g)) / 128 - 0.5).contiguous()
    packed = m._pack_weights()
    table = m.flat_params()[: m._n_table]
    for count in (cap, cap - 12345):
        n_dev = torch.tensor([count], dtype=torch.int32, device=dev)
        out = []
        for mode in (1, 2):
            sig = torch.full((cap,), -7.0, device=dev)
            enc = torch.empty(cap * 32, dtype=torch.float16, device=dev) if mode == 2 else None
            _lib.call("ncn_field_fwd", ptr(pts), ptr(None), I64(cap), ptr(n_dev), ptr(None), ptr(table),
                      m._levels_ptr, F32(m._xyz_min), F32(m._xyz_extent), ptr(packed), I32(m._prec), I32(mode),
                      ptr(sig), ptr(None), ptr(enc), stream())
            out.append(sig)
        torch.cuda.synchronize()
        assert torch.equal(out[0], out[1]), (precision, count)
        assert bool((out[1][count:] == -7.0).all()) and bool(torch.isfinite(out[1][:count]).all())
