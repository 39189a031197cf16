"""The split data-parallel backward (NGPMT.scatter_split): the table levels [0, split) of every
field backward are left for run_deferred_scatter (distributed.reduce_gradients runs it while the
first bucket's all-reduce is in flight).  A step with TWO field backwards must scatter both — the
pending scatters are a list, not one slot that the second backward overwrites — and each pending
scatter keeps its own per-level maxima (the fixed-point scale of its sums): a later backward with a
much smaller, or zero, upstream gradient must not rescale or drop an earlier one's."""
import pytest
import torch

from ncnerf_amd.ngp_mt import NGPMT

pytestmark = pytest.mark.gpu


def _loss(m, x, d, x2, w):
    out = m(x, d)
    s2 = m(x2, d)["sigmas"]
    return (out["sigmas"] * w[0]).sum() + (out["rgbs"] * w[1]).sum() + (s2 * w[2]).sum()


@pytest.mark.parametrize("later", [1.0, 1e-3, 0.0])
def test_two_backwards_both_deferred_scatters_run(dev, later):
    g = torch.Generator(device=dev).manual_seed(3)
    n = 5000
    x = (torch.rand(n, 3, device=dev, generator=g) - 0.5) * 0.98
    x2 = (torch.rand(n, 3, device=dev, generator=g) - 0.5) * 0.98
    d = torch.nn.functional.normalize(torch.randn(n, 3, device=dev, generator=g), dim=1)
    w = [torch.randn(n, device=dev, generator=g) * 1e-2, torch.randn(n, 3, device=dev, generator=g) * 1e-2,
         torch.randn(n, device=dev, generator=g) * 1e-2]
    grads = []
    for split in (None, 10):
        torch.manual_seed(0)
        m = NGPMT(scale=0.5, grid_size=128).to(dev)
        with torch.no_grad():
            m.flat_params()[: m._n_table].uniform_(-0.3, 0.3, generator=torch.Generator(device=dev).manual_seed(5))
        m.amp_state[0] = 1.0  # (order-1e-2 upstream gradients: no loss scale needed)
        m.scatter_split = split
        # two separate backwards in one step (e.g. a density() term and the render's forward())
        _loss(m, x, d, x2, w).backward()
        (m(x2, d)["rgbs"] * (w[1] * later)).sum().backward()
        if split is not None:
            assert len(m._deferred) == 3  # three field backwards, three pending coarse-level scatters
            m.run_deferred_scatter()
            assert m._deferred == []
        torch.cuda.synchronize()
        grads.append(m.flat_grad().clone())
    ref, got = grads
    assert torch.isfinite(got).all()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-6, rel
    # the same non-zero set, up to exact cancellations whose outcome depends on the float order of the
    # flushes (the encoding gradient is stored in fp16, so equal and opposite contributions of two
    # backwards are common: an entry's (q - q) + r and (r + q) - q can round differently).  Such an
    # entry is zero on one side and, on the other, the rounding residual of partials no larger than
    # the table's largest entries: a few ulps of them.  So every entry zero on one side only must lie
    # below ORDER_FLOOR = 2^-20 (16 ulps) of the largest entry, on either side; a dropped scatter zeroes
    # thousands of entries of ordinary size.
    ORDER_FLOOR = 2.0 ** -20 * float(ref.abs().max())
    one_side = (got == 0) != (ref == 0)
    resid = torch.maximum(got[one_side].abs(), ref[one_side].abs())
    assert resid.numel() == 0 or float(resid.max()) <= ORDER_FLOOR, (int(one_side.sum()), float(resid.max()),
                                                                     ORDER_FLOOR)
