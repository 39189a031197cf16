"""The fused test-time render iteration (rendering.render_rays_test; default: driven from the device,
ncn_test_loop_*; test_fused="host": one host read of the alive count per iteration) against the loop
in the reference's structure (test_fused=False: valid mask, host-synced count, masked field evaluation,
scatter back into zero-filled sigmas / rgbs; rendering.py:45-149): opacity, depth, rgb and
total_samples bit-identical, on a random-init model (no ray terminates: the loop runs to the
sample budget) and on a model whose densities were fitted to the room's occupancy (rays stop at the
first surface), for full-image-shaped ray sets."""
import os
import sys

import pytest
import torch

from ncnerf_amd.ngp_mt import NGPMT, register_grid_buffers
from ncnerf_amd.rendering import render
from ncnerf_amd.synthetic import SyntheticScene

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(dev, scene, opaque):
    torch.manual_seed(0)
    m = register_grid_buffers(NGPMT(scale=0.5, grid_size=128).to(dev))
    with torch.no_grad():
        m.density_grid.copy_(torch.from_numpy(scene.density_grid).to(dev) * 10.0)
        m.density_bitfield.copy_(torch.from_numpy(scene.bitfield).to(dev))
    if opaque:
        sys.path.insert(0, ROOT)
        from bench import distill_opaque
        from ncnerf_amd.trainer import Trainer
        distill_opaque(m, Trainer(m, update_grid=False), scene, dev, steps=150)
    return m


@pytest.mark.parametrize("opaque,esf", [(False, 0.0), (True, 0.0), (False, 1.0 / 256)])
def test_fused_test_render_bit_identical(dev, opaque, esf):
    """esf > 0: exponential stepping, where the loop's minimum samples per ray is 4 (rendering.py:65)."""
    scene = SyntheticScene()
    m = _model(dev, scene, opaque)
    ro, rd = scene.image_rays(1, device=dev)
    n = ro.shape[0] // (4 if not opaque else 1)  # (the random model marches the whole budget)
    o, d = ro[:n].contiguous(), rd[:n].contiguous()
    outs = []
    for fused in (False, "host", True):
        st = {}
        with torch.no_grad():
            r = render(m, o, d, near_distance=0.01, max_samples=1024, test_time=True, test_fused=fused,
                       exp_step_factor=esf, loop_stats=st)
        torch.cuda.synchronize()
        outs.append((r, st))
    (a, sa) = outs[0]
    for b, sb in outs[1:]:
        for k in ("opacity", "depth", "rgb"):
            assert torch.equal(a[k], b[k]), k
        assert int(a["total_samples"]) == int(b["total_samples"])
        assert sa["iterations"] <= sb["iterations"] <= sa["iterations"] + 1, (sa, sb)
    if opaque:
        assert float(a["opacity"].mean()) > 0.9  # the fitted model's rays do stop
