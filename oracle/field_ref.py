"""ORACLE — test infrastructure only.  Never imported by the product path.

Pure-PyTorch (CPU, fp32) restatement of the NGPMT field (reference models/ngp_mt.py:10-229):
  * multires hash-grid encoding, tiny-cuda-nn "Grid/Hash" semantics (ngp_mt.py:70-82;
    L=16, F=2, log2_T=19, N_min=16, b = exp(ln(2048*scale/N_min)/(L-1)), ngp_mt.py:40-41);
  * sigma_net 32 -> 64 (ReLU) -> 16, no bias (ngp_mt.py:83-92) and sigma = TruncExp(h[:,0])
    (ngp_mt.py:168-169, custom_functions.py:162-173);
  * rgb_net cat([d/|d|, h]) 19 -> 64 -> 64 -> 3, ReLU hidden, Sigmoid output, no bias
    (ngp_mt.py:103-113, 206-209), in tcnn's padded form: `tcnn.Network(n_input_dims=19)` runs an
    Identity encoding that pads the input to the FullyFusedMLP's 16-alignment (32) with the value
    1.0, and the output layer is padded to 16 rows, so W3 is (64, 32) and W5 (16, 64) (7168
    rgb_net parameters, as tcnn reports) and only rows 0..2 of W5 produce outputs.

tiny-cuda-nn is NOT vendored in the reference (README.md:17, `pip install git+...tiny-cuda-nn` at
no pinned commit) and is not importable here, so this restates tcnn's published algorithm:
  grid_scale(l)  = exp2(l * log2(b)) * N_min - 1           (fp32)
  resolution(l)  = ceil(grid_scale(l)) + 1
  params(l)      = min(next_multiple(resolution^3, 8), 2^19)
  pos            = fma(grid_scale, x, 0.5); pos_grid = floor(pos); frac = pos - floor(pos)
  index          = dense x + y*res + z*res^2 while the stride stays <= params(l), else the
                   coherent prime hash  x*1 ^ y*2654435761 ^ z*805459861  (uint32), then % params(l)
  feature        = sum over the 8 corners of trilinear weight * table[index]
PARITY UNPINNED for this file: no reference test or fixture pins tcnn's numerics.  The documented
deviations from tcnn (fp32 table + fp32 interpolation instead of fp16) are listed in DESIGN.md.
`emulate_f16=True` (or emulate="bf16") rounds the MLP operands to fp16 (bf16) at the same points
the HIP kernel does (MFMA inputs in that type, fp32 accumulation), so the HIP path can be checked
tightly in either precision.
"""
import math

import numpy as np
import torch

L_LEVELS = 16
F_PER_LEVEL = 2
LOG2_T = 19
N_MIN = 16
PRIMES = (1, 2654435761, 805459861)


def grid_levels(scale=0.5, n_levels=L_LEVELS, log2_T=LOG2_T, n_min=N_MIN):
    """Per-level (grid_scale f32, resolution, params, offset, dense?) — ngp_mt.py:40-41 + tcnn."""
    b = math.exp(math.log(2048 * scale / n_min) / (n_levels - 1))
    log2_pls = np.float32(np.log2(np.float32(b)))
    levels = []
    offset = 0
    for l in range(n_levels):
        s = np.float32(np.exp2(np.float32(l) * log2_pls)) * np.float32(n_min) - np.float32(1.0)
        s = np.float32(s)
        res = int(math.ceil(float(s))) + 1
        dense = res ** 3
        params = ((dense + 7) // 8) * 8
        params = min(params, 1 << log2_T)
        levels.append(dict(scale=float(s), res=res, params=params, offset=offset,
                           hashed=res ** 3 > params))
        offset += params
    return levels, offset


def _grid_index(pg, res, params):
    """tcnn grid_index for one level; pg int64 (...,3) holding uint32 values."""
    stride = 1
    index = torch.zeros(pg.shape[:-1], dtype=torch.int64)
    for dim in range(3):
        if stride > params:
            break
        index = (index + pg[..., dim] * stride) & 0xFFFFFFFF
        stride *= res
    if params < stride:
        h = torch.zeros_like(index)
        for dim in range(3):
            h = h ^ ((pg[..., dim] * PRIMES[dim]) & 0xFFFFFFFF)
        index = h
    return index % params


def hash_encode(x01, table, levels):
    """x01: (N,3) f32 in [0,1]; table: (n_entries, 2) f32 -> (N, 32) f32 (level-major, 2 feats).

    All 16 levels x 8 corners are gathered by ONE `table[idx]` (so autograd scatters the table
    gradient once, not 128 times into dense zero tables)."""
    n = x01.shape[0]
    xd = x01.double()
    corner = torch.tensor([[(c >> dim) & 1 for dim in range(3)] for c in range(8)], dtype=torch.int64)  # (8,3)
    idx_l, w_l = [], []
    with torch.no_grad():
        for lv in levels:
            pos = (xd * lv["scale"] + 0.5).float()  # fma(scale, x, 0.5) in fp32 (exact product in f64)
            fl = torch.floor(pos)
            frac = pos - fl
            pg = (fl.to(torch.int64)) & 0xFFFFFFFF  # (uint32)(int)floor
            pc = (pg[:, None, :] + corner[None]) & 0xFFFFFFFF  # (N,8,3)
            # trilinear weight, product over dims in order x, y, z (as tcnn)
            wd = torch.where(corner[None].bool(), frac[:, None, :], 1 - frac[:, None, :])  # (N,8,3)
            w = torch.ones(n, 8, dtype=torch.float32) * wd[..., 0] * wd[..., 1] * wd[..., 2]
            idx_l.append(_grid_index(pc, lv["res"], lv["params"]) + lv["offset"])
            w_l.append(w)
    L = len(levels)
    idx = torch.stack(idx_l, 1)  # (N, L*8), level-major, corner-minor
    wts = torch.stack(w_l, 1).view(n, L, 8, 1)
    g = table[idx].view(n, L, 8, F_PER_LEVEL)
    return (wts * g).sum(2).reshape(n, L * F_PER_LEVEL)


_HG = None


def _hg_lib():
    """oracle/_build/libhashgrid_ref.so (oracle/hashgrid_ref.c), built on first use."""
    global _HG
    if _HG is None:
        import ctypes
        import os
        import subprocess
        here = os.path.dirname(os.path.abspath(__file__))
        so = os.path.join(here, "_build", "libhashgrid_ref.so")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(os.path.join(here, "hashgrid_ref.c")):
            subprocess.check_call(["make", "-s", "-C", here])
        _HG = ctypes.CDLL(so)
    return _HG


def _level_arrays(levels):
    key = id(levels)
    cache = getattr(_level_arrays, "cache", {})
    if key not in cache:
        cache[key] = (levels,
                      np.array([lv["scale"] for lv in levels], np.float32),
                      np.array([lv["res"] for lv in levels], np.int64),
                      np.array([lv["params"] for lv in levels], np.int64),
                      np.array([lv["offset"] for lv in levels], np.int64))
        _level_arrays.cache = cache
    return cache[key][1:]


class _HashEncodeC(torch.autograd.Function):
    """hash_encode through oracle/hashgrid_ref.c (same algorithm; fw gather, serial bw scatter)."""

    @staticmethod
    def forward(ctx, x01, table, levels):
        import ctypes
        L = _hg_lib()
        x = x01.detach().contiguous().float()
        tab = table.detach().contiguous()
        n = x.shape[0]
        enc = torch.empty(n, 2 * len(levels), dtype=torch.float32)
        arrs = _level_arrays(levels)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        L.hashgrid_fwd(P(x), ctypes.c_int64(n), P(tab), *[A(a) for a in arrs], P(enc))
        ctx.save_for_backward(x)
        ctx.levels, ctx.n_table = levels, table.shape
        return enc

    @staticmethod
    def backward(ctx, g):
        import ctypes
        (x,) = ctx.saved_tensors
        g = g.contiguous().float()
        dt = torch.zeros(ctx.n_table, dtype=torch.float32)
        arrs = _level_arrays(ctx.levels)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _hg_lib().hashgrid_bwd(P(x), ctypes.c_int64(x.shape[0]), P(g), *[A(a) for a in arrs], P(dt))
        return None, dt, None


def encode(x01, table, levels, impl="torch"):
    """hash_encode (impl "torch") or its C restatement (impl "c", oracle/hashgrid_ref.c)."""
    if impl == "c":
        return _HashEncodeC.apply(x01, table, levels)
    return hash_encode(x01, table, levels)


class _RoundST(torch.autograd.Function):
    """Round to fp16/bf16 in the forward, straight-through (fp32, unrounded) in the backward: the
    oracle's backward models the kernel's loss-scaled chain (no fp16 underflow), not an autograd
    cast whose backward would round the gradient to fp16 too."""

    @staticmethod
    def forward(ctx, t, dt):
        return t.to(dt).float()

    @staticmethod
    def backward(ctx, g):
        return g, None


class _RoundGrad(torch.autograd.Function):
    """Identity in the forward; in the backward the incoming gradient is rounded as the HIP field
    backward rounds it (ncn_field_bwd, csrc/field.hip bwd_group): carried at the scale K = 128 * S
    (tcnn's fp16 module loss scale x the GradScaler's S), converted to the MLP operand type (fp16
    overflow -> inf, underflow -> subnormal / 0), and handed on unscaled: fp16(g K) / K."""

    @staticmethod
    def forward(ctx, t, dt, K):
        ctx.dt, ctx.K = dt, K
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return (g * ctx.K).to(ctx.dt).float() / ctx.K, None, None


def _grad_rounder(emulate, bwd_scale):
    if emulate is None or bwd_scale is None:
        return lambda t: t
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[emulate]
    return lambda t: _RoundGrad.apply(t, dt, float(bwd_scale))


def _rounder(emulate_f16=False, emulate=None):
    mode = emulate or ("fp16" if emulate_f16 else None)
    if mode is None:
        return lambda t: t
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[mode]
    return lambda t: _RoundST.apply(t, dt)


class FieldParams:
    """fp32 master parameters: table (n_entries,2), W1 (64,32), W2 (16,64), W3 (64,32), W4 (64,64), W5 (16,64)."""

    def __init__(self, table, W1, W2, W3, W4, W5):
        self.table, self.W1, self.W2, self.W3, self.W4, self.W5 = table, W1, W2, W3, W4, W5

    def tensors(self):
        return [self.table, self.W1, self.W2, self.W3, self.W4, self.W5]


def rgb_input(d, h):
    """tcnn Identity encoding of rgb_net's 19 inputs cat[d/|d|, h], padded to 32 with 1.0."""
    return torch.cat([d, h, torch.ones(d.shape[0], 32 - 19, dtype=h.dtype)], dim=1)


def field_forward(xyzs, dirs, P, levels, scale=0.5, emulate_f16=False, emulate=None):
    """NGPMT.forward (ngp_mt.py:196-229) with density() (ngp_mt.py:157-171).
    Returns sigmas (N), rgbs (N,3), h (N,16)."""
    q = _rounder(emulate_f16, emulate)
    x01 = (xyzs - (-scale)) / (2 * scale)  # (x - xyz_min)/(xyz_max - xyz_min), ngp_mt.py:166
    enc = hash_encode(x01, P.table, levels)
    h1 = torch.relu(q(enc) @ q(P.W1).t())
    h = q(h1) @ q(P.W2).t()
    sig = torch.exp(h[:, 0])  # TruncExp forward
    d = dirs / torch.norm(dirs, dim=1, keepdim=True)
    g1 = torch.relu(q(rgb_input(d, h)) @ q(P.W3).t())
    g2 = torch.relu(q(g1) @ q(P.W4).t())
    rgb = torch.sigmoid((q(g2) @ q(P.W5).t())[:, :3])
    return sig, rgb, h


def density(xyzs, P, levels, scale=0.5, chunk=1 << 18, impl="torch", emulate=None):
    """NGPMT.density (ngp_mt.py:157-171): exp(sigma_net(enc(x))[:, 0]), fp32, in chunks (no grad);
    emulate ("fp16"/"bf16"): the MLP operands rounded as in field_forward."""
    q = _rounder(False, emulate)
    out = []
    with torch.no_grad():
        for i in range(0, xyzs.shape[0], chunk):
            x01 = (xyzs[i:i + chunk] - (-scale)) / (2 * scale)
            h = q(torch.relu(q(encode(x01, P.table, levels, impl)) @ q(P.W1).t())) @ q(P.W2).t()
            out.append(torch.exp(h[:, 0]))
    return torch.cat(out) if out else torch.zeros(0)


class _TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173"""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


def field_forward_autograd(xyzs, dirs, P, levels, scale=0.5, emulate_f16=False, emulate=None, impl="torch",
                           bwd_scale=None):
    """Same as field_forward with TruncExp's clamped backward, differentiable w.r.t. P.  With
    emulation the forward operands are rounded where the HIP kernel rounds them (the rounding is
    straight-through in the backward), so ReLU masks match the kernel's.  impl: the encoding's
    statement ("torch" or "c", see encode()).
    bwd_scale (with emulate): the backward's gradients are rounded where csrc/field.hip's bwd_group
    rounds them, at that scale (128 x the GradScaler's scale; 1 for bf16): the pre-sigmoid output
    gradient (dY5), the pre-ReLU gradients of layers 4, 3 and 1 (dD4, dD3, dD1), dL/dh after the rgb
    path and TruncExp's term are added (dhh), and dL/denc — the fp32 product of those rounded
    operands, stored in the operand type as tcnn hands its network's input gradient to the grid
    backward; the weight gradients are fp32 products, as the kernel's MFMA accumulates them."""
    q = _rounder(emulate_f16, emulate)
    rg = _grad_rounder(emulate or ("fp16" if emulate_f16 else None), bwd_scale)
    x01 = (xyzs - (-scale)) / (2 * scale)
    enc = rg(encode(x01, P.table, levels, impl))
    h = rg(q(torch.relu(rg(q(enc) @ q(P.W1).t()))) @ q(P.W2).t())
    sig = _TruncExp.apply(h[:, 0])
    d = dirs / torch.norm(dirs, dim=1, keepdim=True)
    g = torch.relu(rg(q(rgb_input(d, h)) @ q(P.W3).t()))
    g = torch.relu(rg(q(g) @ q(P.W4).t()))
    rgb = torch.sigmoid(rg(q(g) @ q(P.W5).t())[:, :3])
    return sig, rgb, h


def init_params(seed=0, scale=0.5, table_init=1e-4):
    """tcnn-style init: grid U(-1e-4, 1e-4); MLP weights Xavier-uniform."""
    levels, n_entries = grid_levels(scale)
    g = torch.Generator().manual_seed(seed)

    def xavier(o, i):
        a = math.sqrt(6.0 / (i + o))
        return (torch.rand(o, i, generator=g) * 2 - 1) * a

    table = (torch.rand(n_entries, 2, generator=g) * 2 - 1) * table_init
    P = FieldParams(table, xavier(64, 32), xavier(16, 64), xavier(64, 32), xavier(64, 64), xavier(16, 64))
    return P, levels
