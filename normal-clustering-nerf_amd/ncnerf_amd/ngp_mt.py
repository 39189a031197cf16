"""NGPMT field of the reference models/ngp_mt.py:10-368 on the fused gfx950 kernels.

Surface kept: `NGPMT(scale, grid_size, rgb_act='Sigmoid', pred_sem=False, pred_norm=False, **kw)`,
attributes read by render() (center, half_size, density_bitfield, cascades, scale, grid_size,
pred_norm, pred_sem), `forward(x, d) -> {'sigmas', 'rgbs'}`, `density(x, return_feat)`, and the
occupancy-grid maintenance (get_all_cells, sample_uniform_and_occupied_cells,
update_density_grid, mark_invisible_cells).  Parameter names keep tcnn's `<module>.params`
(xyz_encoder.params / sigma_net.params / rgb_net.params) so the reference's optimizer grouping
('xyz_encoder' in name -> no weight decay, train_nerf.py:262-274) applies unchanged.

Memory layout (MI355X): all parameters live in ONE flat fp32 buffer
  [hash table (n_entries x 2) | W1 (64,32) | W2 (16,64) | W3 (64,32) | W4 (64,64) | W5 (16,64)]
(tcnn's padded rgb_net: 19 inputs cat[d/|d|, h] + 13 constant-1 inputs, 3 outputs + 13 unused rows)
and their gradients in a second flat buffer of the same layout, so the gradient all-reduce is a
single RCCL call and the optimizer a single pass.  The backward accumulates straight into
`param.grad` (views of the flat gradient buffer): hash-table gradients by f32 atomics, weight
gradients through a fixed-order slab reduction.

Not provided (off in every reference config, hyperparameters.py:26-30): pred_sem / pred_norm heads,
rgb_act='None' exposure tonemappers.
"""
import math

import numpy as np
import torch
from einops import rearrange
from torch import nn

from . import _lib, vren
from ._lib import I32, I64, F32, call, ptr, stream

L_LEVELS, F_PER_LEVEL, LOG2_T, N_MIN = 16, 2, 19, 16  # ngp_mt.py:40
# tcnn's padded shapes (ngp_mt.py:83-113 through tcnn.Network): sigma_net W1 (64,32) W2 (16,64);
# rgb_net's 19 inputs padded to 32 with 1.0, 3 outputs padded to 16: W3 (64,32) W4 (64,64) W5 (16,64)
MLP_SHAPES = ((64, 32), (16, 64), (64, 32), (64, 64), (16, 64))
N_W = sum(o * i for o, i in MLP_SHAPES)  # NCN_FIELD_NW (10240: sigma_net 3072 + rgb_net 7168)
PRECISIONS = {"fp16": 0, "bf16": 1}  # NCN_PREC_F16 / NCN_PREC_BF16
N_PACKED_HALVES = 19456  # NCN_FIELD_PACKED_HALVES
ENC_BYTES = 64  # NCN_ENC_BYTES_PER_SAMPLE
SORT_MIN_SAMPLES = 8192  # training batches at least this large are evaluated in Morton-window order
W_SIGMA = 64 * 32 + 16 * 64
W_RGB = N_W - W_SIGMA


def grid_levels(scale, n_levels=L_LEVELS, log2_T=LOG2_T, n_min=N_MIN):
    """Per-level tcnn geometry: b = exp(ln(2048*scale/N_min)/(L-1)) (ngp_mt.py:41);
    grid_scale = exp2(l*log2(b))*N_min - 1 (fp32), resolution = ceil(scale)+1,
    params = min(next_multiple(res^3, 8), 2^log2_T).  Returns (levels, n_entries)."""
    b = math.exp(math.log(2048 * scale / n_min) / (n_levels - 1))
    log2_pls = np.float32(np.log2(np.float32(b)))
    levels, offset = [], 0
    for l in range(n_levels):
        s = np.float32(np.float32(np.exp2(np.float32(l) * log2_pls)) * np.float32(n_min) - np.float32(1.0))
        res = int(math.ceil(float(s))) + 1
        params = min(((res ** 3 + 7) // 8) * 8, 1 << log2_T)
        levels.append(dict(scale=float(s), res=res, params=params, offset=offset))
        offset += params
    return levels, offset


def level_words(levels):
    """16 x {scale f32 bits, res, params, offset} as a host uint32 array (the C ABI `levels`)."""
    w = np.zeros(64, np.uint32)
    for l, lv in enumerate(levels):
        w[4 * l] = np.frombuffer(np.float32(lv["scale"]).tobytes(), np.uint32)[0]
        w[4 * l + 1], w[4 * l + 2], w[4 * l + 3] = lv["res"], lv["params"], lv["offset"]
    return w


class _ParamHolder(nn.Module):
    """Stands in for a tcnn module: exposes `.params` (a view of the model's flat buffer)."""

    def __init__(self, flat_view):
        super().__init__()
        self.params = nn.Parameter(flat_view)


class _FieldFunction(torch.autograd.Function):
    """Fused hash-grid + sigma_net + TruncExp + rgb_net (ncn_field_fwd / ncn_field_bwd)."""

    @staticmethod
    def forward(ctx, x, d, table, w_sigma, w_rgb, model, mode, n_dev=None):
        need_grad = any(ctx.needs_input_grad[2:5])  # grad mode is off inside Function.forward
        sigmas, rgbs, enc, packed, order = model._field_fwd(x, d, n_dev, mode, need_grad)
        if need_grad:
            ctx.save_for_backward(x, d, enc, packed, n_dev, order)
            ctx.model = model
        if mode != 0:
            ctx.mark_non_differentiable(rgbs)
        ctx.set_materialize_grads(False)
        return sigmas, rgbs

    @staticmethod
    def backward(ctx, dL_dsigmas, dL_drgbs):
        x, d, enc, packed, n_dev, order = ctx.saved_tensors
        model = ctx.model
        n = x.shape[0]
        g_table, g_w = model._grad_views()
        nb = _lib.lib().ncn_field_bwd_blocks(I64(n))
        slab = torch.empty(nb * N_W, dtype=torch.float32, device=x.device)
        dE_ws = torch.empty(int(_lib.lib().ncn_field_bwd_dE_floats(I64(n))), dtype=torch.float32, device=x.device)
        c = lambda t: None if t is None else t.contiguous().float()
        dsig, drgb = c(dL_dsigmas), c(dL_drgbs)
        if model.scatter_split is None:
            call("ncn_field_bwd", ptr(x), ptr(d), I64(n), ptr(n_dev), ptr(order), model._levels_ptr, F32(model._xyz_min),
                 F32(model._xyz_extent), ptr(packed), I32(model._prec), ptr(enc), ptr(dsig), ptr(drgb),
                 ptr(model._bwd_loss_scale()), ptr(g_table), ptr(slab), ptr(dE_ws), ptr(model._level_max()), stream())
        else:
            lmax = model._level_max()
            call("ncn_field_bwd_mlp", ptr(x), ptr(d), I64(n), ptr(n_dev), ptr(order), ptr(packed), I32(model._prec), ptr(enc),
                 ptr(dsig), ptr(drgb), ptr(model._bwd_loss_scale()),
                 ptr(slab), ptr(dE_ws), ptr(lmax), stream())
            model._scatter(x, n, n_dev, order, dE_ws, lmax, g_table)
        call("ncn_field_reduce_wgrad", ptr(slab), I32(nb), ptr(g_w), stream())
        return None, None, None, None, None, None, None, None


class NGPMT(nn.Module):
    def _bwd_loss_scale(self):
        """The field backward's loss_scale operand (ncn_field_bwd): the internal GradScaler's scale,
        a device 1.0 under external AMP, None for bf16."""
        return self.amp_state if self.amp_state is not None else self._amp_unit

    def _level_max(self):
        """ncn_field_bwd's per-level max |dE| workspace: 16 floats per MLP-pass workgroup (<= 256).
        The scatter reads it as each level's fixed-point scale, so with scatter_split set (a backward
        whose coarse levels are scattered later, run_deferred_scatter) every backward gets its own:
        a shared buffer would hand the earlier pending scatters the LAST backward's maxima
        (overflowing 64-bit sums, or a level dropped when its maximum there is 0)."""
        dev = self._flat.device
        if self.scatter_split is not None:
            return torch.empty(16 * 256, dtype=torch.float32, device=dev)
        if getattr(self, "_lmax", None) is None or self._lmax.device != dev:
            self._lmax = torch.empty(16 * 256, dtype=torch.float32, device=dev)
        return self._lmax

    def __init__(self, scale, grid_size, rgb_act="Sigmoid", pred_sem=False, pred_norm=False, seed=1337,
                 precision="fp16", amp="internal", **kwargs):
        """precision: MFMA operand type of the MLPs, "fp16" (tcnn's FullyFusedMLP, the reference's AMP
        run) or "bf16" (config #3); parameters, table and accumulation stay fp32.
        amp (fp16 only): "internal" — the model keeps its own GradScaler state (`amp_state`, updated by
        FlatAdam / ncn_adam_step) and the field backward applies it at the MLP's boundary, so the
        caller's loss is unscaled (the Trainer path); "external" — the caller runs AMP itself
        (train_nerf.py's PL precision=16 + GradScaler, or torch.cuda.amp.GradScaler): the upstream
        gradient arrives already scaled, the backward applies only tcnn's own fp16 module scale
        (x128 in, /128 out, NCN_TCNN_LOSS_SCALE) and the gradients leave in the caller's scale, as
        tcnn's do; any optimizer (torch.optim.Adam(W), apex FusedAdam) then steps them."""
        super().__init__()
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        if amp not in ("internal", "external"):
            raise ValueError("amp must be 'internal' or 'external'")
        self.amp = amp
        self.precision = precision
        self._prec = PRECISIONS[precision]
        if rgb_act != "Sigmoid":
            raise NotImplementedError("rgb_act='None' (exposure tonemappers) is off in every reference config")
        if pred_sem or pred_norm:
            raise NotImplementedError("pred_sem / pred_norm heads are off in every reference config")
        self.pred_sem, self.pred_norm, self.rgb_act = pred_sem, pred_norm, rgb_act
        self.scale = scale
        self.register_buffer("center", torch.zeros(1, 3))
        self.register_buffer("xyz_min", -torch.ones(1, 3) * scale)
        self.register_buffer("xyz_max", torch.ones(1, 3) * scale)
        self.register_buffer("half_size", (self.xyz_max - self.xyz_min) / 2)
        # the scene box as host floats for the one-launch marcher (no device read per step)
        self._aabb = (tuple(float(v) for v in self.center[0]), tuple(float(v) for v in self.half_size[0]))
        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)  # ngp_mt.py:34
        self.grid_size = grid_size
        self.register_buffer("density_bitfield", torch.zeros(self.cascades * grid_size ** 3 // 8, dtype=torch.uint8))
        self.levels, self.n_entries = grid_levels(scale)
        self._level_words = level_words(self.levels)
        self._levels_ptr = self._level_words.ctypes.data_as(_lib.P)
        self._xyz_min = float(np.float32(-scale))
        self._xyz_extent = float(np.float32(scale) - np.float32(-scale))
        n_table = self.n_entries * F_PER_LEVEL
        self._n_table = n_table
        flat = torch.zeros(n_table + N_W)
        g = torch.Generator().manual_seed(seed)
        flat[:n_table] = (torch.rand(n_table, generator=g) * 2 - 1) * 1e-4  # tcnn grid init U(-1e-4, 1e-4)
        off = n_table
        for o, i in MLP_SHAPES:  # Xavier-uniform MLP weights (tcnn initialises the padded matrices)
            a = math.sqrt(6.0 / (o + i))
            flat[off:off + o * i] = (torch.rand(o * i, generator=g) * 2 - 1) * a
            off += o * i
        self._flat = flat
        self.xyz_encoder = _ParamHolder(flat[:n_table])
        self.sigma_net = _ParamHolder(flat[n_table:n_table + W_SIGMA])
        self.rgb_net = _ParamHolder(flat[n_table + W_SIGMA:])
        self._flat_grad = None
        self._packed = None
        # AMP GradScaler state {scale, growth tracker} of the fp16 MLP (the reference trains with
        # precision=16, train_nerf.py:954: the scaled loss keeps tcnn's fp16 backward from
        # underflowing): the field backward multiplies its upstream gradients by the scale and
        # divides its outputs by it; ncn_adam_step skips non-finite steps and grows / backs off the
        # scale.  bf16 operands (fp32's exponent range) run unscaled, as PL's bf16 mode does.
        f16 = precision == "fp16"
        self.register_buffer("amp_state", torch.tensor([_lib.AMP_INIT_SCALE, 0.0]) if f16 and amp == "internal" else None)
        # external AMP: the backward's loss-scale operand is a constant 1 (only tcnn's x128 remains)
        self.register_buffer("_amp_unit", torch.ones(1) if f16 and amp == "external" else None, persistent=False)
        # None: the backward scatters every level.  An int L (data-parallel step): levels [L, 16)
        # are scattered in the backward, [0, L) by run_deferred_scatter() (grad_buckets(L)).
        self.scatter_split = None
        # Morton-window processing order (ncn_field_sort_windows) for training batches: off by default
        # (measured: forward 88 -> 72 us, but sort 40 us + MLP backward +6 us + scatter +9 us)
        self.sort_samples = False
        self._deferred = []  # pending coarse-level scatters of the split data-parallel step (eager backwards)
        self._deferred_graph = []  # the captured step's coarse-level scatters (Trainer._capture), every replay

    # -- flat buffers --------------------------------------------------------------------------
    def _apply(self, fn, recurse=True):
        # keep the three parameters as views of one flat buffer across .to()/.cuda()
        super()._apply(fn, recurse)
        flat = fn(self._flat)
        n_table = self._n_table
        flat[:n_table].copy_(self.xyz_encoder.params.data)
        flat[n_table:n_table + W_SIGMA].copy_(self.sigma_net.params.data)
        flat[n_table + W_SIGMA:].copy_(self.rgb_net.params.data)
        self._flat = flat
        self.xyz_encoder.params.data = flat[:n_table]
        self.sigma_net.params.data = flat[n_table:n_table + W_SIGMA]
        self.rgb_net.params.data = flat[n_table + W_SIGMA:]
        self._flat_grad = None
        self._packed = None
        return self

    def flat_params(self):
        return self._flat

    def flat_grad(self):
        """The flat gradient buffer; every parameter's .grad is a view of it."""
        self._grad_views()
        return self._flat_grad

    def _grad_views(self):
        ps = (self.xyz_encoder.params, self.sigma_net.params, self.rgb_net.params)
        if self._flat_grad is None or self._flat_grad.device != self._flat.device:
            self._flat_grad = torch.zeros_like(self._flat)
        fg, n_table = self._flat_grad, self._n_table
        views = (fg[:n_table], fg[n_table:n_table + W_SIGMA], fg[n_table + W_SIGMA:])
        for p, v in zip(ps, views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                if p.grad is not None:
                    v.copy_(p.grad)
                else:
                    v.zero_()
                p.grad = v
        return fg[:n_table], fg[n_table:]

    def grad_buckets(self, split):
        """The flat gradient as (levels [split, 16) of the table + the MLP weights, levels [0, split)):
        two contiguous views, the all-reduce buckets of the split data-parallel step."""
        fg = self.flat_grad()
        cut = 2 * self.levels[split]["offset"]
        return fg[cut:], fg[:cut]

    def run_deferred_scatter(self, max_blocks=0, graph=False):
        """Scatter of the levels [0, scatter_split) left by the field backwards: graph=False — the
        eager backwards since the last call (then cleared); graph=True — the captured step's entries
        (Trainer._capture moves them to _deferred_graph: they name the graph's static buffers, refilled
        by every replay, and are run after each replay)."""
        entries = self._deferred_graph if graph else self._deferred
        if not entries:
            raise RuntimeError("run_deferred_scatter: no deferred scatter (scatter_split unset or no backward yet)")
        for x, n, n_dev, order, dE_ws, lmax, g_table in entries:
            call("ncn_field_scatter", ptr(x), I64(n), ptr(n_dev), ptr(order), self._levels_ptr, F32(self._xyz_min),
                 F32(self._xyz_extent), ptr(dE_ws), ptr(lmax), I32(0), I32(self.scatter_split), I32(max_blocks),
                 ptr(g_table), stream())
        if not graph:
            self._deferred = []

    def prepare_weights(self):
        """Pack the MLP weights now (after the optimizer step) so the next forward reuses them.
        The packed fragments are reused by the next forward while `_packed_fresh` is set (FlatAdam's
        packed step sets it: its Adam pass writes the fragments of the weights it updates).  A caller
        that changes the parameters any other way (an in-place edit, a copy from another model, a
        broadcast) must call prepare_weights() afterwards; load_state_dict clears the flag itself."""
        self._pack_weights()
        self._packed_fresh = True

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._packed_fresh = False  # (the loaded weights: the next forward packs them)

    def _take_packed(self):
        if getattr(self, "_packed_fresh", False) and self._packed is not None:
            self._packed_fresh = False
            return self._packed
        return self._pack_weights()

    def pack_target(self):
        """(pack_inv, pack_off, packed, precision) for ncn_adam_step_packed: the optimizer refreshes
        the packed MLP fragments itself (no pack launch between it and the next forward).  pack_inv
        (NCN_FIELD_NW x 2 int32, -1 = none) lists each master weight's packed elements, from
        ncn_field_pack_map; built once.  The packed buffer is allocated (and packed) if needed."""
        if self._packed is None or self._packed.device != self._flat.device:
            self._pack_weights()
        inv = getattr(self, "_pack_inv", None)
        if inv is None or inv.device != self._flat.device:
            src = torch.empty(N_PACKED_HALVES, dtype=torch.int32, device=self._flat.device)
            call("ncn_field_pack_map", ptr(src), stream())
            s = src.cpu().numpy()
            table = np.full((N_W, 2), -1, np.int32)
            fill = np.zeros(N_W, np.int64)
            for q, w in enumerate(s):
                assert 0 <= w < N_W and fill[w] < 2, (q, w)
                table[w, fill[w]] = q
                fill[w] += 1
            inv = self._pack_inv = torch.from_numpy(table).to(self._flat.device)
        return inv, self._n_table, self._packed, self._prec

    def _pack_weights(self):
        if self._packed is None or self._packed.device != self._flat.device:
            self._packed = torch.empty(N_PACKED_HALVES, dtype=torch.float16, device=self._flat.device)
        call("ncn_field_pack_weights", ptr(self._flat[self._n_table:]), ptr(self._packed), I32(self._prec), stream())
        return self._packed

    # -- field -----------------------------------------------------------------------------------
    def _field_fwd(self, x, d, n_dev, mode, need_grad):
        """ncn_field_fwd on x (N,3) / d (N,3) fp32 contiguous (capacity N when n_dev, a device int32
        count, is given) -> (sigmas, rgbs, enc_cache, packed weights, order); enc_cache and order
        (None unless sort_samples) are the backward's inputs, None without need_grad."""
        n = x.shape[0]
        dev = x.device
        sigmas = torch.empty(n, dtype=torch.float32, device=dev)
        rgbs = torch.empty(n, 3, dtype=torch.float32, device=dev) if mode == 0 else sigmas.new_empty(0, 3)
        enc = None
        if need_grad:
            enc = torch.empty(((n + 15) // 16) * 16 * ENC_BYTES // 2, dtype=torch.float16, device=dev)
        packed = self._take_packed()
        order = None
        if need_grad and self.sort_samples and n >= SORT_MIN_SAMPLES:
            # processing order: Morton-sorted windows of 4096 samples (ncn_field_sort_windows); the
            # encoding cache and the backward's dE are kept in it, the outputs stay in sample order
            order = torch.empty(n, dtype=torch.int32, device=dev)
            call("ncn_field_sort_windows", ptr(x), I64(n), ptr(n_dev), F32(self._xyz_min), F32(self._xyz_extent),
                 ptr(order), stream())
        call("ncn_field_fwd", ptr(x), ptr(d) if mode == 0 else ptr(None), I64(n), ptr(n_dev), ptr(order),
             ptr(self.xyz_encoder.params), self._levels_ptr, F32(self._xyz_min), F32(self._xyz_extent), ptr(packed), I32(self._prec), I32(mode),
             ptr(sigmas), ptr(rgbs) if mode == 0 else ptr(None), ptr(enc), stream())
        return sigmas, rgbs, enc, packed, order

    def _scatter(self, x, n, n_dev, order, dE_ws, lmax, g_table, wgrad=None):
        """Table scatter after the MLP pass: every level (scatter_split None), else the levels
        [scatter_split, 16) now and [0, scatter_split) queued for run_deferred_scatter() — the
        data-parallel step scatters them while the all-reduce of the first bucket is in flight.
        wgrad = (slab, sigma-pass rows, rgb-pass rows, grad_w): the split backward's weight-gradient
        reduction, folded into this launch (ncn_field_scatter_wgrad)."""
        split = self.scatter_split
        lo = 0 if split is None else split
        slab, nb_s, nb_r, g_w = wgrad if wgrad is not None else (None, 0, 0, None)
        call("ncn_field_scatter_wgrad", ptr(x), I64(n), ptr(n_dev), ptr(order), self._levels_ptr, F32(self._xyz_min),
             F32(self._xyz_extent), ptr(dE_ws), ptr(lmax), I32(lo), I32(16), I32(0), ptr(g_table), ptr(slab),
             I32(nb_s), I32(nb_r), ptr(g_w), stream())
        if split is not None:
            # (a list: a step with two field backwards — e.g. density() with grad and forward() —
            # leaves two pending coarse-level scatters, both run by run_deferred_scatter)
            self._deferred.append((x, n, n_dev, order, dE_ws, lmax, g_table))

    def density(self, x, return_feat=False):
        """ngp_mt.py:157-171 (density-only kernel mode)."""
        if return_feat:
            raise NotImplementedError("return_feat (the 16-d sigma_net feature) is only needed by the "
                                      "pred_sem/pred_norm heads, which are not provided")
        _lib.check_input(x, "x")
        sigmas, _ = _FieldFunction.apply(x.float().contiguous(), None, self.xyz_encoder.params,
                                         self.sigma_net.params, self.rgb_net.params, self, 1)
        return sigmas

    def forward(self, x, d, **kwargs):
        """ngp_mt.py:196-229 -> {'sigmas': (N,), 'rgbs': (N,3)} (fp32).

        kwargs['n_samples_dev'] (extension): a device int32 sample count <= len(x); x/d are then
        static-capacity buffers and only the first *n_samples_dev rows are evaluated."""
        x = x.float().contiguous()
        d = d.float().contiguous()
        _lib.check_input(x, "x")
        _lib.check_input(d, "d")
        n_dev = kwargs.get("n_samples_dev")
        sigmas, rgbs = _FieldFunction.apply(x, d, self.xyz_encoder.params, self.sigma_net.params,
                                            self.rgb_net.params, self, 0, n_dev)
        return {"sigmas": sigmas, "rgbs": rgbs}

    # -- occupancy grid maintenance (ngp_mt.py:231-368) --------------------------------------------
    @torch.no_grad()
    def get_all_cells(self):
        indices = vren.morton3D(self.grid_coords).long()
        return [(indices, self.grid_coords)] * self.cascades

    @torch.no_grad()
    def sample_uniform_and_occupied_cells(self, M, density_threshold):
        cells = []
        for c in range(self.cascades):
            coords1 = torch.randint(self.grid_size, (M, 3), dtype=torch.int32, device=self.density_grid.device)
            indices1 = vren.morton3D(coords1).long()
            indices2 = torch.nonzero(self.density_grid[c] > density_threshold)[:, 0]
            if len(indices2) > 0:
                rand_idx = torch.randint(len(indices2), (M,), device=self.density_grid.device)
                indices2 = indices2[rand_idx]
            coords2 = vren.morton3D_invert(indices2.int().contiguous())
            cells += [(torch.cat([indices1, indices2]), torch.cat([coords1, coords2]))]
        return cells

    @torch.no_grad()
    def mark_invisible_cells(self, K, dev, poses, img_wh, near_distance, chunk=64 ** 3):
        """ngp_mt.py:274-337 (pinhole K (3,3) tensor branch and the Hypersim NDC tuple branch)."""
        N_cams = poses.shape[0]
        self.count_grid = torch.zeros_like(self.density_grid)
        w2c_R = rearrange(poses[:, :3, :3], "n a b -> n b a")
        w2c_T = -w2c_R @ poses[:, :3, 3:]
        cells = self.get_all_cells()
        if isinstance(K, torch.Tensor):
            K = K.to(dev)
        elif isinstance(K, tuple):
            M_ndc_from_cam, M_uv_from_ndc = K[0].to(dev), K[1].to(dev)
            k_scale = K[3]
        else:
            raise AssertionError
        for c in range(self.cascades):
            indices, coords = cells[c]
            for i in range(0, len(indices), chunk):
                xyzs = coords[i:i + chunk] / (self.grid_size - 1) * 2 - 1
                s = min(2 ** (c - 1), self.scale)
                half_grid_size = s / self.grid_size
                xyzs_w = (xyzs * (s - half_grid_size)).T
                xyzs_c = w2c_R @ xyzs_w + w2c_T
                if isinstance(K, torch.Tensor):
                    uvd = K @ xyzs_c
                    uv = uvd[:, :2] / uvd[:, 2:]
                else:
                    xyzs_c *= 2 * k_scale
                    xyzs_c = torch.cat((xyzs_c, torch.ones_like(xyzs_c)[:, :1, :]), 1)
                    xyz_clip = M_ndc_from_cam @ xyzs_c
                    xyz_ndc = xyz_clip / xyz_clip[:, 3:]
                    uvd = M_uv_from_ndc @ xyz_ndc
                    uv = uvd[:, :2]
                in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < img_wh[0]) & (uv[:, 1] >= 0) & \
                           (uv[:, 1] < img_wh[1])
                covered_by_cam = (uvd[:, 2] >= near_distance) & in_image
                self.count_grid[c, indices[i:i + chunk]] = count = covered_by_cam.sum(0) / N_cams
                too_near_to_cam = (uvd[:, 2] < near_distance) & in_image
                valid_mask = (count > 0) & (~too_near_to_cam.any(0))
                self.density_grid[c, indices[i:i + chunk]] = torch.where(valid_mask, 0., -1.)

    def _grid_side_stream(self):
        if getattr(self, "_grid_side", None) is None:
            self._grid_side = torch.cuda.Stream(device=self.density_grid.device)
        return self._grid_side

    def _grid_ws(self):
        """Device workspace of the grid refresh: hit list (positions, cell indices, densities) of one
        cascade's capacity, the list count, the effective threshold and the reduction scratch."""
        dev, N = self.density_grid.device, self.grid_size ** 3
        ws = getattr(self, "_gws", None)
        if ws is None or ws["xyzs"].device != dev or ws["idx"].numel() != N:
            nbytes = int(_lib.lib().ncn_grid_work_bytes())
            ws = {"xyzs": torch.empty(N, 3, device=dev), "idx": torch.empty(N, dtype=torch.int32, device=dev),
                  "sigmas": torch.empty(N, device=dev), "scal": torch.zeros(4, dtype=torch.int32, device=dev),
                  # the density pass's encodings (ncn_field_fwd mode 2 scratch: 64 B per point)
                  "enc": torch.empty(((N + 15) // 16) * 16 * ENC_BYTES // 2, dtype=torch.float16, device=dev),
                  "work": torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=dev)}
            self._gws = ws
        return ws

    @torch.no_grad()
    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=False, seed=None, beside=None):
        """ngp_mt.py:340-368 on the device (csrc/grid.hip): per cascade ncn_grid_sample -> density
        pass (ncn_field_fwd mode 2 over the hit list, device count) -> ncn_grid_apply, then
        ncn_grid_packbits.  Cells hit: all of them in warmup (get_all_cells), else each cell with the
        marginal probability of the reference's M uniform + M occupied draws with replacement
        (sample_uniform_and_occupied_cells, M = G^3/4) — the documented sampling deviation of
        grid.hip.  The density grid is updated in place (the reference rebinds it to the same values).
        Quirk q12: with no cell > 0 the mean is NaN and the bitfield is cleared — reproduced.
        No host synchronisation; `seed` (default: drawn from torch's CPU generator) fixes the draw.
        beside (optional callable): work issued on the current stream while the first cascade's cell
        sampling — which reads the density grid only, not the parameters — runs on a side stream
        (Trainer: the optimizer step the refresh waits for); joined before the density pass."""
        G, C = self.grid_size, self.cascades
        N = G ** 3
        dg = self.density_grid
        if not (dg.is_cuda and dg.is_contiguous() and dg.dtype == torch.float32 and dg.shape == (C, N)):
            raise RuntimeError("density_grid must be a contiguous CUDA float32 (cascades, grid_size**3) tensor")
        cnt = None
        if erode:
            cnt = self.count_grid.float().contiguous()
        ws = self._grid_ws()
        n_list = ws["scal"][0:1]
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        table = self.xyz_encoder.params
        packed = None
        for c in range(C):
            s = min(2 ** (c - 1), self.scale)
            half_grid_size = s / G
            dgc = dg[c]
            cc = cnt[c] if cnt is not None else None

            def sample():
                call("ncn_grid_sample", ptr(dgc), I64(N), I32(G), F32(s - half_grid_size), F32(half_grid_size),
                     F32(density_threshold), I64(N // 4), I32(1 if warmup else 0),
                     _lib.U64((seed + 0x9E3779B97F4A7C15 * c) % 2 ** 64), F32(decay), ptr(cc), ptr(ws["xyzs"]),
                     ptr(ws["idx"]), ptr(n_list), ptr(ws["work"]), stream())

            if c == 0 and beside is not None:
                cur = torch.cuda.current_stream(dg.device)
                side = self._grid_side_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    sample()
                beside()
                cur.wait_stream(side)
            else:
                sample()
            if packed is None:
                packed = self._take_packed()  # (after `beside`: the optimizer may have refreshed the fragments)
            # density pass, mode 2: the hash-grid encoding split by level over the XCDs into the
            # scratch ws["enc"] (each L2 serves two levels' tables), then sigma_net from it
            call("ncn_field_fwd", ptr(ws["xyzs"]), ptr(None), I64(N), ptr(n_list), ptr(None), ptr(table), self._levels_ptr,
                 F32(self._xyz_min), F32(self._xyz_extent), ptr(packed), I32(self._prec), I32(2), ptr(ws["sigmas"]), ptr(None),
                 ptr(ws["enc"]), stream())
            call("ncn_grid_apply", ptr(dgc), ptr(ws["idx"]), ptr(ws["sigmas"]), ptr(n_list), I64(N), F32(decay),
                 ptr(cc), stream())
        thr_out = ws["scal"][1:2].view(torch.float32)
        call("ncn_grid_packbits", ptr(dg), I64(C * N), _lib.F64(density_threshold), ptr(self.density_bitfield),
             ptr(thr_out), ptr(ws["work"]), stream())


def register_grid_buffers(model):
    """What train_nerf.py:153-157 does: density_grid (C, G^3) and grid_coords (G^3, 3) buffers."""
    G = model.grid_size
    model.register_buffer("density_grid", torch.zeros(model.cascades, G ** 3, device=model.center.device))
    r = torch.arange(G, dtype=torch.int32, device=model.center.device)
    zz, yy, xx = torch.meshgrid(r, r, r, indexing="ij")  # kornia create_meshgrid3d: index (d,h,w) -> (w,h,d)
    coords = torch.stack([xx, yy, zz], -1).reshape(-1, 3)
    model.register_buffer("grid_coords", coords.contiguous())
    return model
