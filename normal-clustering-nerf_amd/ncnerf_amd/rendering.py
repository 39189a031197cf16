"""render() of the reference models/rendering.py:9-242 on the HIP kernels.

Same signature `render(model, rays_o, rays_d, **kwargs)`, same kwargs (near_distance, test_time,
exp_step_factor, max_samples, T_threshold, anneal_*, random_bg, to_cpu/to_numpy, ...) and the same
output dict, including the reference quirks that downstream losses depend on:
  * results['rays_o'] = rays_d  (rendering.py:226-227, quirk q1)
  * white background when exp_step_factor == 0 (rendering.py:232-240, quirk q2)
Removed: the dead `(rays_a[:,2]==0).any()` host sync (rendering.py:195-196).
Extensions (not in the reference): kwargs['march_noise'] injects the marcher noise (test hook);
kwargs['static_shapes']=True keeps every shape independent of the marched sample count (no host
read of the counter), which is what lets Trainer capture the whole step in one HIP graph;
kwargs['premarched'] (a march_train_static() result) skips intersect + march: the pipelined step
marches the next batch while the current one is rendered.
"""
import time

import torch
from einops import rearrange

from .custom_functions import CountJob, RayAABBIntersector, RayMarcher, VolumeRenderer, VolumeRendererBg
from . import _lib, vren


@torch.autocast("cuda")
def render(model, rays_o, rays_d, **kwargs):
    """rendering.py:9-42"""
    near_distance = kwargs["near_distance"]
    rays_o = rays_o.contiguous()
    rays_d = rays_d.contiguous()
    if kwargs.get("premarched") is not None and not kwargs.get("test_time", False):
        return render_rays_train(model, rays_o, rays_d, None, **kwargs)
    if _fused_march_ok(model, kwargs, rays_o.shape[0]):  # intersect + jitter + march + scan + pack in one launch
        kwargs["premarched"] = march_train_fused(model, rays_o, rays_d, near_distance, kwargs["max_samples"],
                                                 kwargs.get("march_noise"), kwargs.get("march_rng"))
        return render_rays_train(model, rays_o, rays_d, None, **kwargs)
    # RayAABBIntersector (no gradient) + the near clamp of rendering.py:28 in one kernel
    _, hits_t, _ = vren.ray_aabb_intersect(rays_o.float(), rays_d.float(), model.center, model.half_size, 1,
                                           near_distance=near_distance)
    render_func = render_rays_test if kwargs.get("test_time", False) else render_rays_train
    results = render_func(model, rays_o, rays_d, hits_t, **kwargs)
    for k, v in results.items():
        if kwargs.get("to_cpu", False):
            v = v.cpu()
            if kwargs.get("to_numpy", False):
                v = v.numpy()
        results[k] = v
    return results


@torch.no_grad()
def render_rays_test(model, rays_o, rays_d, hits_t, **kwargs):
    """rendering.py:45-149: host-driven incremental march/composite of the alive rays."""
    exp_step_factor = kwargs.get("exp_step_factor", 0.0)
    max_samples = kwargs["max_samples"]
    results = {}
    N_rays = len(rays_o)
    device = rays_o.device
    opacity = torch.zeros(N_rays, device=device)
    depth = torch.zeros(N_rays, device=device)
    rend_l = 3 + (3 if model.pred_norm else 0) + (kwargs["n_sem_cls"] if model.pred_sem else 0)
    rend = torch.zeros(N_rays, rend_l, device=device)
    samples = total_samples = 0
    alive_indices = torch.arange(N_rays, device=device)
    min_samples = 1 if exp_step_factor == 0 else 4
    hits_t0 = hits_t[:, 0].contiguous()
    stats = kwargs.get("loop_stats")  # (extension) iteration count and host time blocked at the syncs
    # Fused iteration (default; kwargs test_fused=False keeps the reference's structure): a ray's
    # valid samples are its first N_eff of the marcher's N_samples slots, so one kernel compacts
    # them (ncn_test_compact: per-ray offsets + a device count), the field runs on that device count
    # and the compositor reads through the offsets — the valid mask, its host-synced count, the
    # masked gathers and the scatter back into zero-filled sigmas / rgbs are gone; outputs are
    # bit-identical (the field's arithmetic is per sample).  An all-invalid round composites nothing
    # and retires every ray instead of breaking out of the loop: the loop ends one round later with
    # the same outputs.
    mode = kwargs.get("test_fused", True)
    fused = bool(mode) and not model.pred_norm and not model.pred_sem and hasattr(model, "_field_fwd")
    fwd_kwargs = {k: v for k, v in kwargs.items() if k not in ("loop_stats", "test_fused")}
    if fused and hasattr(model, "prepare_weights"):
        model.prepare_weights()
    if fused and mode is True and N_rays > 0:
        # the same fused iterations driven from the device (no host read per iteration)
        total_samples = _test_loop_device(model, rays_o, rays_d, hits_t0, alive_indices, exp_step_factor, max_samples,
                                          min_samples, float(kwargs.get("T_threshold", 1e-4)), opacity, depth, rend,
                                          stats)
        samples = max_samples  # (loop done)
    while samples < max_samples:
        N_alive = len(alive_indices)
        if N_alive == 0:
            break
        N_samples = max(min(N_rays // N_alive, 64), min_samples)
        samples += N_samples
        xyzs, dirs, deltas, ts, N_eff_samples = vren.raymarching_test(
            rays_o, rays_d, hits_t0, alive_indices, model.density_bitfield, model.cascades, model.scale,
            exp_step_factor, model.grid_size, max_samples, N_samples)
        total_samples += N_eff_samples.sum()
        xyzs = rearrange(xyzs, "n1 n2 c -> (n1 n2) c")
        dirs = rearrange(dirs, "n1 n2 c -> (n1 n2) c")
        if fused:
            if stats is not None:
                stats["iterations"] = stats.get("iterations", 0) + 1
                stats["samples_marched"] = stats.get("samples_marched", 0) + N_alive * N_samples
            if hasattr(model, "prepare_weights"):
                model._packed_fresh = True  # (packed once before the loop: the weights do not change in it)
            # the valid samples compacted on the device (ncn_test_compact), the field on their device
            # count, the compositor through the per-ray offsets
            cap = N_alive * N_samples
            xyz_c = torch.empty(cap, 3, dtype=torch.float32, device=device)
            dir_c = torch.empty(cap, 3, dtype=torch.float32, device=device)
            offs = torch.empty(N_alive, dtype=torch.int32, device=device)
            cnt = torch.empty(1, dtype=torch.int32, device=device)
            _lib.call("ncn_test_compact", _lib.ptr(xyzs), _lib.ptr(dirs), _lib.ptr(N_eff_samples), _lib.I64(N_alive),
                      _lib.I32(N_samples), _lib.ptr(offs), _lib.ptr(xyz_c), _lib.ptr(dir_c), _lib.ptr(cnt),
                      _lib.stream())
            sig, rgb = model._field_fwd(xyz_c, dir_c, cnt, 0, False)[:2]
            _lib.call("ncn_composite_test_fw_compact", _lib.ptr(sig), _lib.ptr(rgb), _lib.ptr(offs), _lib.ptr(deltas),
                      _lib.ptr(ts), _lib.ptr(alive_indices), _lib.I64(N_alive), _lib.I32(N_samples), _lib.I32(3),
                      _lib.F32(float(kwargs.get("T_threshold", 1e-4))), _lib.ptr(N_eff_samples), _lib.ptr(opacity),
                      _lib.ptr(depth), _lib.ptr(rend), _lib.stream())
            if stats is not None:
                t0 = time.perf_counter()
            alive_indices = alive_indices[alive_indices >= 0]  # (host sync: the compaction's size)
            if stats is not None:
                stats["blocked_s"] = stats.get("blocked_s", 0.0) + time.perf_counter() - t0
            continue
        valid_mask = ~torch.all(dirs == 0, dim=1)
        if stats is not None:
            t0 = time.perf_counter()
        if valid_mask.sum() == 0:  # (host sync)
            break
        if stats is not None:
            stats["blocked_s"] = stats.get("blocked_s", 0.0) + time.perf_counter() - t0
            stats["iterations"] = stats.get("iterations", 0) + 1
            stats["samples_marched"] = stats.get("samples_marched", 0) + N_alive * N_samples
        output = model(xyzs[valid_mask], dirs[valid_mask], **fwd_kwargs)
        sigmas = torch.zeros(len(xyzs), device=device)
        sigmas[valid_mask] = output["sigmas"].float()
        sigmas = rearrange(sigmas, "(n1 n2) -> n1 n2", n2=N_samples)
        rgbs = torch.zeros(len(xyzs), 3, device=device)
        rgbs[valid_mask] = output["rgbs"].float()
        raws = rearrange(rgbs, "(n1 n2) c -> n1 n2 c", n2=N_samples)
        for key in (("norms",) if model.pred_norm else ()) + (("sems",) if model.pred_sem else ()):
            extra = torch.zeros(len(xyzs), output[key].shape[1], device=device)
            extra[valid_mask] = output[key].float()
            raws = torch.cat((raws, rearrange(extra, "(n1 n2) c -> n1 n2 c", n2=N_samples)), dim=-1)
        vren.composite_test_multi_fw(sigmas.contiguous(), raws.contiguous(), deltas, ts, hits_t0, alive_indices,
                                     kwargs.get("T_threshold", 1e-4), N_eff_samples, opacity, depth, rend)
        if stats is not None:
            t0 = time.perf_counter()
        alive_indices = alive_indices[alive_indices >= 0]  # (host sync: the compaction's size)
        if stats is not None:
            stats["blocked_s"] += time.perf_counter() - t0
    hits_t[:, 0] = hits_t0
    results["opacity"] = opacity
    results["depth"] = depth
    i = 3
    results["rgb"] = rend[..., :i]
    if model.pred_norm:
        results["norm_nn"] = rend[..., i:i + 3]
        if kwargs.get("pred_norm_nn_norm", False):
            results["norm_nn"] = torch.nn.functional.normalize(results["norm_nn"], p=2.0, dim=-1)
        i += 3
    if model.pred_sem:
        results["sem"] = rend[..., i:i + kwargs["n_sem_cls"]]
    results["total_samples"] = total_samples
    rgb_bg = torch.ones(3, device=device) if exp_step_factor == 0 else torch.zeros(3, device=device)
    results["rgb"] += rgb_bg * rearrange(1 - opacity, "n -> n 1")
    return results


TEST_LOOP_CHECK = 4  # iterations launched between two reads of the device loop's done flag


def _test_loop_device(model, rays_o, rays_d, hits_t0, alive, exp_step_factor, max_samples, min_samples, T_threshold,
                      opacity, depth, rend, stats):
    """render_rays_test's loop (rendering.py:68-105) with the fused iteration, its control on the
    device (ncn_test_loop_*: the alive count, N_samples and the stop test of the loop head formed by
    a kernel after each iteration); the host launches TEST_LOOP_CHECK iterations between reads of the
    done flag (iterations past the end launch empty).  Same outputs as the host-driven loop bit for
    bit: every ray's march and composite are independent of its position in the alive list.  Returns
    total_samples (device int64)."""
    from ._lib import F32, I32, I64, call, ptr, stream
    R, dev = rays_o.shape[0], rays_o.device
    cap = R * min_samples
    f = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)  # noqa: E731
    xyzs, dirs, deltas, ts = f(cap, 3), f(cap, 3), f(cap), f(cap)
    sig, rgb = f(cap), f(cap, 3)
    n_eff = torch.empty(R, dtype=torch.int32, device=dev)
    idx = torch.empty(cap, dtype=torch.int32, device=dev)
    model._packed_fresh = True
    packed = model._take_packed()  # (packed before the loop: the weights do not change in it)
    bufs = [alive, torch.empty(R, dtype=torch.int64, device=dev)]
    # the loop head's N_samples = max(min(N_rays // N_alive, 64), min_samples) (rendering.py:69-70); on
    # the first iteration N_alive == N_rays, so it is max(1, min_samples); test_loop_next forms the rest
    ns0 = max(1, min_samples)
    ctrl = torch.tensor([R, ns0, ns0, 0, 0, 0, 0, 0], dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    count = ctrl[4:5]
    it = 0
    blocked = 0.0
    while it <= max_samples:  # (every iteration adds >= 1 to samples: at most max_samples run)
        for _ in range(TEST_LOOP_CHECK):
            a, b = bufs[it % 2], bufs[(it + 1) % 2]
            call("ncn_test_loop_march", ptr(rays_o), ptr(rays_d), ptr(hits_t0), ptr(a), I64(R), ptr(model.density_bitfield),
                 I32(int(model.cascades)), F32(float(model.scale)), F32(float(exp_step_factor)), I32(int(model.grid_size)),
                 I32(int(max_samples)), ptr(ctrl), ptr(xyzs), ptr(dirs), ptr(deltas), ptr(ts), ptr(n_eff), stream())
            call("ncn_test_loop_index", ptr(n_eff), I64(R), ptr(ctrl), ptr(idx), stream())
            # the field on exactly the valid slots (order = their indices, count on the device)
            call("ncn_field_fwd", ptr(xyzs), ptr(dirs), I64(cap), ptr(count), ptr(idx), ptr(model.xyz_encoder.params),
                 model._levels_ptr, F32(model._xyz_min), F32(model._xyz_extent), ptr(packed), I32(model._prec), I32(0),
                 ptr(sig), ptr(rgb), ptr(None), stream())
            call("ncn_test_loop_composite", ptr(sig), ptr(rgb), ptr(None), ptr(deltas), ptr(ts), ptr(a), I64(R),
                 ptr(ctrl), I32(3), F32(T_threshold), ptr(n_eff), ptr(opacity), ptr(depth), ptr(rend), stream())
            call("ncn_test_loop_next", ptr(a), ptr(b), I64(R), ptr(ctrl), ptr(total), I32(R), I32(int(max_samples)),
                 I32(int(min_samples)), stream())
            it += 1
        t0 = time.perf_counter()
        done = bool(ctrl[3].item())  # (host sync)
        blocked += time.perf_counter() - t0
        if done:
            break
    if stats is not None:
        c = ctrl.tolist()
        stats["iterations"] = stats.get("iterations", 0) + c[6]
        stats["samples_marched"] = stats.get("samples_marched", 0) + c[7]
        stats["blocked_s"] = stats.get("blocked_s", 0.0) + blocked
        stats["launched_iterations"] = stats.get("launched_iterations", 0) + it
    return total[0]


def render_rays_train(model, rays_o, rays_d, hits_t, **kwargs):
    """rendering.py:152-242"""
    exp_step_factor = kwargs.get("exp_step_factor", 0.0)
    max_samples = kwargs["max_samples"]
    results = {}
    anneal_step = kwargs.get("anneal_steps", 0)
    global_step = kwargs.get("global_step", anneal_step)
    if anneal_step > global_step:  # rendering.py:168-188
        strategy = kwargs.get("anneal_strategy", "none")
        if strategy == "avoid_near":
            ps = 0.5
            ray_mid = (hits_t[:, 0, 0] + hits_t[:, 0, 1]) / 2.0
            n_i = min(max(global_step / anneal_step, ps), 1.0)
            hits_t[:, 0, 0] = ray_mid + n_i * (hits_t[:, 0, 0] - ray_mid)
        elif strategy == "depth":
            depth = kwargs["depth"]
            n_i = min(max(global_step / anneal_step, 0.05), 100.0)
            hits_t[:, 0, 0] = torch.max(depth + n_i * (hits_t[:, 0, 0] - depth), hits_t[:, 0, 0])
            hits_t[:, 0, 1] = torch.min(depth + n_i * (hits_t[:, 0, 1] - depth), hits_t[:, 0, 1])
        else:
            assert strategy == "none"
    if hasattr(model, "prepare_weights") and not getattr(model, "_packed_fresh", False):
        model.prepare_weights()  # queue the fp16 weight packing ahead of the marcher's host read of S
    static = bool(kwargs.get("static_shapes", False))
    pm = kwargs.get("premarched")
    if pm is not None:  # marched ahead (march_train_static): same tensors RayMarcher would return
        static = True
        rays_a, xyzs, dirs, results["deltas"], results["ts"], results["rm_samples"] = (
            pm["rays_a"], pm["xyzs"], pm["dirs"], pm["deltas"], pm["ts"], pm["counter"][0])
    else:
        rays_a, xyzs, dirs, results["deltas"], results["ts"], results["rm_samples"] = RayMarcher.apply(
            rays_o, rays_d, hits_t[:, 0], model.density_bitfield, model.cascades, model.scale, exp_step_factor,
            model.grid_size, max_samples, kwargs.get("march_noise"), static)
    for k, v in list(kwargs.items()):  # rendering.py:198-200
        if isinstance(v, torch.Tensor) and k not in ("march_noise", "premarched", "march_rng", "count_acc"):
            if static:
                raise NotImplementedError(f"per-ray tensor kwarg {k!r} on the static-shape path")
            kwargs[k] = torch.repeat_interleave(v[rays_a[:, 0]], rays_a[:, 2], 0)
    if static:  # capacity-sized sample arrays; the field stops at the device count
        kwargs["n_samples_dev"] = results["rm_samples"]
    output = model(xyzs, dirs, **kwargs)
    sigmas = output["sigmas"]
    raws = output["rgbs"]
    if model.pred_norm:
        raws = torch.cat((raws, output["norms"]), dim=-1)
    if model.pred_sem:
        raws = torch.cat((raws, output["sems"]), dim=-1)
    fuse_bg = exp_step_factor == 0 and raws.shape[1] == 3  # white background, rgb only
    renderer = VolumeRendererBg if fuse_bg else VolumeRenderer
    extra = (1.0,) if fuse_bg else ()
    job = CountJob() if fuse_bg and kwargs.get("count_in_loss") else None
    if fuse_bg and (kwargs.get("count_acc") is not None or job is not None):
        # (extension) device-side throughput counters; count_in_loss: the sample count is taken by
        # the loss node's first launch (results["_count_job"]; the caller runs NeRFMTLoss)
        rm = results["rm_samples"]
        rm = rm if isinstance(rm, torch.Tensor) and rm.dtype == torch.int32 and rm.is_cuda else None
        acc = kwargs.get("count_acc")
        extra = (1.0, (rm if acc is not None else None, acc, job))
    (results["vr_samples"], results["opacity"], results["depth"], rend, results["ws"]) = renderer.apply(
        sigmas, raws.contiguous(), results["deltas"], results["ts"], rays_a, kwargs.get("T_threshold", 1e-4), *extra)
    if job is not None and job.out is not None:
        results["_count_job"] = job
    i = 3
    results["rgb"] = rend if rend.shape[-1] == i else rend[..., :i]  # no slice node for rgb-only
    if model.pred_norm:
        results["norm_nn"] = rend[..., i:i + 3]
        if kwargs.get("pred_norm_nn_norm", False):
            results["norm_nn"] = torch.nn.functional.normalize(results["norm_nn"], p=2.0, dim=-1)
        i += 3
    if model.pred_sem:
        results["sem"] = rend[..., i:i + kwargs["n_sem_cls"]]
    results["rays_d"] = rays_d
    results["rays_o"] = rays_d  # rendering.py:227 (quirk q1)
    results["rays_a"] = rays_a
    results["depth_std"] = _ones(results["depth"])  # rendering.py:230 (constant: cached, no fill per call)
    if exp_step_factor == 0:  # white: rgb + 1 * (1 - opacity), fused into the compositor when rgb-only
        if not fuse_bg:
            results["rgb"] = results["rgb"] + (1 - results["opacity"])[:, None]
        return results
    if kwargs.get("random_bg", False):
        rgb_bg = torch.rand(3, device=rays_o.device)
    else:
        rgb_bg = torch.zeros(3, device=rays_o.device)
    results["rgb"] = results["rgb"] + rgb_bg * rearrange(1 - results["opacity"], "n -> n 1")
    return results


_ONES = {}


def _ones(like):
    """A cached all-ones tensor shaped like `like` (read-only by convention)."""
    key = (tuple(like.shape), like.dtype, like.device)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(like.shape, dtype=like.dtype, device=like.device)
    return t


def _fused_march_ok(model, kw, n_rays):
    """The one-launch marcher serves the static-shape training path at constant dt (the configs'
    exp_step_factor == 0) without ray-range annealing or per-ray tensor kwargs."""
    return (kw.get("static_shapes", False) and not kw.get("test_time", False)
            and kw.get("exp_step_factor", 0.0) == 0 and kw.get("anneal_strategy", "none") == "none"
            and getattr(model, "_aabb", None) is not None and n_rays <= 16384
            and not any(isinstance(v, torch.Tensor) for k, v in kw.items()
                        if k not in ("march_noise", "march_rng", "count_acc")))


@torch.no_grad()
def march_train_fused(model, rays_o, rays_d, near_distance, max_samples, noise=None, rng=None, out=None):
    """ncn_march_train_fused: RayAABBIntersector + near clamp (rendering.py:24-28) + RayMarcher
    (custom_functions.py:79-100) in two launches -> {'rays_a', 'xyzs', 'dirs', 'deltas', 'ts', 'counter'}
    with capacity-sized sample arrays (device count counter[0]).  noise: (R,) jitter, else
    rng = (seed, int64 device counter) draws it on the device (graph replays advance the counter),
    else torch.rand_like as the reference (custom_functions.py:83).  out: a previous result (or
    march_buffers()) whose tensors are overwritten in place; its '_slab' scratch is reused."""
    from ._lib import F32, I32, I64, U64, call, check_input, lib, ptr, stream
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    check_input(rays_o, "rays_o")
    check_input(rays_d, "rays_d")
    R, dev, ms = rays_o.shape[0], rays_o.device, int(max_samples)
    cap = R * ms
    if out is None:
        out = march_buffers(R, ms, dev)
    seed, ctr = 0, None
    if noise is not None:
        noise = noise.contiguous().float()
        check_input(noise, "noise")
    elif rng is not None:
        seed, ctr = rng
    else:
        noise = torch.rand_like(rays_o[:, 0])  # custom_functions.py:83
    if out["xyzs"].shape[0] != cap or out["rays_a"].shape[0] != R:
        raise RuntimeError("march_train_fused: out= buffers are sized for another batch")
    slab_xyz, slab_t, slab_dt, ws = out["_slab"]
    c, h = model._aabb
    call("ncn_march_train_fused", ptr(rays_o), ptr(rays_d), I64(R), F32(c[0]), F32(c[1]), F32(c[2]), F32(h[0]),
         F32(h[1]), F32(h[2]), F32(near_distance), ptr(noise), U64(int(seed) % 2 ** 64), ptr(ctr),
         ptr(model.density_bitfield), I32(int(model.cascades)), F32(float(model.scale)), I32(int(model.grid_size)),
         I32(ms), ptr(slab_xyz), ptr(slab_t), ptr(slab_dt), ptr(ws), ptr(out["rays_a"]), ptr(out["xyzs"]),
         ptr(out["dirs"]), ptr(out["deltas"]), ptr(out["ts"]), ptr(out["counter"]), stream())
    return out


def march_buffers(R, max_samples, device, share_scratch=None):
    """Output + scratch buffers of march_train_fused for R rays (capacity R*max_samples samples);
    share_scratch: another march_buffers() whose scratch (slabs, work) is reused (never concurrently)."""
    from ._lib import I64, lib
    cap = R * int(max_samples)
    f = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=device)
    if share_scratch is not None:
        scratch = share_scratch["_slab"]
    else:
        ws = torch.empty((int(lib().ncn_march_train_fused_work_bytes(I64(R))) + 3) // 4, dtype=torch.int32,
                         device=device)
        scratch = (f(cap * 3), f(cap), f(cap), ws)
    out = {"rays_a": torch.empty(R, 3, dtype=torch.int64, device=device), "xyzs": f(cap, 3), "dirs": f(cap, 3),
           "deltas": f(cap), "ts": f(cap), "counter": torch.empty(2, dtype=torch.int32, device=device),
           "_slab": scratch}
    return out



@torch.no_grad()
def march_train_static(model, rays_o, rays_d, out=None, **kwargs):
    """The intersect + march part of render_rays_train on the static-shape path (rendering.py:24-28,
    190-197) as a standalone stage: returns {'rays_a', 'xyzs', 'dirs', 'deltas', 'ts', 'counter'}
    (capacity-sized sample arrays, device count in counter[0]) for render(..., premarched=...).
    out: a previous result whose tensors are overwritten in place (fixed buffers for graphs)."""
    exp_step_factor = kwargs.get("exp_step_factor", 0.0)
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    _, hits_t, _ = vren.ray_aabb_intersect(rays_o, rays_d, model.center, model.half_size, 1,
                                           near_distance=kwargs["near_distance"])
    noise = kwargs.get("march_noise")
    if noise is None:
        noise = torch.rand_like(rays_o[:, 0])  # custom_functions.py:83
    keys = ("rays_a", "xyzs", "dirs", "deltas", "ts", "counter")
    res = vren.raymarching_train(rays_o, rays_d, hits_t[:, 0].contiguous(), model.density_bitfield, model.cascades,
                                 model.scale, exp_step_factor, noise.contiguous(), model.grid_size,
                                 kwargs["max_samples"], static_capacity=True,
                                 out=None if out is None else [out[k] for k in keys])
    return dict(zip(keys, res))
