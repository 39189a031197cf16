"""Drop-in replacement of the reference `vren` extension (models/csrc/binding.cpp:330-349) for the
training hot path, backed by libncnerf.so (gfx950 HIP kernels, C ABI in include/ncnerf.h).

Same function names, argument order and meaning, return structure (lists of newly allocated
tensors; `packbits`, `raymarching_test` and `composite_test_multi_fw` mutate their documented
in-place arguments) and error behaviour: every tensor argument is checked `is_cuda and
is_contiguous` exactly like CHECK_INPUT (models/csrc/include/utils.h:4-6) and a failure raises
RuntimeError.  Kernels run on torch's current stream.

Deliberate differences (DESIGN.md "Parity contract"):
  * `raymarching_train` returns sample tensors sized exactly S = counter[0] instead of
    R*max_samples rows (callers slice by counter[0], custom_functions.py:91-96, so slicing is a
    no-op), and `rays_a` is in ray order (the reference's order comes from atomicAdd).
  * dead-code entry points of the reference (ray_sphere_intersect, the rgb-only composite
    variants) are not provided.
"""
import torch

from . import _lib
from ._lib import F32, I32, I64, call, check_dtype, check_input, ptr, stream


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits, near_distance=None):
    """intersection.cu:59-100 -> [hit_cnt i32 (R), hits_t f32 (R,M,2), hits_voxel_idx i64 (R,M)]
    Extension: near_distance applies render()'s clamp of the first hit (rendering.py:28) in-kernel."""
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (centers, "centers"), (half_sizes, "half_sizes")):
        check_input(t, n)
        check_dtype(t, torch.float32, n)
    R, V = rays_o.shape[0], centers.shape[0]
    dev = rays_o.device
    hit_cnt = torch.empty(R, dtype=torch.int32, device=dev)
    hits_t = torch.empty(R, max_hits, 2, dtype=torch.float32, device=dev)
    hits_idx = torch.empty(R, max_hits, dtype=torch.int64, device=dev)
    if near_distance is None:
        call("ncn_ray_aabb_intersect", ptr(rays_o), ptr(rays_d), I64(R), ptr(centers), ptr(half_sizes), I64(V),
             I32(max_hits), ptr(hit_cnt), ptr(hits_t), ptr(hits_idx), stream())
    else:
        call("ncn_ray_aabb_intersect_near", ptr(rays_o), ptr(rays_d), I64(R), ptr(centers), ptr(half_sizes), I64(V),
             I32(max_hits), F32(float(near_distance)), ptr(hit_cnt), ptr(hits_t), ptr(hits_idx), stream())
    return [hit_cnt, hits_t, hits_idx]


def morton3D(coords):
    """raymarching.cu:72-88"""
    check_input(coords, "coords")
    check_dtype(coords, torch.int32, "coords")
    out = torch.empty(coords.shape[0], dtype=torch.int32, device=coords.device)
    call("ncn_morton3D", ptr(coords), I64(coords.shape[0]), ptr(out), stream())
    return out


def morton3D_invert(indices):
    """raymarching.cu:103-119"""
    check_input(indices, "indices")
    check_dtype(indices, torch.int32, "indices")
    out = torch.empty(indices.shape[0], 3, dtype=torch.int32, device=indices.device)
    call("ncn_morton3D_invert", ptr(indices), I64(indices.shape[0]), ptr(out), stream())
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    """raymarching.cu:143-161 (in place on density_bitfield)"""
    check_input(density_grid, "density_grid")
    check_input(density_bitfield, "density_bitfield")
    check_dtype(density_grid, torch.float32, "density_grid")
    n = density_bitfield.shape[0]
    if density_grid.numel() < 8 * n:
        raise RuntimeError("density_grid has fewer than 8*len(density_bitfield) cells")
    call("ncn_packbits", ptr(density_grid), I64(n), F32(float(density_threshold)), ptr(density_bitfield), stream())


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples, static_capacity=False, out=None):
    """raymarching.cu:283-332 -> [rays_a i64 (R,3), xyzs (S,3), dirs (S,3), deltas (S), ts (S), counter i32 (2)].

    Walk -> scan -> (read S, the reference's own sync point custom_functions.py:91) -> pack.
    static_capacity=True (extension): the host never reads S; the sample arrays have the capacity
    R*max_samples, rows >= counter[0] are unspecified, and consumers take counter[0:1] as the
    device-resident count (the graph-captured training step).  out (static_capacity only): the six
    output tensors to write instead of allocating them (the pipelined step's fixed buffers)."""
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (hits_t, "hits_t"), (density_bitfield, "density_bitfield"),
                 (noise, "noise")):
        check_input(t, n)
    R = rays_o.shape[0]
    dev = rays_o.device
    ms = int(max_samples)
    s = stream()
    counts = torch.empty(R, dtype=torch.int32, device=dev)
    slab_xyz = torch.empty(R * ms * 3, dtype=torch.float32, device=dev)
    slab_t = torch.empty(R * ms, dtype=torch.float32, device=dev)
    slab_dt = torch.empty(R * ms, dtype=torch.float32, device=dev)
    if out is not None and not static_capacity:
        raise ValueError("out= needs static_capacity=True")
    rays_a = out[0] if out is not None else torch.empty(R, 3, dtype=torch.int64, device=dev)
    counter = out[5] if out is not None else torch.empty(2, dtype=torch.int32, device=dev)
    call("ncn_march_train_walk", ptr(rays_o), ptr(rays_d), ptr(hits_t), ptr(noise), I64(R), ptr(density_bitfield),
         I32(int(cascades)), F32(float(scale)), F32(float(exp_step_factor)), I32(int(grid_size)), I32(ms),
         ptr(counts), ptr(slab_xyz), ptr(slab_t), ptr(slab_dt), s)
    call("ncn_march_train_scan", ptr(counts), I64(R), ptr(rays_a), ptr(counter), s)
    S = R * ms if static_capacity else int(counter[0].item())
    if out is not None:
        xyzs, dirs, deltas, ts = out[1:5]
        if xyzs.shape[0] != S or dirs.shape[0] != S or deltas.shape[0] != S or ts.shape[0] != S:
            raise RuntimeError("raymarching_train: out= buffers must hold R*max_samples samples")
    else:
        xyzs = torch.empty(S, 3, dtype=torch.float32, device=dev)
        dirs = torch.empty(S, 3, dtype=torch.float32, device=dev)
        deltas = torch.empty(S, dtype=torch.float32, device=dev)
        ts = torch.empty(S, dtype=torch.float32, device=dev)
    call("ncn_march_train_pack", ptr(rays_d), ptr(rays_a), I64(R), I32(ms), ptr(slab_xyz), ptr(slab_t),
         ptr(slab_dt), ptr(xyzs), ptr(dirs), ptr(deltas), ptr(ts), s)
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def raymarching_train_backward(dL_dxyzs, dL_ddirs, ts, rays_a):
    """RayMarcher.backward (custom_functions.py:102-112) -> [dL_drays_o (R,3), dL_drays_d (R,3)]: the
    reference's segment_csr over indptr = [rays_a[:,1], rays_a[-1,1] + rays_a[-1,2]] in one launch
    (ncn_segment_csr; fixed summation order, bit-identical run to run).  dL_dxyzs / dL_ddirs may be
    None (zero)."""
    check_input(ts, "ts")
    check_input(rays_a, "rays_a")
    check_dtype(ts, torch.float32, "ts")
    check_dtype(rays_a, torch.int64, "rays_a")
    S = ts.shape[0]
    for t, n in ((dL_dxyzs, "dL_dxyzs"), (dL_ddirs, "dL_ddirs")):
        if t is not None:
            check_input(t, n)
            check_dtype(t, torch.float32, n)
            if t.shape != (S, 3):
                raise RuntimeError(f"{n} must be (S, 3) with S = ts.shape[0] = {S} (got {tuple(t.shape)})")
    R = rays_a.shape[0]
    d_o = torch.empty(R, 3, dtype=torch.float32, device=ts.device)
    d_d = torch.empty(R, 3, dtype=torch.float32, device=ts.device)
    if R:
        # every segment end is another row's start or the last row's start + count: all must lie in [0, S]
        st = rays_a[:, 1]
        lo, hi = int(st.min()), max(int(st.max()), int(rays_a[-1, 1] + rays_a[-1, 2]))
        if lo < 0 or hi > S:
            raise RuntimeError(f"rays_a segments reach outside the {S} samples ([{lo}, {hi}))")
    call("ncn_segment_csr", ptr(dL_dxyzs), ptr(dL_ddirs), ptr(ts), ptr(rays_a), I64(R), ptr(d_o), ptr(d_d), stream())
    return [d_o, d_d]


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale, exp_step_factor,
                     grid_size, max_samples, N_samples):
    """raymarching.cu:407-454 -> [xyzs (A,N,3), dirs (A,N,3), deltas (A,N), ts (A,N), N_eff i32 (A)];
    mutates hits_t[:,0] of the marched rays."""
    for t, n in ((rays_o, "rays_o"), (rays_d, "rays_d"), (hits_t, "hits_t"), (alive_indices, "alive_indices"),
                 (density_bitfield, "density_bitfield")):
        check_input(t, n)
    A, N = alive_indices.shape[0], int(N_samples)
    dev = rays_o.device
    xyzs = torch.empty(A, N, 3, dtype=torch.float32, device=dev)
    dirs = torch.empty(A, N, 3, dtype=torch.float32, device=dev)
    deltas = torch.empty(A, N, dtype=torch.float32, device=dev)
    ts = torch.empty(A, N, dtype=torch.float32, device=dev)
    n_eff = torch.empty(A, dtype=torch.int32, device=dev)
    call("ncn_march_test", ptr(rays_o), ptr(rays_d), ptr(hits_t), ptr(alive_indices), I64(A), ptr(density_bitfield),
         I32(int(cascades)), F32(float(scale)), F32(float(exp_step_factor)), I32(int(grid_size)),
         I32(int(max_samples)), I32(N), ptr(xyzs), ptr(dirs), ptr(deltas), ptr(ts), ptr(n_eff), stream())
    return [xyzs, dirs, deltas, ts, n_eff]


def count_samples(total_samples, counter=None, acc=None):
    """total_samples.sum() (int64 scalar tensor) in one kernel (ncn_count_samples); with acc (a device
    float64 (2,) tensor) also acc += (counter[0], the sum): throughput counters kept on the device."""
    check_input(total_samples, "total_samples")
    out = torch.empty((), dtype=torch.int64, device=total_samples.device)
    call("ncn_count_samples", ptr(total_samples), I64(total_samples.shape[0]), ptr(counter), ptr(out), ptr(acc),
         stream())
    return out


def composite_train_multi_fw(sigmas, raws, deltas, ts, rays_a, T_threshold, bg=None):
    """volumerendering.cu:140-176 -> [total_samples i64 (R), opacity (R), depth (R), rend (R,C), ws (S)]
    Extension: bg (float) also returns rgb_bg = rend + bg * (1 - opacity) as a sixth output."""
    for t, n in ((sigmas, "sigmas"), (raws, "raws"), (deltas, "deltas"), (ts, "ts"), (rays_a, "rays_a")):
        check_input(t, n)
    R, S, C = rays_a.shape[0], sigmas.shape[0], raws.shape[1]
    dev = sigmas.device
    total = torch.empty(R, dtype=torch.int64, device=dev)
    opacity = torch.empty(R, dtype=torch.float32, device=dev)
    depth = torch.empty(R, dtype=torch.float32, device=dev)
    rend = torch.empty(R, C, dtype=torch.float32, device=dev)
    ws = torch.empty(S, dtype=torch.float32, device=dev)
    if bg is None:
        call("ncn_composite_train_fw", ptr(sigmas), ptr(raws), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S),
             I32(C), F32(float(T_threshold)), ptr(total), ptr(opacity), ptr(depth), ptr(rend), ptr(ws), stream())
        return [total, opacity, depth, rend, ws]
    rgb_bg = torch.empty(R, C, dtype=torch.float32, device=dev)
    call("ncn_composite_train_fw_bg", ptr(sigmas), ptr(raws), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S),
         I32(C), F32(float(T_threshold)), ptr(total), ptr(opacity), ptr(depth), ptr(rend), ptr(ws), F32(float(bg)),
         ptr(rgb_bg), stream())
    return [total, opacity, depth, rend, ws, rgb_bg]


def composite_train_multi_bw(dL_dopacity, dL_ddepth, dL_drend, dL_dws, sigmas, raws, ws, deltas, ts, rays_a,
                             opacity, depth, rend, T_threshold, bg=None):
    """volumerendering.cu:367-418 -> [dL_dsigmas (S), dL_draws (S,C)].
    Gradient arguments may also be None (treated as zeros: the kernel then skips those terms).
    Extension: with bg, dL_drend is the gradient of rgb_bg (composite_train_multi_fw(bg=...))."""
    for t, n in ((sigmas, "sigmas"), (raws, "raws"), (ws, "ws"), (deltas, "deltas"), (ts, "ts"),
                 (rays_a, "rays_a"), (opacity, "opacity"), (depth, "depth"), (rend, "rend")):
        check_input(t, n)
    for t, n in ((dL_dopacity, "dL_dopacity"), (dL_ddepth, "dL_ddepth"), (dL_drend, "dL_drend"),
                 (dL_dws, "dL_dws")):
        if t is not None:
            check_input(t, n)
    R, S, C = rays_a.shape[0], sigmas.shape[0], raws.shape[1]
    dsig = torch.empty(S, dtype=torch.float32, device=sigmas.device)
    draws = torch.empty(S, C, dtype=torch.float32, device=sigmas.device)
    if bg is None:
        call("ncn_composite_train_bw", ptr(dL_dopacity), ptr(dL_ddepth), ptr(dL_drend), ptr(dL_dws), ptr(sigmas),
             ptr(raws), ptr(ws), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S), I32(C), ptr(opacity), ptr(depth),
             ptr(rend), F32(float(T_threshold)), ptr(dsig), ptr(draws), stream())
    else:
        call("ncn_composite_train_bw_bg", ptr(dL_dopacity), ptr(dL_ddepth), ptr(dL_drend), ptr(dL_dws), ptr(sigmas),
             ptr(raws), ptr(ws), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), I64(S), I32(C), ptr(opacity), ptr(depth),
             ptr(rend), F32(float(T_threshold)), F32(float(bg)), ptr(dsig), ptr(draws), stream())
    return [dsig, draws]


def composite_test_multi_fw(sigmas, raws, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples, opacity,
                            depth, rend):
    """volumerendering.cu:553-586; in place on alive_indices, opacity, depth, rend."""
    for t, n in ((sigmas, "sigmas"), (raws, "raws"), (deltas, "deltas"), (ts, "ts"), (hits_t, "hits_t"),
                 (alive_indices, "alive_indices"), (N_eff_samples, "N_eff_samples"), (opacity, "opacity"),
                 (depth, "depth"), (rend, "rend")):
        check_input(t, n)
    A, N, C = sigmas.shape[0], sigmas.shape[1], raws.shape[2]
    call("ncn_composite_test_fw", ptr(sigmas), ptr(raws), ptr(deltas), ptr(ts), ptr(alive_indices), I64(A), I32(N),
         I32(C), F32(float(T_threshold)), ptr(N_eff_samples), ptr(opacity), ptr(depth), ptr(rend), stream())


def distortion_loss_fw(ws, deltas, ts, rays_a):
    """losses.cu:69-100 -> [loss (R) by ray_idx, ws_inclusive_scan (S), wts_inclusive_scan (S)]."""
    for t, n in ((ws, "ws"), (deltas, "deltas"), (ts, "ts"), (rays_a, "rays_a")):
        check_input(t, n)
    R, S = rays_a.shape[0], ws.shape[0]
    loss = torch.zeros(R, dtype=torch.float32, device=ws.device)
    wsi = torch.zeros(S, dtype=torch.float32, device=ws.device)
    wtsi = torch.zeros(S, dtype=torch.float32, device=ws.device)
    call("ncn_distortion_loss_fw", ptr(ws), ptr(deltas), ptr(ts), ptr(rays_a), I64(R), ptr(loss), ptr(wsi), ptr(wtsi),
         stream())
    return [loss, wsi, wtsi]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    """losses.cu:143-175 -> dL_dws (S)."""
    for t, n in ((dL_dloss, "dL_dloss"), (ws_inclusive_scan, "ws_inclusive_scan"),
                 (wts_inclusive_scan, "wts_inclusive_scan"), (ws, "ws"), (deltas, "deltas"), (ts, "ts"),
                 (rays_a, "rays_a")):
        check_input(t, n)
    dws = torch.zeros(ws.shape[0], dtype=torch.float32, device=ws.device)
    call("ncn_distortion_loss_bw", ptr(dL_dloss), ptr(ws_inclusive_scan), ptr(wts_inclusive_scan), ptr(ws),
         ptr(deltas), ptr(ts), ptr(rays_a), I64(rays_a.shape[0]), ptr(dws), stream())
    return dws
