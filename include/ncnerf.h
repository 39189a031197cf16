/*
 * ncnerf.h — C ABI of libncnerf.so, the MI355X (gfx950) hot path of the normal-clustering NeRF
 * training step.  Every entry point:
 *   - takes plain device pointers, element counts and a hipStream_t passed as `void*`
 *     (the caller's current stream; never the legacy default stream);
 *   - never allocates, frees or synchronises: buffers are sized by the caller (the one size that
 *     is data dependent — the marched sample count — is produced on device by the count/scan pass
 *     and read back by the caller, exactly where the reference slices by counter[0]);
 *   - returns 0 (hipSuccess) or a hipError_t code; ncn_last_error() returns a message.
 * No torch types cross this boundary.  The Python drop-in (normal-clustering-nerf_amd/ncnerf_amd/
 * vren.py, custom_functions.py, ngp_mt.py, losses.py) binds these with ctypes; INTEGRATION.md shows
 * the binding a maintainer adds on the reference side.
 *
 * Layout conventions: float3 arrays are AoS (N,3) contiguous as in the reference; rays_a is (R,3)
 * int64 (ray_idx, start, n_samples) in RAY ORDER (the reference's atomic order is
 * nondeterministic, raymarching.cu:237-238).
 */
#ifndef NCNERF_H
#define NCNERF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* ncn_last_error(void);
int ncn_version(void);

/* ---- occupancy utilities: replaces vren.morton3D / morton3D_invert / packbits
 *      (binding.cpp:42-72, raymarching.cu:62-161) ---- */
int ncn_morton3D(const int32_t* coords, int64_t n, int32_t* out, void* stream);
int ncn_morton3D_invert(const int32_t* indices, int64_t n, int32_t* coords, void* stream);
int ncn_packbits(const float* density_grid, int64_t n_bytes, float threshold, uint8_t* bitfield, void* stream);

/* ---- distortion loss: replaces vren.distortion_loss_fw / _bw (binding.cpp, losses.cu:47-175;
 *      losses.py:16-44).  fw: loss (R, by ray_idx), ws/wts inclusive scans (S); bw: dL_dws (S) for
 *      every sample of every ray (the caller zero-fills samples outside all rays, as the
 *      reference's torch::zeros). ---- */
int ncn_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                           float* loss, float* ws_inclusive_scan, float* wts_inclusive_scan, void* stream);
int ncn_distortion_loss_bw(const float* dL_dloss, const float* ws_inclusive_scan, const float* wts_inclusive_scan,
                           const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* dL_dws, void* stream);

/* ---- occupancy-grid refresh: replaces NGPMT.update_density_grid (ngp_mt.py:340-368) and its
 *      sample_uniform_and_occupied_cells (ngp_mt.py:245-262) / get_all_cells (:237-243).
 *      Per cascade c: ncn_grid_sample (cells hit: all when warmup, else each cell independently
 *      with the marginal hit probability of M uniform + M occupied draws; the others are decayed
 *      in place) -> ncn_field_fwd(mode 1, n_dev = n_list) over list_xyzs -> ncn_grid_apply; then
 *      ncn_grid_packbits over all cascades (min(mean of positive cells, threshold) -> packbits,
 *      the threshold written to *thr_out).  list_xyzs / list_idx hold n_cells entries; n_list and
 *      thr_out are device scalars; work is ncn_grid_work_bytes() bytes, zero before the first call
 *      (its arrival counter is left zero).  Nothing is read back on the host. ---- */
int64_t ncn_grid_work_bytes(void);
int ncn_grid_sample(float* density_grid_c, int64_t n_cells, int grid_size, float s_minus_half_grid, float half_grid,
                    float threshold, int64_t M, int warmup, uint64_t seed, float decay, const float* count_grid_c,
                    float* list_xyzs, int32_t* list_idx, int32_t* n_list, void* work, void* stream);
int ncn_grid_apply(float* density_grid_c, const int32_t* list_idx, const float* sigmas, const int32_t* n_list,
                   int64_t capacity, float decay, const float* count_grid_c, void* stream);
int ncn_grid_packbits(const float* density_grid, int64_t n_total, double threshold, uint8_t* bitfield,
                      float* thr_out, void* work, void* stream);

/* ---- ray / AABB: replaces vren.ray_aabb_intersect (binding.cpp:12-24, intersection.cu:59-100).
 *      hits_t (R,max_hits,2) and hits_voxel_idx (R,max_hits) are fully written (-1 when empty). ---- */
int ncn_ray_aabb_intersect(const float* rays_o, const float* rays_d, int64_t n_rays,
                           const float* centers, const float* half_sizes, int64_t n_voxels, int max_hits,
                           int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx, void* stream);
/* ray_aabb_intersect with render()'s near clamp fused (rendering.py:28): the first hit's t1 is set
 * to near_distance when it lies in [0, near_distance). */
int ncn_ray_aabb_intersect_near(const float* rays_o, const float* rays_d, int64_t n_rays, const float* centers,
                                const float* half_sizes, int64_t n_voxels, int max_hits, float near_distance,
                                int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx, void* stream);

/* ---- training marcher: replaces vren.raymarching_train (raymarching.cu:283-332).
 * Pass 1 (walk): one walk per ray; samples go to a per-ray slab [R][max_samples] (xyz: 3 floats,
 *   t, dt) and counts[r] = n_samples.  slab_* sized R*max_samples (no zero fill needed).
 * Pass 2 (scan): rays_a[r] = (r, exclusive_scan(counts)[r], counts[r]); counter = {S, R}.
 * Pass 3 (pack): compacts the slab into xyzs (S,3), dirs (S,3), deltas (S), ts (S).
 * hits_t is (R,2) (the caller's hits_t[:,0] view made contiguous). ---- */
int ncn_march_train_walk(const float* rays_o, const float* rays_d, const float* hits_t, const float* noise,
                         int64_t n_rays, const uint8_t* bitfield, int cascades, float scale,
                         float exp_step_factor, int grid_size, int max_samples,
                         int32_t* counts, float* slab_xyz, float* slab_t, float* slab_dt, void* stream);
int ncn_march_train_scan(const int32_t* counts, int64_t n_rays, int64_t* rays_a, int32_t* counter, void* stream);
int ncn_march_train_pack(const float* rays_d, const int64_t* rays_a, int64_t n_rays, int max_samples,
                         const float* slab_xyz, const float* slab_t, const float* slab_dt,
                         float* xyzs, float* dirs, float* deltas, float* ts, void* stream);

/* RayMarcher.backward (custom_functions.py:102-112): torch_scatter.segment_csr (sum) over
 * indptr = [rays_a[:,1], rays_a[-1,1] + rays_a[-1,2]]:
 *   dL_drays_o[r] = sum_{s in [indptr[r], indptr[r+1])} dL_dxyzs[s]              (n_rays, 3)
 *   dL_drays_d[r] = sum_{s in [indptr[r], indptr[r+1])} dL_dxyzs[s] * ts[s] + dL_ddirs[s]
 * One wave per row, fixed summation order (no atomics): deterministic run to run.  dL_dxyzs or
 * dL_ddirs may be NULL (a zero gradient). */
int ncn_segment_csr(const float* dL_dxyzs, const float* dL_ddirs, const float* ts, const int64_t* rays_a,
                    int64_t n_rays, float* dL_drays_o, float* dL_drays_d, void* stream);

/* raymarching_train for the training step in two launches (constant dt, exp_step_factor == 0):
 * render()'s single-AABB intersection + near clamp (intersection.cu:5-56, rendering.py:24-28), the
 * jitter (custom_functions.py:83; `noise` (R) or, when NULL, a counter-based uniform of (seed,
 * *rng_counter, ray): graph replays draw fresh noise through the device counter) and the walk; then
 * the placement (every workgroup adds the sample counts of the rays before it) and the packing:
 * writes rays_a, the packed xyzs/dirs/deltas/ts (capacity R*max_samples rows, first counter[0]
 * valid) and counter = {S, R}.  Sample segments are in ray order; rays_a ROWS put the rays with
 * more than 256 samples first (each class in ray order), so the compositors start them first (the
 * reference's rows are in atomicAdd order: any row order is within its contract).  Slabs as ncn_march_train_walk; work =
 * ncn_march_train_fused_work_bytes(R) bytes of scratch.  R <= 16384. */
int64_t ncn_march_train_fused_work_bytes(int64_t n_rays);
int ncn_march_train_fused(const float* rays_o, const float* rays_d, int64_t n_rays, float cx, float cy, float cz,
                          float hx, float hy, float hz, float near_distance, const float* noise, uint64_t seed,
                          const int64_t* rng_counter, const uint8_t* bitfield, int cascades, float scale,
                          int grid_size, int max_samples, float* slab_xyz, float* slab_t, float* slab_dt, void* work,
                          int64_t* rays_a, float* xyzs, float* dirs, float* deltas, float* ts, int32_t* counter,
                          void* stream);

/* ---- test-time marcher: replaces vren.raymarching_test (raymarching.cu:407-454).
 * Outputs (A,N_samples[,3]) are fully written (zeros past n_eff).  Mutates hits_t[r][0]. ---- */
int ncn_march_test(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive, int64_t n_alive,
                   const uint8_t* bitfield, int cascades, float scale, float exp_step_factor, int grid_size,
                   int max_samples, int n_samples, float* xyzs, float* dirs, float* deltas, float* ts,
                   int32_t* n_eff, void* stream);

/* ---- compositing: replaces vren.composite_train_multi_fw / _bw / composite_test_multi_fw
 *      (volumerendering.cu:140-176, 367-418, 553-586).  All outputs fully written (no pre-zeroing).
 *      In _bw any of dL_dopacity / dL_ddepth / dL_drend / dL_dws may be NULL (== zeros). ---- */
int ncn_composite_train_fw(const float* sigmas, const float* raws, const float* deltas, const float* ts,
                           const int64_t* rays_a, int64_t n_rays, int64_t n_samples, int n_rend, float T_threshold,
                           int64_t* total_samples, float* opacity, float* depth, float* rend, float* ws,
                           void* stream);
int ncn_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drend,
                           const float* dL_dws, const float* sigmas, const float* raws, const float* ws,
                           const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                           int64_t n_samples, int n_rend, const float* opacity, const float* depth,
                           const float* rend, float T_threshold, float* dL_dsigmas, float* dL_draws, void* stream);

/* VolumeRenderer.forward's total_samples.sum() (custom_functions.py:139-146) -> *sum_out (int64),
 * one workgroup; with acc != NULL also acc[0] += counter[0] (the marcher's sample count; counter may
 * be NULL) and acc[1] += the sum: device-resident throughput counters of a captured step. */
int ncn_count_samples(const int64_t* total_samples, int64_t n_rays, const int32_t* counter, int64_t* sum_out,
                      double* acc, void* stream);

/* render()'s white/zero background fused into the compositor (rendering.py:232-240, used by the
 * train path when exp_step_factor == 0): the forward additionally writes rgb_bg = rend + bg *
 * (1 - opacity) (R, n_rend); the backward takes dL/drgb_bg in place of dL/drend and adds the
 * background's -bg * sum_i dL/drgb_i to dL/dopacity.  bg = 0 / rgb_bg = NULL is the plain kernel. */
int ncn_composite_train_fw_bg(const float* sigmas, const float* raws, const float* deltas, const float* ts,
                              const int64_t* rays_a, int64_t n_rays, int64_t n_samples, int n_rend, float T_threshold,
                              int64_t* total_samples, float* opacity, float* depth, float* rend, float* ws, float bg,
                              float* rgb_bg, void* stream);
int ncn_composite_train_bw_bg(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                              const float* dL_dws, const float* sigmas, const float* raws, const float* ws,
                              const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                              int64_t n_samples, int n_rend, const float* opacity, const float* depth,
                              const float* rend, float T_threshold, float bg, float* dL_dsigmas, float* dL_draws,
                              void* stream);
int ncn_composite_test_fw(const float* sigmas, const float* raws, const float* deltas, const float* ts,
                          int64_t* alive, int64_t n_alive, int n_samples, int n_rend, float T_threshold,
                          const int32_t* n_eff, float* opacity, float* depth, float* rend, void* stream);
/* Fused test-render iteration (no reference counterpart; rendering.py:80-101's valid mask + masked
 * field evaluation + scatter back, restructured): ncn_test_compact copies the valid samples of the
 * ncn_march_test output (ray n's first n_eff[n] of n_samples slots) to consecutive rows of xyz_c /
 * dir_c (n_alive * n_samples x 3 capacity), ray n's rows from offsets[n] (n_alive int32), and writes
 * the total to count[0] (device int32, set by the call) — the field then runs on *count rows
 * (n_dev); ncn_composite_test_fw_compact is ncn_composite_test_fw reading sigmas / raws through
 * offsets (deltas / ts stay in the (n_alive, n_samples) layout).  Outputs equal the reference
 * structure's bit for bit (the field's arithmetic is per sample). */
int ncn_test_compact(const float* xyzs, const float* dirs, const int32_t* n_eff, int64_t n_alive, int n_samples,
                     int32_t* offsets, float* xyz_c, float* dir_c, int32_t* count, void* stream);
int ncn_composite_test_fw_compact(const float* sigmas_c, const float* raws_c, const int32_t* offsets,
                                  const float* deltas, const float* ts, int64_t* alive, int64_t n_alive,
                                  int n_samples, int n_rend, float T_threshold, const int32_t* n_eff, float* opacity,
                                  float* depth, float* rend, void* stream);
/* Device-driven test loop (the fused iteration without a host read per iteration): ctrl is a
 * device int32[8] = {0 alive rays A, 1 samples per ray NS, 2 samples so far, 3 done, 4 valid samples
 * of the iteration, 5 next alive count, 6 iterations run, 7 sum of A x NS}; the caller initialises it
 * for the first iteration ({n_rays, NS0, NS0, 0, 0, 0, 0, 0}, NS0 = max(1, min_samples)) and sizes
 * every per-sample buffer for n_rays x min_samples samples (A x NS never exceeds it) and every
 * per-ray buffer for max_alive = n_rays.  One iteration: ncn_test_loop_march (ncn_march_test with
 * A / NS from ctrl), ncn_test_loop_index (the valid slots' indices into idx, their count into
 * ctrl[4], which must be 0), ncn_field_fwd on the march output with n_dev = ctrl + 4 and
 * order = idx (it evaluates and writes back exactly those slots), ncn_test_loop_composite (offsets
 * NULL: the (A, NS) layout), then ncn_test_loop_next (the kept rays of `alive` compacted into
 * alive_next, total_samples += ctrl[4], and the next A / NS formed as rendering.py:68-73 does:
 * done when no ray is alive or samples >= max_samples).  A done loop keeps A = 0: further iterations
 * launch empty, so the caller reads ctrl[3] only every few iterations. */
int ncn_test_loop_march(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive,
                        int64_t max_alive, const uint8_t* bitfield, int cascades, float scale, float exp_step_factor,
                        int grid_size, int max_samples, const int32_t* ctrl, float* xyzs, float* dirs, float* deltas,
                        float* ts, int32_t* n_eff, void* stream);
int ncn_test_loop_index(const int32_t* n_eff, int64_t max_alive, int32_t* ctrl, int32_t* idx, void* stream);
int ncn_test_loop_composite(const float* sigmas_c, const float* raws_c, const int32_t* offsets, const float* deltas,
                            const float* ts, int64_t* alive, int64_t max_alive, const int32_t* ctrl, int n_rend,
                            float T_threshold, const int32_t* n_eff, float* opacity, float* depth, float* rend,
                            void* stream);
int ncn_test_loop_next(const int64_t* alive, int64_t* alive_next, int64_t max_alive, int32_t* ctrl,
                       int64_t* total_samples, int n_rays, int max_samples, int min_samples, void* stream);

/* ---- NGPMT field: replaces tcnn Encoding(Grid/Hash) + sigma_net + rgb_net + TruncExp
 *      (ngp_mt.py:70-113, 157-229; custom_functions.py:162-173).
 * Hash grid geometry (16 levels, 2 features) is described by `levels` = 16 x {scale f32 bits,
 *   resolution, params, offset} as uint32 (see ncnerf_amd/ngp_mt.py:grid_levels).
 * Weights: fp32 masters in tcnn's padded shapes, concatenated (NCN_FIELD_NW floats): sigma_net
 *   W1 (64,32) W2 (16,64); rgb_net W3 (64,32) W4 (64,64) W5 (16,64) — tcnn pads rgb_net's 19 inputs
 *   cat[d/|d|, h] to 32 with constant 1.0 (columns 19..31 of W3 act as a bias) and its 3 outputs
 *   to 16 (rows 3..15 of W5 are parameters whose outputs are discarded).
 * precision: NCN_PREC_F16 (tcnn's FullyFusedMLP precision) or NCN_PREC_BF16 — the MFMA operand
 *   type of weights_packed, enc_cache and the activations; accumulation is fp32 either way.
 * weights_packed: NCN_FIELD_PACKED_HALVES 16-bit MFMA fragments (16-byte aligned) produced by
 *   ncn_field_pack_weights(precision) from the fp32 masters.
 * enc_cache: encoding cache for the backward in the operand precision, NCN_ENC_BYTES_PER_SAMPLE
 *   bytes per sample (rounded up to 16 samples, 16-byte aligned); may be NULL for inference.
 * mode 0: full (sigmas + rgbs), mode 1: density only (sigmas; dirs/rgbs ignored), mode 2: density
 *   only with the encoding split by level over the XCDs first (the grid refresh's points: each L2
 *   then serves two levels' tables; order must be NULL): enc_cache is required, as scratch of
 *   NCN_ENC_BYTES_PER_SAMPLE bytes per point; same sigmas as mode 1, bit for bit.
 * n_dev: NULL, or a device int32 holding the real sample count (<= n): then n is the capacity of
 *   the buffers (static-shape / graph-captured step, where the host never reads the marcher's
 *   counter); grids are sized from n, the kernels stop at *n_dev. ---- */
#define NCN_FIELD_NW (64 * 32 + 16 * 64 + 64 * 32 + 64 * 64 + 16 * 64)
#define NCN_FIELD_PACKED_HALVES 19456
#define NCN_ENC_BYTES_PER_SAMPLE 64
#define NCN_PREC_F16 0
#define NCN_PREC_BF16 1
int ncn_field_pack_weights(const float* w_master, uint16_t* weights_packed, int precision, void* stream);
/* The packing's map: src_index[q] (NCN_FIELD_PACKED_HALVES int32) = the master weight index (into the
 * NCN_FIELD_NW floats) that packed element q holds; every master weight appears at most twice (its
 * forward and its transposed backward fragment).  Used to build ncn_adam_step_packed's pack_inv. */
int ncn_field_pack_map(int32_t* src_index, void* stream);
/* Processing order of a training batch (no reference counterpart: tcnn evaluates in input order):
 * every window of 4096 consecutive samples sorted by the 30-bit Morton code of its normalised
 * positions; order[p] = the sample evaluated at position p (n int32, a permutation of each window).
 * `order` of ncn_field_fwd / _bwd / _bwd_mlp / _scatter: NULL (identity) or this array; enc_cache
 * and dE_ws are then in processing order, sigmas / rgbs / dL_d* stay in sample order. */
int ncn_field_sort_windows(const float* xyzs, int64_t n, const int32_t* n_dev, float xyz_min, float xyz_extent,
                           int32_t* order, void* stream);
int ncn_field_fwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                  const float* table,
                  const uint32_t* levels, float xyz_min, float xyz_extent, const uint16_t* weights_packed,
                  int precision, int mode, float* sigmas, float* rgbs, uint16_t* enc_cache, void* stream);
/* Backward: accumulates (+=) into grad_table (n_entries,2) and writes per-block weight-gradient
 * slabs (n_blocks x NCN_FIELD_NW) into `slab`; ncn_field_reduce_wgrad sums them into grad_w (+=).
 * loss_scale: NULL, or a device float S (a power of two): the AMP loss scale of the reference's
 * precision=16 run (torch GradScaler, train_nerf.py:954) — the MLP chain runs on the upstream
 * gradients times S (no fp16 underflow) and the outputs leave divided by S (ncn_adam_step's
 * amp_state keeps S and its growth/backoff).  With precision NCN_PREC_F16 the chain also carries
 * tcnn's own module loss scale NCN_TCNN_LOSS_SCALE (tinycudann/modules.py: fp16 modules multiply
 * dL/doutput by 128 and divide the input and parameter gradients by 128, on top of the caller's
 * GradScaler): the factor is S * 128 in, 1 / (S * 128) out.  An "external" AMP caller (the
 * upstream gradient already carries its GradScaler's scale, as tcnn sees it under PL precision=16)
 * passes a device 1.0f: the chain then runs at the upstream scale * 128, the outputs keep the
 * upstream scale.
 * n_blocks is returned by ncn_field_bwd_blocks(n).  dE_ws is a device workspace of
 * ncn_field_bwd_dE_floats(n) floats: a 4-float header, the level-major encoding gradient between the
 * MLP pass and the LDS-aggregating table scatter pass, and the sample positions xyzs in the
 * scatter's load order (four copies, one per unit class: a wave's round / grab reads one contiguous
 * stretch).  The MLP pass (its rgb part; not with `order`) writes the two coarse classes' positions
 * and marks them in the header (a class mask); the scatter reads a marked class's copy, and xyzs in
 * sample order for the others.  The last 32 words are the scatter's unit queue (a draw and a
 * departure counter per launch's first level): the MLP pass that writes the header (its sigma part,
 * or the one-pass MLP) zeroes them, and every scatter launch leaves them zero, so a workspace the
 * caller fills itself starts from zeroed memory.  Two scatter launches with the same level_lo must
 * not run concurrently on one workspace. */
int ncn_field_bwd_blocks(int64_t n);
int64_t ncn_field_bwd_dE_floats(int64_t n);
int ncn_field_bwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                  const uint32_t* levels,
                  float xyz_min, float xyz_extent, const uint16_t* weights_packed, int precision,
                  const uint16_t* enc_cache, const float* dL_dsigmas, const float* dL_drgbs, const float* loss_scale,
                  float* grad_table, float* slab, float* dE_ws,
                  float* level_max /* 16 * ncn_field_bwd_blocks(n) floats of workspace (per-level max |dE|) */,
                  void* stream);
/* ncn_field_bwd in its two passes (the data-parallel step overlaps the gradient all-reduce of one
 * level range with the scatter of the others): the MLP pass (weight-gradient slabs, dE_ws,
 * level_max), then the table scatter of the levels [level_lo, level_hi) into grad_table (+=).
 * max_blocks > 0 caps the scatter's workgroups (one per CU otherwise), leaving CUs to a concurrent
 * collective. */
int ncn_field_bwd_mlp(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                      const uint16_t* weights_packed,
                      int precision, const uint16_t* enc_cache, const float* dL_dsigmas, const float* dL_drgbs,
                      const float* loss_scale, float* slab, float* dE_ws, float* level_max, void* stream);
/* The MLP pass split by the gradient's source (the fused training step runs the rgb part while
 * the normal clustering computes the depth gradient): part 1 (rgb) = the rgb_net path from
 * dL_drgbs alone — slab tiles of W3..W5 (rows [0, its grid)) and the rgb part of dL/dh into
 * dh_stash (ncn_field_bwd_stash_floats(n) floats, 16-byte aligned: the MLP-operand-rounded values
 * the sigma pass consumes, plus the fp32 element the TruncExp term is added to — 36 B per sample);
 * it also zeroes level_max.
 * ORDERING: part 2 reads the stash and max-reduces (atomicMax) into the level_max rows part 1
 * zeroed, so part 2 must be stream-ordered after a COMPLETED part 1 on the same stash and level_max
 * (when part 1 runs on another stream, join that stream first, e.g. cur.wait_stream(side)); part 2
 * on its own would read a stale stash and the previous step's maxima.
 * Part 2 (sigma) = dL/dh = stash + TruncExp'(h0) * (dL_dsigmas + dL_dsigmas2) (either may be
 * NULL), then sigma_net: slab tiles of W1, W2 (rows [0, its grid)), dE_ws, level_max (max-reduced
 * into the 16 * ncn_field_bwd_blocks(n) floats the scatter reads).  Part 3 = ncn_field_bwd_mlp
 * (plus the second dsigma term).  Each part's grid is n_blocks when > 0 (capped at
 * ncn_field_bwd_part_blocks(n, part); a cap leaves CUs to a concurrent kernel), else
 * ncn_field_bwd_part_blocks(n, part) — part 2 keeps less LDS and runs twice the workgroups.
 * The slab holds max(grid 1, grid 2) rows; ncn_field_reduce_wgrad_parts(slab, grid 2, grid 1)
 * then sums each net's rows.  Parts 1 + 2 on equal grids give ncn_field_bwd_mlp's outputs bit for
 * bit (one dsigma term). */
int64_t ncn_field_bwd_stash_floats(int64_t n);
int ncn_field_bwd_part_blocks(int64_t n, int part);
int ncn_field_bwd_mlp_part(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                           const uint16_t* weights_packed, int precision, const uint16_t* enc_cache,
                           const float* dL_dsigmas, const float* dL_dsigmas2, const float* dL_drgbs,
                           const float* loss_scale, int part, int n_blocks, float* slab, float* dE_ws,
                           float* level_max, float* dh_stash, void* stream);
int ncn_field_reduce_wgrad_parts(const float* slab, int n_blocks_sigma, int n_blocks_rgb, float* grad_w,
                                 void* stream);
/* The positions of dE_ws's permuted region written from xyzs (n capacity, n_dev the device count or
 * NULL) and marked ready: what the MLP pass's rgb part does in the training step, for a caller that
 * fills dE_ws itself (the scatter then loads coalesced). */
int ncn_field_scatter_positions(const float* xyzs, int64_t n, const int32_t* n_dev, float* dE_ws, void* stream);
int ncn_field_scatter(const float* xyzs, int64_t n, const int32_t* n_dev, const int32_t* order,
                      const uint32_t* levels, float xyz_min,
                      float xyz_extent, const float* dE_ws, const float* level_max, int level_lo, int level_hi,
                      int max_blocks, float* grad_table, void* stream);
int ncn_field_reduce_wgrad(const float* slab, int n_blocks, float* grad_w, void* stream);
/* ncn_field_scatter with ncn_field_reduce_wgrad_parts(slab, n_blocks_sigma, n_blocks_rgb, grad_w)
 * folded into the same launch (its workgroups sum slices of the slab rows before their table units:
 * one kernel boundary and launch ramp less on the split backward's critical path).  slab NULL =
 * ncn_field_scatter. */
int ncn_field_scatter_wgrad(const float* xyzs, int64_t n, const int32_t* n_dev, const int32_t* order,
                            const uint32_t* levels, float xyz_min, float xyz_extent, const float* dE_ws,
                            const float* level_max, int level_lo, int level_hi, int max_blocks, float* grad_table,
                            const float* slab, int n_blocks_sigma, int n_blocks_rgb, float* grad_w, void* stream);

/* ---- normal clustering loss path: replaces _extract_normals_from_ray_batch
 *      (hypersim_src/utils.py:504-541) and the faiss + torch cluster block of NeRFMTLoss
 *      (losses.py:47-166, 420-478). ---- */
/* ncn_photo_loss_fwd + ncn_normals_fwd in one launch (the fused loss node's independent parts). */
int ncn_photo_normals_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays,
                          float w_opacity, float* loss, const float* rays_o, const float* rays_d, const float* depth,
                          const int64_t* x1, const int64_t* x2, const int64_t* x3, int64_t n_tri, float* normals,
                          void* stream);
/* The same plus the render's composited-sample count (ncn_count_samples: *count_out =
 * sum(total_samples[0..n_count)), count_acc += {counter[0], the sum} when non-NULL) in one extra
 * workgroup of the launch; total_samples NULL = ncn_photo_normals_fwd. */
int ncn_photo_normals_count_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays,
                                float w_opacity, float* loss, const float* rays_o, const float* rays_d,
                                const float* depth, const int64_t* x1, const int64_t* x2, const int64_t* x3,
                                int64_t n_tri, float* normals, const int64_t* total_samples, int64_t n_count,
                                const int32_t* counter, int64_t* count_out, double* count_acc, void* stream);
int ncn_normals_fwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1,
                    const int64_t* x2, const int64_t* x3, int64_t n_tri, float* normals, void* stream);
/* dL_ddepth += ...; if term_weights (3 device floats) is non-NULL, dL_dnormals is the (3,n_tri,3)
 * per-term output of ncn_cluster_loss and is combined as sum_q term_weights[q] * dL_dnormals[q]. */
int ncn_normals_bwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1,
                    const int64_t* x2, const int64_t* x3, int64_t n_tri, const float* dL_dnormals,
                    const float* term_weights, float* dL_ddepth, void* stream);
/* Photometric MSE + weighted opacity entropy (losses.py:349-362) with the validity filter
 * (losses.py:246-262): loss[0] = mean((rgb-gt)^2), loss[1] = w_opacity*mean(-o log o), o = opacity+1e-10,
 * loss[2..3] = 1 if the term is finite (else the term and its gradient are 0).  The backward
 * scales by the upstream gradient (2 device floats, or NULL = 1). */
int ncn_photo_loss_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                       float* loss, void* stream);
int ncn_photo_loss_bwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                       const float* loss, const float* upstream, float* dL_drgb, float* dL_dopacity, void* stream);
/* faiss k-means plan: the random draws of faiss's Clustering::train for every valid-point count
 * nx <= n_tri, built on the HOST with std::mt19937 (faiss's RandomGenerator engine):
 * subsample_training_set's rand_perm(seed) membership when nx > K*256, the init picks (first K of
 * rand_perm(seed + 1) of the training set, as indices into the valid points), and 4096 floats of
 * split_clusters' RandomGenerator(1234).  ncn_kmeans_plan_words(n_tri, K) 32-bit words; the caller
 * copies the filled host buffer to the device once and passes it to every ncn_cluster_loss call
 * with the same (n_tri, K).  seed: faiss ClusteringParameters::seed (1234 in the reference). */
int64_t ncn_kmeans_plan_words(int n_tri, int K);
int ncn_kmeans_plan_fill(int n_tri, int K, uint32_t seed, uint32_t* host_out);
/* Validity filter, spherical k-means (K in {10,20}, niter Lloyd iterations), cluster selection,
 * the three cluster losses and their gradient w.r.t. the normals, scaled by w_ort / w_dot / w_l1,
 * in ONE launch of 16 co-resident workgroups (KM_BLOCKS in csrc/loss.hip; tagged partial words between
 * the Lloyd rounds, grid barriers between the later phases).  n_tri <= 16384.
 * kmeans_plan: device copy of ncn_kmeans_plan_fill(n_tri, K, seed) (a mismatched plan sets the
 * status word, ncn_cluster_status_offset).
 * out_losses (11 floats): [0..2] = unweighted (ort, centr_dot, centr_L1) after the validity filter;
 * [3] = valid n; [4..6] = the weighted terms; [7..9] = the weights used; [10] = total (only when
 * photo_loss is given: photo_loss[0] + photo_loss[1] + [4] + [5] + [6], losses.py's sum over the
 * loss dict); out_labels (n_tri) int32 in {0,+-1,+-2,+-3} (-9 = invalid normal);
 * out_centroids (K,3); dL_dnormals (3,n_tri,3) fully written: the gradient of w_ort*ort, w_dot*centr_dot and w_l1*centr_L1
 * separately, so any upstream weighting of the three terms is a 3-term combination.
 * w_dev: NULL, or 3 device floats that replace (w_ort, w_dot, w_l1).
 * step_dev: NULL, or the device training step: the weights become the schedule of losses.py:217,
 *   max(0, min(w, (step - sched_start) * (w / sched_grow))), evaluated on the device (graph-safe).
 * photo_loss: NULL, or the 4 floats of ncn_photo_loss_fwd (for out_losses[10]).
 * workspace: ncn_cluster_workspace_words(K) 32-bit words of device scratch, ZERO-initialised once
 *   before its first use and reused across calls (every call leaves its barrier words at zero);
 *   one workspace per stream (two concurrent calls must not share one). */
int64_t ncn_cluster_workspace_words(int K);
/* Index (in 32-bit words) of the workspace's sticky error word: non-zero once a grid barrier or a
 * Lloyd hand-off of any call on this workspace timed out (its partial sums may be incomplete).
 * While it is set, every call drops its cluster terms as the reference's validity filter drops an
 * invalid term (losses.py:246-262): out_losses[0..2] and [4..6] are 0, dn is 0, out_losses[10] is
 * the photometric part only — so no gradient of a timed-out clustering is ever applied.  The
 * caller reads the word outside the hot loop (the training step: every few steps) and fails. */
int64_t ncn_cluster_status_offset(int K);
/* Co-residency guarantee of ncn_cluster_loss's grid barriers: its workgroups (16 x 512 threads) must
 * all be resident at once.  *capacity = (the device's CUs - busy_cus) x the kernel's workgroups per
 * CU; returns 0 when that holds the 16, else hipErrorCooperativeLaunchTooLarge (a caller that runs
 * work beside the clustering — the split step's rgb pass, one workgroup per CU — checks it before
 * capturing the step; ncn_cluster_loss itself refuses when the idle device cannot hold them). */
int ncn_cluster_coresidency(int K, int busy_cus, int* capacity);
int ncn_cluster_loss(const float* normals, int64_t n_tri, int K, int niter, const uint32_t* kmeans_plan,
                     float t_similar,
                     float w_ort, float w_dot, float w_l1, const float* w_dev, const int64_t* step_dev,
                     float sched_start, float sched_grow, const float* photo_loss, float* out_losses,
                     int32_t* out_labels, float* out_centroids, float* dL_dnormals, float* workspace, void* stream);
/* Backward of the whole NeRFMTLoss in the reference configuration (photometric + opacity +
 * normal-clustering terms, `all_images_triang_patch` 8x8 patches: n_rays a multiple of 64, the
 * triangles of losses.py:307-313 in patch order, dL_dnormals the (3, 49*n_rays/64, 3) output of
 * ncn_cluster_loss).  One thread per ray: dL_drgb (R,3) and dL_dopacity (R) of the photometric
 * terms, and dL_ddepth (R) GATHERED from the ray's triangle roles (written, not accumulated: no
 * zero-fill, no atomics).  up_total: NULL or the device gradient of `total`; up_terms: NULL or 5
 * device floats (gradients of the rgb, opacity, ort, centr_dot, centr_L1 outputs), added to it.
 * The two output groups can be taken apart: dL_drgb = dL_dopacity = NULL skips the photometric
 * part, dL_ddepth = NULL the clustering part (dL_dnormals is then not read), so the photometric
 * gradient can flow back while ncn_cluster_loss still runs. */
int ncn_nerf_loss_bwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                      const float* photo_loss, const float* rays_o, const float* rays_d, const float* depth,
                      const float* dL_dnormals, const float* up_total, const float* up_terms, float* dL_drgb,
                      float* dL_dopacity, float* dL_ddepth, void* stream);

/* ---- step inputs (train_nerf.py:208: the batch handed to training_step): copies n_bufs <= 8 device
 *      buffers (src[b] -> dst[b], n_bytes[b]; HOST arrays of device pointers), writes `step` to
 *      *step_dst and `flag` to *flag_dst (either may be NULL) in ONE launch — the new batch into a
 *      captured step's static inputs (flag: the deferred optimizer step's gate). ---- */
int ncn_step_inputs(int n_bufs, const void* const* src, void* const* dst, const int64_t* n_bytes, int64_t* step_dst,
                    int64_t step, int32_t* flag_dst, int32_t flag, void* stream);

/* ---- optimizer (train_nerf.py:262-291, 954-955): global-norm clip + Adam over a flat buffer. ---- */
/* step_inc: NULL, or a device int incremented once (the optimizer step counter of a captured step) */
int ncn_sumsq(const float* x, int64_t n, float* out_partial /* >= 1024 floats */, int* step_inc, void* stream);
/* lr_dev / step_dev: NULL, or device scalars that override lr / step (step_dev: bias corrections
 * 1 - beta^step are formed on the device), so a graph-captured step needs no host values. */
int ncn_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
             const float* sumsq_partial, float max_norm, float lr, float beta1, float beta2, float eps,
             float weight_decay, int step, const float* lr_dev, const int* step_dev, void* stream);
/* The whole step in two launches (sum of squares whose last workgroup forms the clip factor and
 * step scalars, then Adam of both groups): elements [0, n_group0) use weight decay wd0 (apex group
 * 0, the hash grid), the rest wd1.  The gradient used is grads * grad_scale (1/world after an
 * all-reduce SUM: the average of DDP without a separate division pass), clipped by its L2 norm.  step_dev is incremented (device step counter) and drives the
 * bias corrections; work holds ncn_adam_step_work_floats() floats, zero before the first call (its
 * arrival counter is left zero by every call).  zero_grads != 0: the Adam pass also writes zeros over
 * the gradient it consumed (the next step's zero_grad folded in).  Buffers 16-byte aligned. */
int ncn_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t n_group0,
                  float grad_scale, float max_norm, float lr, double beta1, double beta2, float eps, float wd0, float wd1,
                  const float* lr_dev, int* step_dev, float* work, int zero_grads, float* amp_state, const int* gate,
                  void* stream);
/* gate: NULL, or a device int: 0 = no gradient pending, the step is skipped (a deferred step of a
 * captured graph whose previous step has already been applied).
 * amp_state: NULL, or the GradScaler state of an AMP (fp16) run, device floats {scale, growth
 * tracker}: a gradient whose norm is not finite skips the update (parameters and moments unchanged,
 * step counter not advanced; the gradient is still zeroed with zero_grads) and halves the scale;
 * after NCN_AMP_GROWTH_INTERVAL finite steps in a row the scale doubles (torch.cuda.amp.GradScaler
 * defaults: init 2^16, factors 2 / 0.5, interval 2000). */
#define NCN_AMP_INIT_SCALE 65536.0f
#define NCN_TCNN_LOSS_SCALE 128.0f /* tcnn fp16 module loss scale (ncn_field_bwd) */
#define NCN_AMP_GROWTH_INTERVAL 2000
int64_t ncn_adam_step_work_floats(void);
/* ncn_adam_step that also refreshes the field's packed MLP fragments (the ncn_field_pack_weights
 * launch between the optimizer and the next forward, folded into the Adam pass): the parameters
 * [pack_off, n) are the NCN_FIELD_NW master weights; pack_inv (NCN_FIELD_NW x 2 int32, -1 = none,
 * built from ncn_field_pack_map) lists the packed elements of each; `packed` receives the updated
 * (or, on a skipped step, the unchanged) weights rounded to pack_prec (NCN_PREC_F16 / _BF16) — the
 * same values ncn_field_pack_weights writes. */
int ncn_adam_step_packed(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t n_group0,
                         float grad_scale, float max_norm, float lr, double beta1, double beta2, float eps, float wd0,
                         float wd1, const float* lr_dev, int* step_dev, float* work, int zero_grads, float* amp_state,
                         const int* gate, const int32_t* pack_inv, int64_t pack_off, uint16_t* packed, int pack_prec,
                         void* stream);
/* Data-parallel gradient wire format (replaces DDP's fp16 gradient buckets, train_nerf.py:944-952:
 * the reference's tcnn parameters and gradients are fp16 at the GradScaler's scale, and torch DDP's
 * default hook divides each bucket by the world size before the all-reduce SUM,
 * ddp_comm_hooks/default_hooks.py _allreduce_fut).
 * pack: wire[i] = fp16(float(fp16(grad[i] * scale[0])) / world) — the bucket's rounding, then DDP's
 * div_(world) rounding (round to nearest even; overflow -> inf, a step the GradScaler of
 * ncn_adam_step then skips); unpack: grad[i] = float(wire[i]) / scale[0] (overwrites): after the
 * SUM this is already the average over the ranks.
 * scale: NULL (1) or a device float, the AMP scale S (amp_state[0], a power of two).  world >= 1.
 * n elements, grad and wire 16-byte aligned. */
int ncn_grad_pack_f16(const float* grad, int64_t n, const float* scale, int world, uint16_t* wire, void* stream);
int ncn_grad_unpack_f16(const uint16_t* wire, int64_t n, const float* scale, float* grad, void* stream);

#ifdef __cplusplus
}
#endif
#endif
