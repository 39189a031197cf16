/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * path (normal-clustering-nerf_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C CPU restatement of the reference `vren` CUDA kernels on the training hot path
 * (reference: /root/reference/models/csrc/{raymarching,intersection,volumerendering}.cu).  Each function cites the reference lines it
 * restates.  Built by oracle/Makefile with `-O2 -ffp-contract=off` so that the only fused
 * multiply-adds are the explicit fmaf() calls below.
 *
 * Floating-point contract for the marching / intersection code (bit-exact target):
 *   The reference is built by nvcc -O2 with its default --fmad=true (models/csrc/setup.py:27-29),
 *   which contracts `a + b*c` / `b*c + a` / `b*c - a` into FMA.  We restate those sites with
 *   explicit fmaf() and forbid every other contraction.  The HIP kernels use the identical
 *   expression forms, so sample positions, voxel indices and sample counts are bit-identical.
 *
 * Ordering contract: the reference assigns `rays_a` rows and sample start offsets with
 * atomicAdd (raymarching.cu:237-238), i.e. in a nondeterministic order.  This restatement (and
 * the HIP path) uses ray order: rays_a[r] = (r, exclusive_prefix_sum(N)[r], N[r]).  Parity with
 * the reference is therefore per ray (compare segments after sorting by ray_idx).
 *
 * Parity status: the reference kernels are CUDA and cannot be built or run in this container
 * (no nvcc/CUDA toolkit, no NVIDIA GPU; DESIGN.md "Oracle").  The kernels below are pinned by
 * (a) known-answer tests (tests/test_oracle_kat.py), (b) gradient checks of composite_bw against
 * finite differences of composite_fw, and (c) golden vectors produced by the reference Python
 * glue (render(), VolumeRenderer/RayMarcher autograd wiring) driven through this oracle
 * (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SQRT3 1.73205080757f

/* helper_math.h:280-283  clamp(f,a,b) = fmaxf(a, fminf(f,b)) (device fminf/fmaxf = IEEE minNum/maxNum) */
static inline float clampf_(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }
/* raymarching.cu:7 */
static inline float signf_(float x) { return copysignf(1.0f, x); }
static inline int imin_(int a, int b) { return a < b ? a : b; }
static inline int imax_(int a, int b) { return a > b ? a : b; }

/* raymarching.cu:11-13 */
static inline float calc_dt(float t, float exp_step_factor, int max_samples, int grid_size, float scale) {
    return clampf_(t * exp_step_factor, SQRT3 / (float)max_samples, SQRT3 * 2 * scale / (float)grid_size);
}

/* raymarching.cu:19-23 */
static inline int mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int exponent;
    frexpf(mx, &exponent);
    return imin_(cascades - 1, imax_(0, exponent + 1));
}

/* raymarching.cu:29-32 */
static inline int mip_from_dt(float dt, int grid_size, int cascades) {
    int exponent;
    frexpf(dt * (float)grid_size, &exponent);
    return imin_(cascades - 1, imax_(0, exponent));
}

/* raymarching.cu:35-50 */
static inline uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static inline uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
/* raymarching.cu:52-60 */
static inline uint32_t morton3D_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

/* raymarching.cu:62-70 */
void ref_morton3D(const int32_t* coords, int64_t n, int32_t* out) {
    for (int64_t i = 0; i < n; i++)
        out[i] = (int32_t)morton3D((uint32_t)coords[3 * i], (uint32_t)coords[3 * i + 1], (uint32_t)coords[3 * i + 2]);
}

/* raymarching.cu:90-101 */
void ref_morton3D_invert(const int32_t* idx, int64_t n, int32_t* coords) {
    for (int64_t i = 0; i < n; i++) {
        const int32_t ind = idx[i];
        coords[3 * i + 0] = (int32_t)morton3D_invert((uint32_t)(ind >> 0));
        coords[3 * i + 1] = (int32_t)morton3D_invert((uint32_t)(ind >> 1));
        coords[3 * i + 2] = (int32_t)morton3D_invert((uint32_t)(ind >> 2));
    }
}

/* raymarching.cu:122-141 (n_bytes = density_bitfield.size(0), :148) */
void ref_packbits(const float* grid, int64_t n_bytes, float threshold, uint8_t* bitfield) {
    for (int64_t n = 0; n < n_bytes; n++) {
        uint8_t bits = 0;
        for (int i = 0; i < 8; i++) bits |= (grid[8 * n + i] > threshold) ? (uint8_t)(1u << i) : 0;
        bitfield[n] = bits;
    }
}

/* intersection.cu:5-21 */
static inline void ray_aabb(const float o[3], const float inv_d[3], const float c[3], const float h[3],
                            float* t1o, float* t2o) {
    float tmin[3], tmax[3];
    for (int k = 0; k < 3; k++) {
        tmin[k] = (c[k] - h[k] - o[k]) * inv_d[k];
        tmax[k] = (c[k] + h[k] - o[k]) * inv_d[k];
    }
    float a1[3], a2[3];
    for (int k = 0; k < 3; k++) { a1[k] = fminf(tmin[k], tmax[k]); a2[k] = fmaxf(tmin[k], tmax[k]); }
    const float t1 = fmaxf(fmaxf(a1[0], a1[1]), a1[2]);
    const float t2 = fminf(fminf(a2[0], a2[1]), a2[2]);
    if (t1 > t2) { *t1o = -1.0f; *t2o = -1.0f; return; }
    *t1o = t1; *t2o = t2;
}

/* intersection.cu:25-56 + 59-100.  Hits are gathered in voxel order (the deterministic version of
 * the atomicAdd order) and the max_hits slots — including the (-1,-1) empty slots, exactly as
 * torch::sort on hits_t[...,0] does (intersection.cu:95-97) — are stably sorted by t1. */
void ref_ray_aabb_intersect(const float* rays_o, const float* rays_d, int64_t n_rays,
                            const float* centers, const float* half_sizes, int64_t n_voxels, int max_hits,
                            int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx) {
    for (int64_t r = 0; r < n_rays; r++) {
        const float* o = rays_o + 3 * r;
        const float* d = rays_d + 3 * r;
        float inv_d[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
        float* ht = hits_t + (int64_t)r * max_hits * 2;
        int64_t* hv = hits_voxel_idx + (int64_t)r * max_hits;
        for (int k = 0; k < max_hits; k++) { ht[2 * k] = -1.0f; ht[2 * k + 1] = -1.0f; hv[k] = -1; }
        int cnt = 0;
        for (int64_t v = 0; v < n_voxels; v++) {
            float t1, t2;
            ray_aabb(o, inv_d, centers + 3 * v, half_sizes + 3 * v, &t1, &t2);
            if (t2 > 0) {
                if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hv[cnt] = v; }
                cnt++;
            }
        }
        hit_cnt[r] = cnt;
        /* stable insertion sort of the max_hits slots by t1 */
        for (int i = 1; i < max_hits; i++) {
            float a = ht[2 * i], b = ht[2 * i + 1];
            int64_t vi = hv[i];
            int j = i - 1;
            while (j >= 0 && ht[2 * j] > a) {
                ht[2 * (j + 1)] = ht[2 * j]; ht[2 * (j + 1) + 1] = ht[2 * j + 1]; hv[j + 1] = hv[j];
                j--;
            }
            ht[2 * (j + 1)] = a; ht[2 * (j + 1) + 1] = b; hv[j + 1] = vi;
        }
    }
}

/* One ray of raymarching_train_kernel (raymarching.cu:184-279).  If xyz != NULL the samples are
 * written at [0, N) of the given buffers.  Returns N_samples. */
static int march_train_ray(float ox, float oy, float oz, float dx, float dy, float dz, float t1, float t2,
                           float noise, const uint8_t* bitfield, int cascades, int grid_size, float scale,
                           float exp_step_factor, int max_samples,
                           float* xyz, float* dir, float* deltas, float* ts) {
    const uint32_t grid_size3 = (uint32_t)grid_size * grid_size * grid_size;
    const float grid_size_inv = 1.0f / (float)grid_size;
    const float dx_inv = 1.0f / dx, dy_inv = 1.0f / dy, dz_inv = 1.0f / dz;
    if (t1 >= 0) { /* :195-198 */
        const float dt = calc_dt(t1, exp_step_factor, max_samples, grid_size, scale);
        t1 = fmaf(dt, noise, t1);
    }
    float t = t1;
    int n = 0;
    while (0 <= t && t < t2 && n < max_samples) { /* :204 */
        const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
        const float dt = calc_dt(t, exp_step_factor, max_samples, grid_size, scale);
        const int mip = imax_(mip_from_pos(x, y, z, cascades), mip_from_dt(dt, grid_size, cascades));
        const float mip_bound = fminf(scalbnf(1.0f, mip - 1), scale);
        const float mip_bound_inv = 1.0f / mip_bound;
        /* :215-217  (int)clamp(0.5f*(x*inv+1)*G, 0, G-1) */
        const int nx = (int)clampf_(0.5f * fmaf(x, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
        const int ny = (int)clampf_(0.5f * fmaf(y, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
        const int nz = (int)clampf_(0.5f * fmaf(z, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
        const uint32_t idx = (uint32_t)mip * grid_size3 + morton3D((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
        const int occ = bitfield[idx / 8] & (1u << (idx % 8));
        if (occ) { /* :222-223, 263-268 */
            if (xyz) {
                xyz[3 * n] = x; xyz[3 * n + 1] = y; xyz[3 * n + 2] = z;
                dir[3 * n] = dx; dir[3 * n + 1] = dy; dir[3 * n + 2] = dz;
                ts[n] = t; deltas[n] = dt;
            }
            t += dt;
            n++;
        } else { /* :224-233 */
            const float tx = fmaf(fmaf(0.5f, signf_(dx), (float)nx + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -x) * dx_inv;
            const float ty = fmaf(fmaf(0.5f, signf_(dy), (float)ny + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -y) * dy_inv;
            const float tz = fmaf(fmaf(0.5f, signf_(dz), (float)nz + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -z) * dz_inv;
            const float t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
            do {
                t += calc_dt(t, exp_step_factor, max_samples, grid_size, scale);
            } while (t < t_target);
        }
    }
    return n;
}

/* raymarching.cu:166-332 (train marcher) in ray order.
 *   hits_t: (R,2) near/far; noise: (R); outputs sized by the caller to >= total samples
 *   rays_a: (R,3) int64 (ray_idx, start, N); counter: [total_samples, n_rays].
 * Pass xyzs == NULL to only count (rays_a[:,2] and counter[0] are still written). */
void ref_raymarching_train(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                           const uint8_t* bitfield, int cascades, float scale, float exp_step_factor,
                           const float* noise, int grid_size, int max_samples,
                           int64_t* rays_a, float* xyzs, float* dirs, float* deltas, float* ts, int32_t* counter) {
    int64_t offset = 0;
    for (int64_t r = 0; r < n_rays; r++) {
        const float* o = rays_o + 3 * r;
        const float* d = rays_d + 3 * r;
        int n = march_train_ray(o[0], o[1], o[2], d[0], d[1], d[2], hits_t[2 * r], hits_t[2 * r + 1], noise[r],
                                bitfield, cascades, grid_size, scale, exp_step_factor, max_samples,
                                xyzs ? xyzs + 3 * offset : NULL, xyzs ? dirs + 3 * offset : NULL,
                                xyzs ? deltas + offset : NULL, xyzs ? ts + offset : NULL);
        rays_a[3 * r] = r; rays_a[3 * r + 1] = offset; rays_a[3 * r + 2] = n;
        offset += n;
    }
    counter[0] = (int32_t)offset;
    counter[1] = (int32_t)n_rays;
}

/* raymarching.cu:335-404 (test marcher).  NOTE quirk q3: calc_dt is passed `cascades` where
 * `scale` belongs (:370, :399); restated as-is.  Mutates hits_t[r][0]. */
void ref_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive,
                          int64_t n_alive, const uint8_t* bitfield, int cascades, float scale,
                          float exp_step_factor, int grid_size, int max_samples, int N_samples,
                          float* xyzs, float* dirs, float* deltas, float* ts, int32_t* n_eff) {
    const uint32_t grid_size3 = (uint32_t)grid_size * grid_size * grid_size;
    const float grid_size_inv = 1.0f / (float)grid_size;
    const float cscale = (float)cascades;
    for (int64_t n = 0; n < n_alive; n++) {
        const int64_t r = alive[n];
        const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
        const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
        const float dx_inv = 1.0f / dx, dy_inv = 1.0f / dy, dz_inv = 1.0f / dz;
        float t = hits_t[2 * r], t2 = hits_t[2 * r + 1];
        int s = 0;
        float* X = xyzs + 3 * n * (int64_t)N_samples;
        float* D = dirs + 3 * n * (int64_t)N_samples;
        float* DT = deltas + n * (int64_t)N_samples;
        float* TS = ts + n * (int64_t)N_samples;
        for (int k = 0; k < N_samples; k++) {
            X[3 * k] = X[3 * k + 1] = X[3 * k + 2] = 0.0f;
            D[3 * k] = D[3 * k + 1] = D[3 * k + 2] = 0.0f;
            DT[k] = 0.0f; TS[k] = 0.0f;
        }
        while (t < t2 && s < N_samples) {
            const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
            const float dt = calc_dt(t, exp_step_factor, max_samples, grid_size, cscale);
            const int mip = imax_(mip_from_pos(x, y, z, cascades), mip_from_dt(dt, grid_size, cascades));
            const float mip_bound = fminf(scalbnf(1.0f, mip - 1), scale);
            const float mip_bound_inv = 1.0f / mip_bound;
            const int nx = (int)clampf_(0.5f * fmaf(x, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
            const int ny = (int)clampf_(0.5f * fmaf(y, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
            const int nz = (int)clampf_(0.5f * fmaf(z, mip_bound_inv, 1.0f) * (float)grid_size, 0.0f, grid_size - 1.0f);
            const uint32_t idx = (uint32_t)mip * grid_size3 + morton3D((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
            const int occ = bitfield[idx / 8] & (1u << (idx % 8));
            if (occ) {
                X[3 * s] = x; X[3 * s + 1] = y; X[3 * s + 2] = z;
                D[3 * s] = dx; D[3 * s + 1] = dy; D[3 * s + 2] = dz;
                TS[s] = t; DT[s] = dt;
                t += dt;
                hits_t[2 * r] = t;
                s++;
            } else {
                const float tx = fmaf(fmaf(0.5f, signf_(dx), (float)nx + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -x) * dx_inv;
                const float ty = fmaf(fmaf(0.5f, signf_(dy), (float)ny + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -y) * dy_inv;
                const float tz = fmaf(fmaf(0.5f, signf_(dz), (float)nz + 0.5f) * grid_size_inv * 2 - 1, mip_bound, -z) * dz_inv;
                const float t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
                do {
                    t += calc_dt(t, exp_step_factor, max_samples, grid_size, cscale);
                } while (t < t_target);
            }
        }
        n_eff[n] = s;
    }
}

/* volumerendering.cu:97-137 (composite_train_multi_fw_kernel) + :140-176 (zero-initialised outputs).
 * rays_a rows are processed in the given order; outputs indexed by ray_idx. */
void ref_composite_train_fw(const float* sigmas, const float* raws, const float* deltas, const float* ts,
                            const int64_t* rays_a, int64_t n_rays, int64_t n_samples, int n_rend, float T_thr,
                            int64_t* total_samples, float* opacity, float* depth, float* rend, float* ws) {
    memset(ws, 0, sizeof(float) * n_samples);
    for (int64_t n = 0; n < n_rays; n++) {
        const int64_t ray = rays_a[3 * n]; opacity[ray] = 0; depth[ray] = 0;
        for (int i = 0; i < n_rend; i++) rend[ray * n_rend + i] = 0;
        total_samples[ray] = 0;
    }
    for (int64_t n = 0; n < n_rays; n++) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        int64_t samples = 0;
        float T = 1.0f;
        while (samples < N) {
            const int64_t s = start + samples;
            const float a = 1.0f - expf(-sigmas[s] * deltas[s]);
            const float w = a * T;
            for (int i = 0; i < n_rend; i++) rend[ray * n_rend + i] += w * raws[s * n_rend + i];
            depth[ray] += w * ts[s];
            opacity[ray] += w;
            ws[s] = w;
            T *= 1.0f - a;
            if (T <= T_thr) break; /* :133 break before samples++ (quirk q6) */
            samples++;
        }
        total_samples[ray] = samples;
    }
}

/* volumerendering.cu:297-364 (composite_train_multi_bw_kernel) + :367-418.  dL_dws may be NULL
 * (== all zeros, the configs' case: losses.py:290 feeds ts as ws, quirk q5). */
void ref_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drend,
                            const float* dL_dws, const float* sigmas, const float* raws, const float* ws,
                            const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                            int64_t n_samples, int n_rend, const float* opacity, const float* depth,
                            const float* rend, float T_thr, float* dL_dsigmas, float* dL_draws) {
    memset(dL_dsigmas, 0, sizeof(float) * n_samples);
    memset(dL_draws, 0, sizeof(float) * n_samples * n_rend);
    float* pre = (float*)malloc(sizeof(float) * (n_samples > 0 ? n_samples : 1));
    float* rend_tmp = (float*)malloc(sizeof(float) * (n_rend > 0 ? n_rend : 1));
    for (int64_t n = 0; n < n_rays; n++) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        /* :331-335 inclusive scan of dL_dws*ws over the whole marched segment */
        float acc = 0.0f;
        for (int64_t k = 0; k < N; k++) {
            acc += dL_dws ? dL_dws[start + k] * ws[start + k] : 0.0f;
            pre[start + k] = acc;
        }
        const float total = acc;
        const float O = opacity[ray], D = depth[ray];
        float T = 1.0f, d = 0.0f;
        for (int i = 0; i < n_rend; i++) rend_tmp[i] = 0.0f;
        for (int64_t samples = 0; samples < N; samples++) {
            const int64_t s = start + samples;
            const float a = 1.0f - expf(-sigmas[s] * deltas[s]);
            const float w = a * T;
            for (int i = 0; i < n_rend; i++) rend_tmp[i] += w * raws[s * n_rend + i];
            d += w * ts[s];
            T *= 1.0f - a;
            const float dws = dL_dws ? dL_dws[s] : 0.0f;
            float g = dL_dopacity[ray] * (1 - O) + dL_ddepth[ray] * (ts[s] * T - (D - d)) + T * dws - (total - pre[s]);
            for (int i = 0; i < n_rend; i++) {
                dL_draws[s * n_rend + i] = dL_drend[ray * n_rend + i] * w;
                g += dL_drend[ray * n_rend + i] * (raws[s * n_rend + i] * T - (rend[ray * n_rend + i] - rend_tmp[i]));
            }
            dL_dsigmas[s] = g * deltas[s];
            if (T <= T_thr) break;
        }
    }
    free(pre);
    free(rend_tmp);
}

/* volumerendering.cu:504-550 (composite_test_multi_fw_kernel).  In-place on alive, opacity, depth, rend. */
void ref_composite_test_fw(const float* sigmas, const float* raws, const float* deltas, const float* ts,
                           int64_t* alive, int64_t n_alive, int N_samples, int n_rend, float T_thr,
                           const int32_t* n_eff, float* opacity, float* depth, float* rend) {
    for (int64_t n = 0; n < n_alive; n++) {
        if (n_eff[n] == 0) { alive[n] = -1; continue; }
        const int64_t r = alive[n];
        float T = 1.0f - opacity[r];
        for (int s = 0; s < n_eff[n]; s++) {
            const int64_t k = n * (int64_t)N_samples + s;
            const float a = 1.0f - expf(-sigmas[k] * deltas[k]);
            const float w = a * T;
            for (int i = 0; i < n_rend; i++) rend[r * n_rend + i] += w * raws[k * n_rend + i];
            depth[r] += w * ts[k];
            opacity[r] += w;
            T *= 1.0f - a;
            if (T <= T_thr) { alive[n] = -1; break; }
        }
    }
}
