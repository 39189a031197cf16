// Normal-clustering loss path for gfx950:
//  * normals from rendered depth over pixel triangles  (datasets/hypersim_src/utils.py:504-541)
//  * spherical k-means + Manhattan cluster selection + cluster losses and their analytic gradient
//    (losses.py:47-166, 420-478), all inside ONE persistent launch of KM_BLOCKS = 16 workgroups (Lloyd partials
//    exchanged as tagged words), so the per-step clustering needs no device->host round trip (the
//    reference copies the normals to the host for faiss, losses.py:434).
#pragma clang fp contract(off)

#include <algorithm>
#include <atomic>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

// ---- normals: P = o + d*depth ; n = normalize(cross(P2-P1, P3-P1)) (F.normalize eps 1e-12) ----
__device__ __forceinline__ void tri_points(const float* __restrict__ o, const float* __restrict__ d,
                                           const float* __restrict__ depth, int64_t i, float P[3]) {
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = o[3 * i + k] + d[3 * i + k] * depth[i];
}

__device__ __forceinline__ void normals_fwd_one(const float* __restrict__ o, const float* __restrict__ d,
                                                const float* __restrict__ depth, const int64_t* __restrict__ x1,
                                                const int64_t* __restrict__ x2, const int64_t* __restrict__ x3,
                                                int64_t t, float* __restrict__ normals) {
    float P1[3], P2[3], P3[3];
    tri_points(o, d, depth, x1[t], P1);
    tri_points(o, d, depth, x2[t], P2);
    tri_points(o, d, depth, x3[t], P3);
    const float a0 = P2[0] - P1[0], a1 = P2[1] - P1[1], a2 = P2[2] - P1[2];
    const float b0 = P3[0] - P1[0], b1 = P3[1] - P1[1], b2 = P3[2] - P1[2];
    const float c0 = a1 * b2 - a2 * b1, c1 = a2 * b0 - a0 * b2, c2 = a0 * b1 - a1 * b0;
    const float nrm = fmaxf(sqrtf(c0 * c0 + c1 * c1 + c2 * c2), 1e-12f);
    normals[3 * t] = c0 / nrm;
    normals[3 * t + 1] = c1 / nrm;
    normals[3 * t + 2] = c2 / nrm;
}

__global__ void normals_fwd_kernel(const float* __restrict__ o, const float* __restrict__ d,
                                   const float* __restrict__ depth, const int64_t* __restrict__ x1,
                                   const int64_t* __restrict__ x2, const int64_t* __restrict__ x3, int64_t T,
                                   float* __restrict__ normals) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    normals_fwd_one(o, d, depth, x1, x2, x3, t, normals);
}

// d/d depth through P_k = o + d*depth, a = P2-P1, b = P3-P1, c = a x b, n = c / max(|c|, eps):
// the three vertex gradients (g1, g2, g3) of triangle t for the normal gradient g.
__device__ __forceinline__ void tri_depth_grads(const float* __restrict__ o, const float* __restrict__ d,
                                                const float* __restrict__ depth, int64_t i1, int64_t i2, int64_t i3,
                                                const float g[3], float& g1, float& g2, float& g3) {
    float P1[3], P2[3], P3[3];
    tri_points(o, d, depth, i1, P1);
    tri_points(o, d, depth, i2, P2);
    tri_points(o, d, depth, i3, P3);
    const float a[3] = {P2[0] - P1[0], P2[1] - P1[1], P2[2] - P1[2]};
    const float b[3] = {P3[0] - P1[0], P3[1] - P1[1], P3[2] - P1[2]};
    const float c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    const float len = sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    float dc[3];
    if (len > 1e-12f) {
        const float n[3] = {c[0] / len, c[1] / len, c[2] / len};
        const float ng = n[0] * g[0] + n[1] * g[1] + n[2] * g[2];
#pragma unroll
        for (int k = 0; k < 3; k++) dc[k] = (g[k] - n[k] * ng) / len;
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) dc[k] = g[k] / 1e-12f;
    }
    // c = a x b :  da = b x dc ,  db = dc x a
    const float da[3] = {b[1] * dc[2] - b[2] * dc[1], b[2] * dc[0] - b[0] * dc[2], b[0] * dc[1] - b[1] * dc[0]};
    const float db[3] = {dc[1] * a[2] - dc[2] * a[1], dc[2] * a[0] - dc[0] * a[2], dc[0] * a[1] - dc[1] * a[0]};
    g2 = da[0] * d[3 * i2] + da[1] * d[3 * i2 + 1] + da[2] * d[3 * i2 + 2];
    g3 = db[0] * d[3 * i3] + db[1] * d[3 * i3 + 1] + db[2] * d[3 * i3 + 2];
    g1 = -((da[0] + db[0]) * d[3 * i1] + (da[1] + db[1]) * d[3 * i1 + 1] + (da[2] + db[2]) * d[3 * i1 + 2]);
}
// normal gradient of triangle t: dn (T,3), or with term weights tw the (3,T,3) per-term stack
__device__ __forceinline__ void tri_normal_grad(const float* __restrict__ dn, const float* tw, int64_t T, int64_t t,
                                                float g[3]) {
#pragma unroll
    for (int k = 0; k < 3; k++) g[k] = dn[3 * t + k];
    if (tw) {
#pragma unroll
        for (int k = 0; k < 3; k++) g[k] = tw[0] * g[k] + tw[1] * dn[T * 3 + 3 * t + k] + tw[2] * dn[T * 6 + 3 * t + k];
    }
}

__global__ void normals_bwd_kernel(const float* __restrict__ o, const float* __restrict__ d,
                                   const float* __restrict__ depth, const int64_t* __restrict__ x1,
                                   const int64_t* __restrict__ x2, const int64_t* __restrict__ x3, int64_t T,
                                   const float* __restrict__ dn, const float* __restrict__ tw,
                                   float* __restrict__ ddepth) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const int64_t i1 = x1[t], i2 = x2[t], i3 = x3[t];
    float g[3], g1, g2, g3;
    tri_normal_grad(dn, tw, T, t, g);
    tri_depth_grads(o, d, depth, i1, i2, i3, g, g1, g2, g3);
    atomicAdd(ddepth + i1, g1);
    atomicAdd(ddepth + i2, g2);
    atomicAdd(ddepth + i3, g3);
}

// ---- photometric MSE + opacity entropy (losses.py:349-362, validity filter :246-262) ----
// One workgroup: loss[0] = mean((rgb - gt)^2), loss[1] = w_op * mean(-o log o), o = opacity + 1e-10.
constexpr int PH_THREADS = 1024;
__device__ __forceinline__ void photo_loss_fwd_wg(const float* __restrict__ rgb, const float* __restrict__ gt,
                                                  const float* __restrict__ op, int64_t R, float w_op,
                                                  float* __restrict__ loss) {
    __shared__ float red[2][PH_THREADS / 64];
    float a = 0.f, b = 0.f;
    for (int64_t i = threadIdx.x; i < R; i += PH_THREADS) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float d = rgb[3 * i + c] - gt[3 * i + c];
            a += d * d;
        }
        const float o = op[i] + 1e-10f;
        b += -o * logf(o);
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float sa = 0.f, sb = 0.f;
        for (int w = 0; w < PH_THREADS / 64; w++) { sa += red[0][w]; sb += red[1][w]; }
        const float mse = sa / (float)(3 * R), ent = w_op * (sb / (float)R);
        loss[0] = isfinite(mse) ? mse : 0.f;  // validity filter
        loss[1] = isfinite(ent) ? ent : 0.f;
        loss[2] = isfinite(mse) ? 1.f : 0.f;
        loss[3] = isfinite(ent) ? 1.f : 0.f;
    }
}

__global__ __launch_bounds__(PH_THREADS) void photo_loss_fwd_kernel(const float* __restrict__ rgb,
                                                                    const float* __restrict__ gt,
                                                                    const float* __restrict__ op, int64_t R,
                                                                    float w_op, float* __restrict__ loss) {
    photo_loss_fwd_wg(rgb, gt, op, R, w_op, loss);
}

// The photometric/opacity reduction (workgroup 0) and the normals from depth (the other
// workgroups, one triangle per thread) in one launch: the two independent forward parts of the
// fused loss node.
// With cnt_total: one more workgroup (block 1) sums the compositor's per-ray sample counts (the
// vr_samples of the render, ncn_count_samples' work) beside them instead of in a launch of its own.
__global__ __launch_bounds__(PH_THREADS) void photo_normals_fwd_kernel(
    const float* __restrict__ rgb, const float* __restrict__ gt, const float* __restrict__ op, int64_t R, float w_op,
    float* __restrict__ loss, const float* __restrict__ o, const float* __restrict__ d,
    const float* __restrict__ depth, const int64_t* __restrict__ x1, const int64_t* __restrict__ x2,
    const int64_t* __restrict__ x3, int64_t T, float* __restrict__ normals, const int64_t* __restrict__ cnt_total,
    int64_t cnt_n, const int32_t* __restrict__ cnt_counter, int64_t* __restrict__ cnt_out, double* __restrict__ cnt_acc) {
    if (blockIdx.x == 0) {
        photo_loss_fwd_wg(rgb, gt, op, R, w_op, loss);
        return;
    }
    const int nb0 = cnt_total ? 2 : 1;  // workgroups in front of the normals
    if (cnt_total && blockIdx.x == 1) {
        count_samples_wg(cnt_total, cnt_n, cnt_counter, cnt_out, cnt_acc);
        return;
    }
    const int64_t t = (int64_t)(blockIdx.x - nb0) * PH_THREADS + threadIdx.x;
    if (t < T) normals_fwd_one(o, d, depth, x1, x2, x3, t, normals);
}
// grads scaled by the upstream gradient g[0..1] (device scalars) and zeroed for filtered terms
__global__ void photo_loss_bwd_kernel(const float* __restrict__ rgb, const float* __restrict__ gt,
                                      const float* __restrict__ op, int64_t R, float w_op,
                                      const float* __restrict__ loss, const float* __restrict__ g,
                                      float* __restrict__ drgb, float* __restrict__ dop) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= R) return;
    const float ga = g ? g[0] * loss[2] : loss[2], gb = g ? g[1] * loss[3] : loss[3];
    const float sa = 2.f / (float)(3 * R);
#pragma unroll
    for (int c = 0; c < 3; c++) drgb[3 * i + c] = ga == 0.f ? 0.f : ga * sa * (rgb[3 * i + c] - gt[3 * i + c]);
    const float o = op[i] + 1e-10f;
    dop[i] = gb == 0.f ? 0.f : gb * w_op * (-(logf(o) + 1.f)) / (float)R;  // filtered term: no NaN leaks
}

// ---- fused backward of NeRFMTLoss for the reference configuration (losses.py:349-362 + 420-478,
// `all_images_triang_patch` 8x8 patches, base.py:53-58 / losses.py:307-313): one thread per ray
// writes dL/drgb and dL/dopacity of the photometric terms and GATHERS dL/ddepth from the (at most
// three) patch triangles the ray is a vertex of, so no zero-fill and no atomics:
//   local (i,j) is x1 of triangle (i,j) [i,j >= 1], x2 of (i+1,j) [i <= 6, j >= 1], x3 of (i,j+1)
//   [i >= 1, j <= 6]; triangle (i,j) of patch p is index p*49 + 7(i-1) + (j-1).
// Upstream gradients: up_total (the `total` output) + up_terms[5] (rgb, opacity, ort, centr_dot,
// centr_L1 outputs), either may be NULL (= 0).
__global__ void nerf_loss_bwd_kernel(const float* __restrict__ rgb, const float* __restrict__ gt,
                                     const float* __restrict__ op, int64_t R, float w_op,
                                     const float* __restrict__ photo, const float* __restrict__ o,
                                     const float* __restrict__ d, const float* __restrict__ depth,
                                     const float* __restrict__ dn, const float* __restrict__ up_total,
                                     const float* __restrict__ up_terms, float* __restrict__ drgb,
                                     float* __restrict__ dop, float* __restrict__ ddepth) {
    const int64_t ray = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (ray >= R) return;
    const float ut = up_total ? *up_total : 0.f;
    float u[5];
#pragma unroll
    for (int q = 0; q < 5; q++) u[q] = ut + (up_terms ? up_terms[q] : 0.f);
    // photometric (photo_loss_bwd_kernel)
    if (drgb) {
        const float ga = u[0] * photo[2], gb = u[1] * photo[3];
        const float sa = 2.f / (float)(3 * R);
#pragma unroll
        for (int c = 0; c < 3; c++) drgb[3 * ray + c] = ga == 0.f ? 0.f : ga * sa * (rgb[3 * ray + c] - gt[3 * ray + c]);
        const float oo = op[ray] + 1e-10f;
        dop[ray] = gb == 0.f ? 0.f : gb * w_op * (-(logf(oo) + 1.f)) / (float)R;
    }
    if (!ddepth) return;
    // normals -> depth, gathered over this ray's triangle roles
    const int64_t T = (R / 64) * 49;
    const float tw[3] = {u[2], u[3], u[4]};
    const int64_t p = ray >> 6;
    const int loc = (int)(ray & 63), i = loc >> 3, j = loc & 7;
    const int64_t b = p * 64;
    float acc = 0.f;
    float g[3], g1, g2, g3;
    if (i >= 1 && j >= 1) {  // x1 of (i, j)
        const int64_t t = p * 49 + 7 * (i - 1) + (j - 1);
        tri_normal_grad(dn, tw, T, t, g);
        tri_depth_grads(o, d, depth, ray, b + 8 * (i - 1) + j, b + 8 * i + (j - 1), g, g1, g2, g3);
        acc += g1;
    }
    if (i <= 6 && j >= 1) {  // x2 of (i+1, j)
        const int64_t t = p * 49 + 7 * i + (j - 1);
        tri_normal_grad(dn, tw, T, t, g);
        tri_depth_grads(o, d, depth, b + 8 * (i + 1) + j, ray, b + 8 * (i + 1) + (j - 1), g, g1, g2, g3);
        acc += g2;
    }
    if (i >= 1 && j <= 6) {  // x3 of (i, j+1)
        const int64_t t = p * 49 + 7 * (i - 1) + j;
        tri_normal_grad(dn, tw, T, t, g);
        tri_depth_grads(o, d, depth, b + 8 * i + (j + 1), b + 8 * (i - 1) + (j + 1), ray, g, g1, g2, g3);
        acc += g3;
    }
    ddepth[ray] = acc;
}

// ---- clustering ----
// faiss.Kmeans(3, K, niter, spherical=True) + index.search (losses.py:86-89) restated on the device
// (the algorithm of oracle/losses_ref.py:spherical_kmeans; its random draws — subsample
// permutation, init picks, split walk — come precomputed from a host-built plan).  The kernel
// layout is described at cluster_kernel.
constexpr int CL_MAX_TRI = 16384;
constexpr int NCN_MAX_NQ = 80;       // K * 4 at K = 20
#ifndef KM_THREADS_CFG
#define KM_THREADS_CFG 512
#endif
#ifndef KM_BLOCKS_CFG
#define KM_BLOCKS_CFG 16
#endif
constexpr int KM_THREADS = KM_THREADS_CFG;  // threads per workgroup of the clustering kernel
constexpr int KM_BLOCKS = KM_BLOCKS_CFG;    // co-resident workgroups (grid barriers)
constexpr int KM_CHUNK_MAX = CL_MAX_TRI / KM_BLOCKS;
// Copies of a Lloyd round's per-cluster LDS accumulators: lane l adds into copy l % KM_ACC_COPIES,
// so the lanes of one wave that picked the same cluster (same-address u64 atomics serialise) are
// spread over the copies; the publishing thread sums its word's copies (exact integers: the result
// does not depend on the split).
#ifndef KM_ACC_COPIES
#define KM_ACC_COPIES 4
#endif


__device__ __forceinline__ bool valid_normal(float a, float b, float c) {
    const bool zero = (fabsf(a) + fabsf(b) + fabsf(c)) == 0.0f;
    const bool bad = isnan(a) || isnan(b) || isnan(c) || isinf(a) || isinf(b) || isinf(c);
    return !(zero || bad);
}

// argmax_k <x, C_k> with ((x0 c0 + x1 c1) + x2 c2) in f32, no FMA (contract(off) above); ties ->
// lowest k.  (Tried: two clusters per packed-f32 instruction, v_pk_mul_f32 / v_pk_add_f32 with the
// same IEEE products and sums per half — 87 vs 82 us for the whole kernel: building the register
// pairs from the LDS centroids costs more than the halved multiplies save.)
template <int K>
__device__ __forceinline__ int nearest(const float (*C)[3], float x, float y, float z) {
    int best = 0;
    float bv = x * C[0][0] + y * C[0][1] + z * C[0][2];
#pragma unroll
    for (int k = 1; k < K; k++) {
        const float v = x * C[k][0] + y * C[k][1] + z * C[k][2];
        if (v > bv) { bv = v; best = k; }
    }
    return best;
}

// Workspace layout (32-bit words): cross-workgroup partial sums (double-buffered for the Lloyd
// iterations) and the grid-barrier words.  The barrier words must be zero before the first call
// and are left zero by every call (the last workgroup to leave resets them).
struct KmWs {
    long long* part;  // [2][KM_BLOCKS][K][4] fixed-point (x, y, z, count) per cluster
    long long* p2;    // [KM_BLOCKS][12] flipped member sums + counts per selected cluster
    long long* p3;    // [KM_BLOCKS][16] x.c, |x-c|_1, sign(x-c) sums per selected cluster
    unsigned* sync;   // [0] barrier arrivals, [1] departures, [2] error flag (stuck barrier), [3] launch sequence
};
__host__ __device__ inline KmWs km_ws(float* base, int K) {
    KmWs w;
    w.part = (long long*)base;
    w.p2 = w.part + 2 * KM_BLOCKS * K * 4;
    w.p3 = w.p2 + KM_BLOCKS * 12;
    w.sync = (unsigned*)(w.p3 + KM_BLOCKS * 16);
    return w;
}
__host__ __device__ inline int64_t km_ws_words(int K) { return 2 * (2 * KM_BLOCKS * K * 4 + KM_BLOCKS * 28) + 4; }

// Every sum of the pipeline is exact: values (all |v| <= 8) are added as 64-bit fixed point
// v * 2^40 (LDS u64 atomics inside a workgroup, then int64 partials across workgroups), so the
// result is independent of order and partition, and is rounded to f32 once.
constexpr double KM_FX = 1099511627776.0;  // 2^40
__device__ __forceinline__ unsigned long long km_fix(float v) {
    return (unsigned long long)__double2ll_rn((double)v * KM_FX);
}
__device__ __forceinline__ float km_unfix(long long q) { return (float)((double)q * (1.0 / KM_FX)); }
__device__ __forceinline__ unsigned long long km_fixl(float v) {  // Lloyd partials: 2^39 (tagged words)
    return (unsigned long long)__double2ll_rn((double)v * 549755813888.0);
}

// Cross-workgroup data moves with agent-scope (sc1) loads and stores only (MI355X_MICROARCH.md,
// inter-workgroup visibility, hand-off row 1): each storing wave waits for its stores, the
// workgroup meets at a barrier, ONE lane adds to the arrival counter; the poller's workgroup meets
// again before any sc1 load of the published bytes.
__device__ __forceinline__ long long ld_c(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_c(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Grid barrier number `phase` (1, 2, ...) over the KM_BLOCKS co-resident workgroups.  The spin is
// bounded: a barrier that does not complete within ~2^22 polls sets the error word (sync[2],
// sticky; ncn_cluster_status_offset) and lets the workgroup run on (never a hang); the launch then
// drops its cluster terms (zero losses and gradients, the grad stage below), and the training step
// reads the word every few steps and raises (losses.check_cluster_status).
// NCN_KM_SPIN_LIMIT / NCN_KM_POLL_LIMIT: diagnostic builds force the flag with a limit of 1.
#ifndef NCN_KM_SPIN_LIMIT
#define NCN_KM_SPIN_LIMIT (1u << 22)
#endif
#ifndef NCN_KM_POLL_LIMIT
#define NCN_KM_POLL_LIMIT (1u << 20)
#endif
__device__ __forceinline__ void km_grid_sync(unsigned* sync, unsigned phase) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = phase * (unsigned)KM_BLOCKS;
        unsigned spins = 0;
        while (__hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins >= NCN_KM_SPIN_LIMIT) {
                __hip_atomic_store(&sync[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}
// Every workgroup calls this once, last: the final departure resets the barrier words and advances
// the launch sequence of the Lloyd tags (every launch, so a launch that did not cluster never
// leaves the next one with the tags of an older launch's partials).  Returns (to every thread of
// the LAST departing workgroup only) whether the error word is set: every workgroup's output
// stores are drained (vmcnt(0)) before its departure, so that workgroup can still overwrite the
// whole launch's outputs — the drop decision is then uniform even when a workgroup timed out after
// another one had read the word.
__device__ __forceinline__ bool km_grid_exit(unsigned* sync) {
    __shared__ int late_drop;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        late_drop = 0;
        const unsigned d = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (d == KM_BLOCKS - 1) {  // everyone has passed every barrier: nobody polls any more
            late_drop = __hip_atomic_load(&sync[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0u;
            __hip_atomic_store(&sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&sync[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // launch sequence (tags)
        }
    }
    __syncthreads();
    return late_drop != 0;
}

// This workgroup's contiguous chunk of the compacted points.
__device__ __forceinline__ void km_chunk(int nv, int& m0, int& len) {
    const int chunk = (nv + KM_BLOCKS - 1) / KM_BLOCKS;
    m0 = blockIdx.x * chunk;
    len = max(0, min(nv, m0 + chunk) - m0);
}

// Exact sum of KM_BLOCKS int64 partial rows published by other workgroups (all loads issued
// before the first add: one round trip), as f32.
__device__ __forceinline__ float sum_rows(const long long* __restrict__ p, int row, int off) {
    long long v[KM_BLOCKS];
#pragma unroll
    for (int b = 0; b < KM_BLOCKS; b++) v[b] = ld_c(p + b * row + off);
    long long a = 0;
#pragma unroll
    for (int b = 0; b < KM_BLOCKS; b++) a += v[b];
    return km_unfix(a);
}
__device__ __forceinline__ void sum_partials(const long long* __restrict__ p, int row, int nq, float* out) {
    if (threadIdx.x < nq) out[threadIdx.x] = sum_rows(p, row, threadIdx.x);
}

// Lloyd-round partials are published as TAGGED words instead of behind a grid barrier: each
// int64 word = tag << 50 | (fixed-point value mod 2^50), value = sum * 2^39 (a workgroup's sum of
// at most KM_CHUNK_MAX = 512 unit components: |value| <= 2^48; the precision of the barrier-based
// 2^40 sums within a factor 2).  tag = ((launch sequence + 1) mod 2^9) << 5 | round; every launch
// writes every word of both buffers (a launch that does not cluster writes void tags), so a word
// is never older than the previous launch and 9 sequence bits cannot alias,
// so a reader polls the words themselves until all KM_BLOCKS rows carry the round's tag: one
// store and (usually) one load round trip per round instead of store + arrive + poll + load.
// The rows are double-buffered by round parity: a workgroup writes round it+2 only after it read
// round it+1 from every workgroup, each of which published it+1 only after reading round it.
constexpr double KM_FXL = 549755813888.0;  // 2^39
constexpr int KM_TAG_SHIFT = 50;
constexpr unsigned long long KM_VMASK = (1ull << KM_TAG_SHIFT) - 1;
constexpr unsigned KM_VOID_ROUND = 31;  // round field of the void words (niter <= 30)
__device__ __forceinline__ long long km_tagged(unsigned tag, long long v) {
    return (long long)(((unsigned long long)tag << KM_TAG_SHIFT) | ((unsigned long long)v & KM_VMASK));
}
__device__ __forceinline__ unsigned km_round_tag(unsigned seq, int it) { return (((seq + 1u) & 0x1FFu) << 5) | (unsigned)it; }
// Exact sum of the KM_BLOCKS tagged words p[b * row + off] once every one carries `tag` (bounded
// poll: a row that never arrives sets the error word, as km_grid_sync does).
__device__ __forceinline__ float sum_rows_tagged(const long long* __restrict__ p, int row, int off, unsigned tag,
                                                 unsigned* sync) {
    long long v[KM_BLOCKS];
    for (unsigned spins = 0;; spins++) {
#pragma unroll
        for (int b = 0; b < KM_BLOCKS; b++) v[b] = ld_c(p + b * row + off);
        bool ready = true;
#pragma unroll
        for (int b = 0; b < KM_BLOCKS; b++) ready &= ((unsigned long long)v[b] >> KM_TAG_SHIFT) == tag;
        if (ready) break;
        if (spins + 1 >= NCN_KM_POLL_LIMIT) {
            __hip_atomic_store(&sync[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    long long a = 0;
#pragma unroll
    for (int b = 0; b < KM_BLOCKS; b++)  // sign-extend the 50-bit values
        a += (long long)((unsigned long long)v[b] << (64 - KM_TAG_SHIFT)) >> (64 - KM_TAG_SHIFT);
    return (float)((double)a * (1.0 / KM_FXL));
}

// faiss's k-means plan (host-built by ncn_kmeans_plan_fill; the faiss restatement of
// oracle/losses_ref.py): header words, init picks per point count, training-set membership masks
// per point count above the subsampling cap, split_clusters' RandomGenerator(1234) floats.
struct KmPlan {
    const uint32_t* p;
    __device__ __forceinline__ int n_tri() const { return (int)p[1]; }
    __device__ __forceinline__ int K() const { return (int)p[2]; }
    __device__ __forceinline__ int cap() const { return (int)p[3]; }
    __device__ __forceinline__ int n_rand() const { return (int)p[4]; }
    __device__ __forceinline__ int init(int nx, int k) const {
        return (int)((const uint16_t*)(p + p[5]))[(int64_t)nx * p[2] + k];
    }
    __device__ __forceinline__ bool member(int nx, int rank) const {
        if (nx <= (int)p[3]) return true;
        const int mw = ((int)p[1] + 31) >> 5;
        return (p[p[6] + (int64_t)(nx - (int)p[3] - 1) * mw + (rank >> 5)] >> (rank & 31)) & 1u;
    }
    __device__ __forceinline__ float rnd(int i) const { return __uint_as_float(p[p[7] + i]); }
};

// faiss fvec_renorm_L2 of one 3-vector: x *= (float)(1.0 / sqrtf(|x|^2)) when |x|^2 > 0
__device__ __forceinline__ void faiss_renorm3(float* x) {
    const float nr = x[0] * x[0] + x[1] * x[1] + x[2] * x[2];
    if (nr > 0.f) {
        const float inv = (float)(1.0 / (double)sqrtf(nr));
        x[0] *= inv; x[1] *= inv; x[2] *= inv;
    }
}

// One faiss iteration's update (Clustering.cpp compute_centroids + split_clusters +
// post_process_centroids): centroid = sum * (1 / count); each empty cluster ci, in order, takes
// the cluster cj found by walking cj = 0, 1, ... (mod K) until RandomGenerator(1234).rand_float()
// < (count_cj - 1) / (n_train - K), a +-1/1024 perturbation splits the two, and the counts halve
// (float); then every centroid is L2-renormalised.  The random floats come from the plan.
// Lanes 4k..4k+3 of waves 0-1 sum (cluster k, component c) over the workgroups' tagged rows, the
// count and the components meet inside the quad (DPP), and the renormalised centroid goes to C
// with ONE workgroup barrier; the same float operations as compute-then-renorm (faiss_renorm3's
// order), so the result is bit-identical.  A rare empty cluster takes the serial split path
// (thread 0, from the means and counts in LDS) behind two more barriers.  The thread that published
// acc[t] last round clears it here (the next round's sums start from zero).
template <int CTRL>
__device__ __forceinline__ float km_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int Q>
__device__ __forceinline__ float km_quad_get(float v) { return km_dpp<Q | (Q << 2) | (Q << 4) | (Q << 6)>(v); }
template <int K>
struct KmUpdLds {
    float nc[K][3];
    float cnt[K];
    int emp[2];  // per wave: an empty cluster this round (waves 0 and 1)
};
template <int K>
__device__ void km_update(const long long* __restrict__ part, float (*C)[3], KmUpdLds<K>& L,
                          unsigned long long* __restrict__ acc, unsigned tag, unsigned* sync, const KmPlan& plan,
                          int n_train) {
    static_assert(K * 4 <= 128, "the sums of a round are taken by waves 0 and 1");
    const int t = threadIdx.x;
    if (t < K * 4) {  // (quads whole: K * 4 lanes)
#pragma unroll
        for (int c = 0; c < KM_ACC_COPIES; c++) acc[c * NCN_MAX_NQ + t] = 0ull;
        const int k = t >> 2, c = t & 3;
        const float v = sum_rows_tagged(part, K * 4, t, tag, sync);
        const float n = km_quad_get<3>(v);
        const float inv = n > 0.f ? 1.0f / n : 0.f;
        const float m = v * inv;  // (0 for an empty cluster)
        const float x0 = km_quad_get<0>(m), x1 = km_quad_get<1>(m), x2 = km_quad_get<2>(m);
        if (c < 3) L.nc[k][c] = m;
        else L.cnt[k] = n;
        const uint64_t em = __ballot(c == 3 && n == 0.f);
        if ((t & 63) == 0) L.emp[t >> 6] = em != 0;
        const float nr = x0 * x0 + x1 * x1 + x2 * x2;  // faiss_renorm3
        const float y = nr > 0.f ? m * (float)(1.0 / (double)sqrtf(nr)) : m;
        if (c < 3) C[k][c] = y;
    }
    __syncthreads();
    if (L.emp[0] | L.emp[1]) {  // (uniform, rare)
        if (threadIdx.x == 0) {
            const float EPS = 1.0f / 1024.0f;
            const double denom = (double)(float)(n_train - K);
            int ri = 0;
            const int nr = plan.n_rand();
            for (int ci = 0; ci < K; ci++) {
                if (L.cnt[ci] != 0.f) continue;
                int cj = 0;
                for (;; cj = (cj + 1) % K) {
                    const float pr = (float)(((double)L.cnt[cj] - 1.0) / denom);
                    if (ri >= nr) {  // (a split walk longer than the plan's table: flag and take cj)
                        __hip_atomic_store(&sync[2], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    if (plan.rnd(ri++) < pr) break;
                }
                for (int q = 0; q < 3; q++) {
                    L.nc[ci][q] = L.nc[cj][q];
                    if (q % 2 == 0) { L.nc[ci][q] *= 1 + EPS; L.nc[cj][q] *= 1 - EPS; }
                    else { L.nc[ci][q] *= 1 - EPS; L.nc[cj][q] *= 1 + EPS; }
                }
                L.cnt[ci] = L.cnt[cj] / 2;
                L.cnt[cj] -= L.cnt[ci];
            }
        }
        __syncthreads();
        if (threadIdx.x < K) {
            const int k = threadIdx.x;
            float c[3] = {L.nc[k][0], L.nc[k][1], L.nc[k][2]};
            faiss_renorm3(c);
#pragma unroll
            for (int q = 0; q < 3; q++) C[k][q] = c[q];
        }
        __syncthreads();
    }
}

// Cluster selection of losses.py:75-166 from the final centroids and sizes -> label_map[K]
// (+-1..3 for the three orthogonal main clusters and their opposites, 0 otherwise).
template <int K>
struct SelLds {
    float sim[K][K];
    float cmin[K];
    int cargmin[K];
};

template <int K>
__device__ void select_clusters(const float (*C)[3], const float* cnt, float t_sim, SelLds<K>& L, int* label_map) {
    const int tid = threadIdx.x;
    for (int q = tid; q < K * K; q += KM_THREADS) {
        const int i = q / K, j = q % K;
        L.sim[i][j] = C[i][0] * C[j][0] + C[i][1] * C[j][1] + C[i][2] * C[j][2];
    }
    __syncthreads();
    int c1 = 0;  // biggest cluster (topk(sorted)[0]; ties -> lowest index)
    for (int k = 1; k < K; k++)
        if (cnt[k] > cnt[c1]) c1 = k;
    if (tid < K) {  // criteria[i][j] = |s(i,c1)| + |s(c1,j)| + |s(i,j)| ; min over i (first) per column j
        const int j = tid;
        float mn = 0.f;
        int mi = -1;
        for (int i = 0; i < K; i++) {
            const float cr = fabsf(L.sim[i][c1]) + fabsf(L.sim[c1][j]) + fabsf(L.sim[i][j]);
            if (mi < 0 || cr < mn) { mn = cr; mi = i; }
        }
        L.cmin[j] = mn;
        L.cargmin[j] = mi;
    }
    __syncthreads();
    if (tid < 64) {  // one wave: c2 = first argmin of cmin, its c3, then per-cluster labels
        // (wave-uniform serial scans over the K LDS values: independent broadcast loads and a short
        // compare chain, instead of 6 dependent cross-lane shuffles per argmin)
        auto first_argmin = [&](const float* v) {  // ties -> lowest index
            float b = v[0];
            int bi = 0;
#pragma unroll
            for (int k = 1; k < K; k++)
                if (v[k] < b) { b = v[k]; bi = k; }
            return bi;
        };
        const int c2 = first_argmin(L.cmin), c3 = L.cargmin[c2];
        const int cs[3] = {c1, c2, c3};
        // opposite of each main cluster: first argmin of sim[cs[q]][*]
        int co[3];
#pragma unroll
        for (int q = 0; q < 3; q++) co[q] = first_argmin(L.sim[cs[q]]);
        if (tid < K) {  // the sequential overwrite order of losses.py: main clusters, then opposites
            const int k = tid;
            int lab = 0;
            for (int q = 0; q < 3; q++)
                if (L.sim[cs[q]][k] > t_sim) lab = q + 1;
            for (int q = 0; q < 3; q++)
                if (-1.0f * L.sim[cs[q]][co[q]] > t_sim && L.sim[co[q]][k] > t_sim) lab = -(q + 1);
            label_map[k] = lab;
        }
    }
    __syncthreads();
}

// Per selected cluster: count, mean m, |m| and c = m/|m| from the p2 partials; ok = no empty cluster
// (the mean of an empty cluster is NaN -> every term filtered, losses.py:246-262).
struct ClStats {
    float st[12];
    float cnt[3], cm[3][3], cmn[3], cc[3][3];
    int ok;
};
__device__ void cluster_stats(const KmWs& ws, ClStats& S) {
    sum_partials(ws.p2, 12, 12, S.st);
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        for (int c = 0; c < 3; c++) {
            S.cnt[c] = S.st[4 * c + 3];
            if (S.cnt[c] == 0.f) ok = 0;
            for (int q = 0; q < 3; q++) S.cm[c][q] = S.cnt[c] > 0.f ? S.st[4 * c + q] / S.cnt[c] : 0.f;
            const float nr = sqrtf(S.cm[c][0] * S.cm[c][0] + S.cm[c][1] * S.cm[c][1] + S.cm[c][2] * S.cm[c][2]);
            S.cmn[c] = nr;
            for (int q = 0; q < 3; q++) S.cc[c][q] = S.cm[c][q] / fmaxf(nr, 1e-12f);
        }
        S.ok = ok;
    }
    __syncthreads();
}

template <int K>
struct ClusterLds {
    float pv[3][KM_CHUNK_MAX];  // this workgroup's chunk of the compacted normals (flip-signed after select)
    int pidx[KM_CHUNK_MAX];     // their original index
    int pk[KM_CHUNK_MAX];       // k-means assignment, then selected cluster 0..2 (-1 unselected)
    int plab[KM_CHUNK_MAX];     // selected label +-1..3 / 0
    unsigned long long acc[NCN_MAX_NQ];  // this workgroup's fixed-point sums of the phase
    unsigned long long accr[KM_ACC_COPIES][NCN_MAX_NQ];  // the Lloyd rounds' sums (per-lane copies)
    float C[K][3];
    float cnt[K];
    int label_map[K];
    int wcnt[CL_MAX_TRI / KM_THREADS][KM_THREADS / 64];
    int woff[CL_MAX_TRI / KM_THREADS][KM_THREADS / 64];
    int pick[K];       // init picks (ranks), sorted ascending
    int pick_ord[K];   // the centroid index of sorted pick k
    int picki[K];
    float pickv[K][3];  // the init picks' normals (register-resident compaction)
    unsigned char pmem[KM_CHUNK_MAX];  // training-set membership of the chunk's points (faiss subsampling)
    int total;
    int timed_out;  // the sticky error word, read once after the last grid barrier
    KmUpdLds<K> upd;
    SelLds<K> sel;
    ClStats S;
    float st3[15];
    float G[3][3][3];  // G[term][cluster][xyz]
};

// The whole clustering pipeline in ONE launch of KM_BLOCKS co-resident workgroups, the phases
// separated by grid barriers instead of kernel boundaries (23 of them at niter = 20):
//   compaction  (no barrier: every workgroup ranks all normals itself and keeps its chunk in LDS)
//               validity filter + ordered compaction (losses.py:427-430), faiss's training-set
//               membership and init picks from the plan
//   niter + 1 Lloyd rounds: C_i = update(partials_{i-1}, C_{i-1}) (i > 0), assign every point to
//               argmax <x, C_i>, per-workgroup partial sums (x, y, z, count) per cluster; the last
//               round (i = niter) is faiss's final search and keeps the assignment
//   select      cluster selection (losses.py:75-166) -> label per point, flipped partial sums
//   sums        per-cluster partials of x.c, |x-c|_1, sign(x-c)
//   grad        the three cluster losses and their analytic gradient per point (losses.py:469-478),
//               labels (-9 invalid), the weight schedule of losses.py:217 and the loss total
// Every workgroup reduces the same partials in the same fixed order, so all of them hold
// bit-identical centroids/statistics and the result is run-to-run deterministic.
#ifdef NCN_DIAG_CL_TIMES
__device__ unsigned long long ncn_cl_times[64];
#define CL_STAMP(i) \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (i) < 64) ncn_cl_times[(i)] = __builtin_amdgcn_s_memrealtime()
#else
#define CL_STAMP(i)
#endif
template <int K>
__global__ __launch_bounds__(KM_THREADS) void cluster_kernel(
    const float* __restrict__ normals, int n_tri, int niter, const uint32_t* __restrict__ plan_words, float t_sim,
    float w_ort, float w_dot,
    float w_l1, const float* __restrict__ w_dev, const int64_t* __restrict__ step_dev, float sched_start,
    float sched_grow, const float* __restrict__ photo, float* __restrict__ wsb, float* __restrict__ out_losses,
    int32_t* __restrict__ out_labels, float* __restrict__ out_centroids, float* __restrict__ dn) {
    constexpr int NW = KM_THREADS / 64;
    __shared__ ClusterLds<K> L;
    const KmWs ws = km_ws(wsb, K);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t T3 = (int64_t)n_tri * 3;
    CL_STAMP(0);
    // ---- compaction: ranks of the valid normals in index order, this workgroup's chunk to LDS ----
    const int R = (n_tri + KM_THREADS - 1) / KM_THREADS;  // <= 64 rounds
    // R <= 16 (n_tri <= 16 * KM_THREADS: 8192 at 512 threads; config #2 has 6272): the loaded
    // normals stay in registers and the chunk / init picks are stored from them (no second gather)
    const bool regs = R <= 16;
    uint64_t flags = 0;
    float a[16][3];
    for (int r0 = 0; r0 < R; r0 += 16) {  // 16 rounds of loads in flight before their ballots
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int i = (r0 + u) * KM_THREADS + tid;
            const bool in = r0 + u < R && i < n_tri;
#pragma unroll
            for (int q = 0; q < 3; q++) a[u][q] = in ? normals[3 * i + q] : 0.f;  // zero = invalid
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if (r0 + u >= R) break;  // uniform
            const bool v = valid_normal(a[u][0], a[u][1], a[u][2]);
            flags |= (uint64_t)v << (r0 + u);
            const uint64_t b = __ballot(v);
            if (lane == 0) L.wcnt[r0 + u][wid] = __popcll(b);
        }
    }
    __syncthreads();
    if (wid == 0) {  // exclusive scan of the R*NW counts in (round, wave) order: 4 per lane
        int v[4], sacc = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int q = 4 * lane + e;
            v[e] = q < R * NW ? (&L.wcnt[0][0])[q] : 0;
            sacc += v[e];
        }
        const int incl = wave_incl_sum_i(sacc, lane);
        int run = incl - sacc;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int q = 4 * lane + e;
            if (q < R * NW) (&L.woff[0][0])[q] = run;
            run += v[e];
        }
        if (lane == 63) L.total = incl;
    }
    __syncthreads();
    const int nv = L.total;
    const bool clustered = nv >= K;
    int m0, len;
    km_chunk(nv, m0, len);
    KmPlan plan;
    plan.p = plan_words;
    const bool plan_ok = plan.n_tri() == n_tri && plan.K() == K;
    if (!plan_ok && tid == 0) __hip_atomic_store(&ws.sync[2], 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // faiss: training set = rand_perm(seed) subsample of nv > K*256 points; nv == K is its copy corner
    // case (centroids = the points, no iteration)
    const int n_train = (plan_ok && nv > plan.cap()) ? plan.cap() : nv;
    const int niter_eff = n_train == K ? 0 : niter;
    // init picks (plan: first K of rand_perm(seed + 1)), loaded by K threads at once, then sorted
    // with their index by rank (thread k: its position = the picks below it, ties in index order —
    // the order of a stable sort; one LDS pass per thread instead of a serial insertion sort, whose
    // dependent LDS round trips cost ~5 us in one thread)
    if (clustered && tid < K) L.picki[tid] = plan_ok ? plan.init(nv, tid) : tid;
    __syncthreads();
    if (clustered && tid < K) {
        const int v = L.picki[tid];
        int rk = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int u = L.picki[j];
            rk += (u < v || (u == v && j < tid)) ? 1 : 0;
        }
        L.pick[rk] = v;
        L.pick_ord[rk] = tid;
    }
    for (int j = tid; j < len; j += KM_THREADS) L.pmem[j] = plan_ok ? plan.member(nv, m0 + j) : 1;
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int picks[K];
#pragma unroll
    for (int k = 0; k < K; k++) picks[k] = clustered ? __builtin_amdgcn_readfirstlane(L.pick[k]) : -1;
    CL_STAMP(56);
    // per-lane copies for the round loop: lane r holds round r's first rank, lane k pick k (sorted),
    // so a round's rank range is two readlanes and its picks two ballots (no LDS round trip and no
    // K-long scalar scan per round)
    const int wo_lane = lane < R ? L.woff[lane][0] : nv;
    const int pk_lane = (clustered && lane < K) ? L.pick[lane] : INT_MAX;
    auto rank_round = [&](int r, const float* ar) {
        // uniform skip of the rounds that hold neither a rank of this chunk, nor an init pick, nor
        // invalid normals this workgroup labels
        const int rlo = __builtin_amdgcn_readlane(wo_lane, r);
        const int rhi = r + 1 < R ? __builtin_amdgcn_readlane(wo_lane, r + 1) : nv;
        // the (sorted) picks inside [rlo, rhi): k in [kbeg, kend)
        const int kbeg = (int)__popcll(__ballot(pk_lane < rlo)), kend = (int)__popcll(__ballot(pk_lane < rhi));
        if (!(rlo < m0 + len && rhi > m0) && r % KM_BLOCKS != (int)blockIdx.x && kbeg == kend) return;
        const bool v = (flags >> r) & 1u;
        const int rank = L.woff[r][wid] + __popcll(__ballot(v) & lt);
        if (v) {
            const int i = r * KM_THREADS + tid;
            if (rank >= m0 && rank < m0 + len) {
                L.pidx[rank - m0] = i;
                if (ar) {
#pragma unroll
                    for (int q = 0; q < 3; q++) L.pv[q][rank - m0] = ar[q];
                }
            }
            for (int k = kbeg; k < kend; k++)  // usually none or one
                if (picks[k] == rank) {
                    L.picki[L.pick_ord[k]] = i;
                    if (ar) {
#pragma unroll
                        for (int q = 0; q < 3; q++) L.pickv[L.pick_ord[k]][q] = ar[q];
                    }
                }
        } else if (r * KM_THREADS + tid < n_tri && r % KM_BLOCKS == (int)blockIdx.x) {  // invalid: label -9, zero grad
            const int i = r * KM_THREADS + tid;
            out_labels[i] = -9;
#pragma unroll
            for (int q = 0; q < 3; q++) dn[3 * i + q] = dn[T3 + 3 * i + q] = dn[2 * T3 + 3 * i + q] = 0.f;
        }
    };
    if (regs) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            if (r < R) rank_round(r, a[r]);  // (uniform; register indices are compile-time)
    } else {
        for (int r = 0; r < R; r++) rank_round(r, nullptr);
    }
    __syncthreads();
    if (!regs)
        for (int j = tid; j < len; j += KM_THREADS) {  // this chunk's normals and the init centroids
            const int i = L.pidx[j];
#pragma unroll
            for (int q = 0; q < 3; q++) L.pv[q][j] = normals[3 * i + q];
        }
    if (clustered && tid < K) {  // faiss: centroids = the picked points, post-processed (renormalised)
        float c[3];
#pragma unroll
        for (int q = 0; q < 3; q++) c[q] = regs ? L.pickv[tid][q] : normals[3 * L.picki[tid] + q];
        if (niter_eff > 0) faiss_renorm3(c);
#pragma unroll
        for (int q = 0; q < 3; q++) L.C[tid][q] = c[q];
    }
    __syncthreads();
    CL_STAMP(1);
    unsigned phase = 0;
    const unsigned seq = __hip_atomic_load(&ws.sync[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!clustered || niter_eff == 0) {  // the buffers the Lloyd rounds do not write get void words
        const long long vw = km_tagged(km_round_tag(seq, KM_VOID_ROUND), 0);
        for (int q = tid; q < K * 4; q += KM_THREADS) {
            if (!clustered) st_c(ws.part + blockIdx.x * K * 4 + q, vw);
            st_c(ws.part + (KM_BLOCKS + blockIdx.x) * K * 4 + q, vw);
        }
    }
    if (clustered) {
        // ---- Lloyd rounds (tagged partials, no grid barrier) ----
        constexpr int NQ = K * 4;
        for (int it = 0; it <= niter_eff; it++) {
            if (it > 0) {  // (clears L.acc behind its barrier)
                km_update<K>(ws.part + ((it - 1) & 1) * KM_BLOCKS * NQ, L.C, L.upd, &L.accr[0][0], km_round_tag(seq, it - 1),
                             ws.sync, plan, n_train);
            } else {
                if (tid < NQ) {
#pragma unroll
                    for (int c = 0; c < KM_ACC_COPIES; c++) L.accr[c][tid] = 0ull;
                }
                if (tid == 0) L.upd.emp[1] = 0;  // (K * 4 <= 64: wave 1 never writes it)
                __syncthreads();
            }
            CL_STAMP(2 + 2 * it);
            // assignment + per-cluster (x, y, z, count) sums of the chunk (fixed point, LDS u64 atomics):
            // training rounds over the training set, the final search (it == niter_eff) over all points
            for (int j = tid; j < len; j += KM_THREADS) {
                const float x = L.pv[0][j], y = L.pv[1][j], z = L.pv[2][j];
                const int a = nearest<K>(L.C, x, y, z);
                L.pk[j] = a;
                if (it < niter_eff && !L.pmem[j]) continue;
                unsigned long long* ac = L.accr[lane % KM_ACC_COPIES];
                atomicAdd(&ac[4 * a], km_fixl(x));
                atomicAdd(&ac[4 * a + 1], km_fixl(y));
                atomicAdd(&ac[4 * a + 2], km_fixl(z));
                atomicAdd(&ac[4 * a + 3], (unsigned long long)KM_FXL);
            }
            __syncthreads();
            if (tid < NQ) {
                unsigned long long sum = 0ull;
#pragma unroll
                for (int c = 0; c < KM_ACC_COPIES; c++) sum += L.accr[c][tid];
                st_c(ws.part + (it & 1) * KM_BLOCKS * NQ + blockIdx.x * NQ + tid,
                     km_tagged(km_round_tag(seq, it), (long long)sum));
            }
            CL_STAMP(3 + 2 * it);
        }
        // ---- select: final cluster sizes = count column of the final-search partials ----
        if (tid < K)
            L.cnt[tid] = sum_rows_tagged(ws.part + (niter_eff & 1) * KM_BLOCKS * NQ, NQ, 4 * tid + 3,
                                         km_round_tag(seq, niter_eff), ws.sync);
        __syncthreads();
        CL_STAMP(57);
        select_clusters<K>(L.C, L.cnt, t_sim, L.sel, L.label_map);
        CL_STAMP(58);
        for (int j = tid; j < len; j += KM_THREADS) {
            const int lb = L.label_map[L.pk[j]];
            L.plab[j] = lb;
            const float sg = lb < 0 ? -1.f : 1.f;
            L.pk[j] = (lb < 0 ? -lb : lb) - 1;
            L.pv[0][j] *= sg;
            L.pv[1][j] *= sg;
            L.pv[2][j] *= sg;
        }
        if (tid < 12) L.acc[tid] = 0ull;
        __syncthreads();
        for (int j = tid; j < len; j += KM_THREADS) {
            const int c = L.pk[j];
            if (c < 0) continue;
#pragma unroll
            for (int q = 0; q < 3; q++) atomicAdd(&L.acc[4 * c + q], km_fix(L.pv[q][j]));
            atomicAdd(&L.acc[4 * c + 3], (unsigned long long)KM_FX);
        }
        __syncthreads();
        if (tid < 12) st_c(ws.p2 + blockIdx.x * 12 + tid, (long long)L.acc[tid]);
        km_grid_sync(ws.sync, ++phase);
        // ---- sums ----
        CL_STAMP(59);
        cluster_stats(ws, L.S);
        CL_STAMP(61);
        if (L.S.ok) {
            if (tid < 15) L.acc[tid] = 0ull;
            __syncthreads();
            for (int j = tid; j < len; j += KM_THREADS) {
                const int c = L.pk[j];
                if (c < 0) continue;
                const float x0 = L.pv[0][j], x1 = L.pv[1][j], x2 = L.pv[2][j];
                const float* cc = L.S.cc[c];
                atomicAdd(&L.acc[5 * c], km_fix(x0 * cc[0] + x1 * cc[1] + x2 * cc[2]));
                atomicAdd(&L.acc[5 * c + 1], km_fix(fabsf(x0 - cc[0]) + fabsf(x1 - cc[1]) + fabsf(x2 - cc[2])));
#pragma unroll
                for (int q = 0; q < 3; q++) {
                    const float u = L.pv[q][j] - cc[q];
                    atomicAdd(&L.acc[5 * c + 2 + q], km_fix(u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f)));
                }
            }
            __syncthreads();
            if (tid < 15) st_c(ws.p3 + blockIdx.x * 16 + tid, (long long)L.acc[tid]);
        }
        km_grid_sync(ws.sync, ++phase);  // uniform: S.ok is the same in every workgroup
        CL_STAMP(62);
        if (L.S.ok) sum_partials(ws.p3, 16, 15, L.st3);
        __syncthreads();
        CL_STAMP(63);
    }
    // ---- grad ----
    if (w_dev) { w_ort = w_dev[0]; w_dot = w_dev[1]; w_l1 = w_dev[2]; }
    if (step_dev) {  // losses.py:217: max(0, min(w, (step - start) * (w / grow)))
        const float ds = (float)(*step_dev) - sched_start;
        w_ort = fmaxf(0.f, fminf(w_ort, ds * (w_ort / sched_grow)));
        w_dot = fmaxf(0.f, fminf(w_dot, ds * (w_dot / sched_grow)));
        w_l1 = fmaxf(0.f, fminf(w_l1, ds * (w_l1 / sched_grow)));
    }
    // A barrier / hand-off timeout (this launch's or an earlier one's: the word is sticky until the
    // host clears it) means the partial sums may be incomplete.  The cluster terms are then dropped
    // as the reference's validity filter drops an invalid term (losses.py:246-262): losses 0, no
    // gradient, so no corrupt gradient is ever applied while the host's periodic status read
    // (losses.check_cluster_status) is pending.  Read after the last grid barrier: every flag store
    // is drained (vmcnt(0)) by the storing wave before its workgroup's next arrival, so a workgroup
    // whose data depends on a timed-out one sees the word.
    if (tid == 0) L.timed_out = (int)__hip_atomic_load(&ws.sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool ok = clustered && L.S.ok && L.timed_out == 0;
    if (blockIdx.x == 0 && tid < K * 3) out_centroids[tid] = clustered ? (&L.C[0][0])[tid] : 0.f;
    if (tid == 0) {
        float ort = 0.f, cdot = 0.f, cl1 = 0.f;
        if (ok) {
            const float(*cc)[3] = L.S.cc;
            const float d12 = cc[0][0] * cc[1][0] + cc[0][1] * cc[1][1] + cc[0][2] * cc[1][2];
            const float d13 = cc[0][0] * cc[2][0] + cc[0][1] * cc[2][1] + cc[0][2] * cc[2][2];
            const float d23 = cc[1][0] * cc[2][0] + cc[1][1] * cc[2][1] + cc[1][2] * cc[2][2];
            ort = (fabsf(d12) + fabsf(d13) + fabsf(d23)) / 3.0f;
            for (int c = 0; c < 3; c++) {
                cdot += 1.0f - L.st3[5 * c] / L.S.cnt[c];
                cl1 += L.st3[5 * c + 1] / L.S.cnt[c];
            }
            cdot /= 3.0f;
            cl1 /= 3.0f;
            // upstream gradient w.r.t. each centroid c_k, per term
            const float s12 = d12 > 0.f ? 1.f : (d12 < 0.f ? -1.f : 0.f);
            const float s13 = d13 > 0.f ? 1.f : (d13 < 0.f ? -1.f : 0.f);
            const float s23 = d23 > 0.f ? 1.f : (d23 < 0.f ? -1.f : 0.f);
            for (int q = 0; q < 3; q++) {
                const float go[3] = {(s12 * cc[1][q] + s13 * cc[2][q]) / 3.0f,
                                     (s12 * cc[0][q] + s23 * cc[2][q]) / 3.0f,
                                     (s13 * cc[0][q] + s23 * cc[1][q]) / 3.0f};
                for (int c = 0; c < 3; c++) {
                    L.G[0][c][q] = w_ort * go[c];
                    L.G[1][c][q] = (w_dot / 3.0f) * (-L.S.cm[c][q]);
                    L.G[2][c][q] = (w_l1 / 3.0f) * (-L.st3[5 * c + 2 + q] / L.S.cnt[c]);
                }
            }
            // project through c = m/|m| : dL/dm = (G - c (c.G)) / |m|, then dm/dx = 1/N
            for (int tm = 0; tm < 3; tm++)
                for (int c = 0; c < 3; c++) {
                    const float cg = cc[c][0] * L.G[tm][c][0] + cc[c][1] * L.G[tm][c][1] + cc[c][2] * L.G[tm][c][2];
                    for (int q = 0; q < 3; q++)
                        L.G[tm][c][q] = (L.G[tm][c][q] - cc[c][q] * cg) / (fmaxf(L.S.cmn[c], 1e-12f) * L.S.cnt[c]);
                }
        }
        if (blockIdx.x == 0) {
            out_losses[0] = ort; out_losses[1] = cdot; out_losses[2] = cl1; out_losses[3] = (float)nv;
            out_losses[4] = w_ort * ort; out_losses[5] = w_dot * cdot; out_losses[6] = w_l1 * cl1;
            out_losses[7] = w_ort; out_losses[8] = w_dot; out_losses[9] = w_l1;
            if (photo) {  // `total` in the order of losses.py's sum over the loss dict
                float tot = 0.f;
                tot += photo[0];
                tot += photo[1];
                tot += out_losses[4];
                tot += out_losses[5];
                tot += out_losses[6];
                out_losses[10] = tot;
            }
        }
    }
    __syncthreads();
    // per-normal label and gradient (direct terms + through the centroid), times the flip sign
    for (int j = tid; j < len; j += KM_THREADS) {
        const int i = L.pidx[j];
        const int lb = clustered ? L.plab[j] : 0;
        out_labels[i] = lb;
        const int c = clustered ? L.pk[j] : -1;
        if (!ok || c < 0) {
#pragma unroll
            for (int q = 0; q < 3; q++) dn[3 * i + q] = dn[T3 + 3 * i + q] = dn[2 * T3 + 3 * i + q] = 0.f;
            continue;
        }
        const float sg = lb < 0 ? -1.f : 1.f;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float u = L.pv[q][j] - L.S.cc[c][q];
            const float su = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
            dn[3 * i + q] = sg * L.G[0][c][q];
            dn[T3 + 3 * i + q] = sg * ((w_dot / 3.0f) * (-L.S.cc[c][q] / L.S.cnt[c]) + L.G[1][c][q]);
            dn[2 * T3 + 3 * i + q] = sg * ((w_l1 / 3.0f) * (su / L.S.cnt[c]) + L.G[2][c][q]);
        }
    }
    CL_STAMP(60);
    // every launch (clustered or not) advances the tag sequence; the last workgroup out re-reads the
    // error word and, when it is set, drops the cluster terms of the WHOLE launch (a workgroup that
    // read the word before a late timeout set it has applied its gradient rows: they are zeroed here)
    if (km_grid_exit(ws.sync)) {
        for (int64_t i = tid; i < 3 * T3; i += KM_THREADS) dn[i] = 0.f;
        if (tid == 0) {
            out_losses[0] = out_losses[1] = out_losses[2] = 0.f;
            out_losses[4] = out_losses[5] = out_losses[6] = 0.f;
            if (photo) out_losses[10] = photo[0] + photo[1];
        }
    }
}

template <int K>
static void launch_cluster(const float* normals, int n_tri, int niter, const uint32_t* plan, float t_sim, float w_ort,
                           float w_dot, float w_l1, const float* w_dev, const int64_t* step_dev, float sched_start,
                           float sched_grow, const float* photo, float* out_losses, int32_t* out_labels,
                           float* out_centroids, float* dn, float* ws, hipStream_t s) {
    hipLaunchKernelGGL(cluster_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, n_tri, niter, plan, t_sim,
                       w_ort, w_dot, w_l1, w_dev, step_dev, sched_start, sched_grow, photo, ws, out_losses, out_labels,
                       out_centroids, dn);
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int64_t ncn_cluster_workspace_words(int K) { return km_ws_words(K); }

// ---- faiss k-means plan (host) ----
static constexpr int KMP_MAX_PTS = 256;  // faiss ClusteringParameters::max_points_per_centroid
static constexpr int KMP_N_RAND = 4096;
static int64_t kmp_init_words(int n_tri, int K) { return ((int64_t)(n_tri + 1) * K + 1) / 2; }
static int64_t kmp_mask_rows(int n_tri, int K) { return std::max<int64_t>(0, n_tri - (int64_t)K * KMP_MAX_PTS); }

int64_t ncn_kmeans_plan_words(int n_tri, int K) {
    if (n_tri < 0 || K <= 0) return 0;
    return 8 + kmp_init_words(n_tri, K) + kmp_mask_rows(n_tri, K) * ((n_tri + 31) / 32) + KMP_N_RAND;
}

// faiss rand_perm(perm, n, seed) (utils/random.cpp) for its first m steps: Fisher-Yates with
// RandomGenerator::rand_int(max) = mt() % max over std::mt19937((unsigned)seed).
static void kmp_rand_perm(std::vector<int>& perm, int n, uint32_t seed, int m) {
    perm.resize(n);
    std::iota(perm.begin(), perm.end(), 0);
    std::mt19937 mt(seed);
    for (int i = 0; i < std::min(m, n - 1); i++) {
        const int i2 = i + (int)(mt() % (uint32_t)(n - i));
        std::swap(perm[i], perm[i2]);
    }
}

int ncn_kmeans_plan_fill(int n_tri, int K, uint32_t seed, uint32_t* out) {
    NCN_REQUIRE(out != nullptr && n_tri >= 0 && n_tri < 65536 && K > 0, hipErrorInvalidValue,
                "ncn_kmeans_plan_fill: bad arguments");
    const int cap = K * KMP_MAX_PTS, mw = (n_tri + 31) / 32;
    const int64_t init_off = 8, mask_off = init_off + kmp_init_words(n_tri, K);
    const int64_t rand_off = mask_off + kmp_mask_rows(n_tri, K) * mw;
    std::fill(out, out + ncn_kmeans_plan_words(n_tri, K), 0u);
    const uint32_t head[8] = {0x4B4D5031u, (uint32_t)n_tri, (uint32_t)K, (uint32_t)cap, (uint32_t)KMP_N_RAND,
                              (uint32_t)init_off, (uint32_t)mask_off, (uint32_t)rand_off};
    std::copy(head, head + 8, out);
    uint16_t* init = (uint16_t*)(out + init_off);
    std::vector<int> perm, perm1;
    kmp_rand_perm(perm1, std::max(cap, 1), seed + 1, K);  // init picks of a subsampled training set
    for (int nx = K; nx <= n_tri; nx++) {
        if (nx == K) {  // faiss's nx == k corner case: the points themselves, in order
            for (int k = 0; k < K; k++) init[(int64_t)nx * K + k] = (uint16_t)k;
        } else if (nx <= cap) {
            kmp_rand_perm(perm, nx, seed + 1, K);  // redo 0: seed + 1 + 0 * 15486557
            for (int k = 0; k < K; k++) init[(int64_t)nx * K + k] = (uint16_t)perm[k];
        } else {
            kmp_rand_perm(perm, nx, seed, cap);  // subsample_training_set
            uint32_t* mask = out + mask_off + (int64_t)(nx - cap - 1) * mw;
            for (int i = 0; i < cap; i++) mask[perm[i] >> 5] |= 1u << (perm[i] & 31);
            for (int k = 0; k < K; k++) init[(int64_t)nx * K + k] = (uint16_t)perm[perm1[k]];
        }
    }
    std::mt19937 mt(1234u);  // split_clusters: RandomGenerator rng(1234); rand_float = mt() / float(mt.max())
    for (int i = 0; i < KMP_N_RAND; i++) {
        const float r = (float)mt() / (float)mt.max();
        memcpy(out + rand_off + i, &r, 4);
    }
    return 0;
}

int64_t ncn_cluster_status_offset(int K) {
    float* base = nullptr;
    return (int64_t)((float*)(km_ws(base, K).sync + 2) - base);
}

int ncn_photo_loss_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                       float* loss, void* stream) {
    hipLaunchKernelGGL(photo_loss_fwd_kernel, dim3(1), dim3(PH_THREADS), 0, (hipStream_t)stream, rgb, rgb_gt, opacity,
                       n_rays, w_opacity, loss);
    NCN_LAUNCH_CHECK("ncn_photo_loss_fwd");
    return 0;
}

int ncn_photo_loss_bwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                       const float* loss, const float* upstream, float* dL_drgb, float* dL_dopacity, void* stream) {
    if (n_rays <= 0) return 0;
    hipLaunchKernelGGL(photo_loss_bwd_kernel, dim3(cdiv(n_rays, 256)), dim3(256), 0, (hipStream_t)stream, rgb, rgb_gt,
                       opacity, n_rays, w_opacity, loss, upstream, dL_drgb, dL_dopacity);
    NCN_LAUNCH_CHECK("ncn_photo_loss_bwd");
    return 0;
}

int ncn_photo_normals_count_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays,
                                float w_opacity, float* loss, const float* rays_o, const float* rays_d,
                                const float* depth, const int64_t* x1, const int64_t* x2, const int64_t* x3,
                                int64_t n_tri, float* normals, const int64_t* total_samples, int64_t n_count,
                                const int32_t* counter, int64_t* count_out, double* count_acc, void* stream) {
    NCN_REQUIRE(!total_samples || count_out, hipErrorInvalidValue, "ncn_photo_normals_count_fwd: count_out needed");
    const int nb0 = total_samples ? 2 : 1;
    hipLaunchKernelGGL(photo_normals_fwd_kernel, dim3(nb0 + cdiv(std::max<int64_t>(n_tri, 0), PH_THREADS)),
                       dim3(PH_THREADS), 0, (hipStream_t)stream, rgb, rgb_gt, opacity, n_rays, w_opacity, loss, rays_o,
                       rays_d, depth, x1, x2, x3, n_tri, normals, total_samples, n_count, counter, count_out,
                       count_acc);
    NCN_LAUNCH_CHECK("ncn_photo_normals_fwd");
    return 0;
}

int ncn_photo_normals_fwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays,
                          float w_opacity, float* loss, const float* rays_o, const float* rays_d, const float* depth,
                          const int64_t* x1, const int64_t* x2, const int64_t* x3, int64_t n_tri, float* normals,
                          void* stream) {
    return ncn_photo_normals_count_fwd(rgb, rgb_gt, opacity, n_rays, w_opacity, loss, rays_o, rays_d, depth, x1, x2,
                                       x3, n_tri, normals, nullptr, 0, nullptr, nullptr, nullptr, stream);
}

int ncn_normals_fwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1, const int64_t* x2,
                    const int64_t* x3, int64_t n_tri, float* normals, void* stream) {
    if (n_tri <= 0) return 0;
    hipLaunchKernelGGL(normals_fwd_kernel, dim3(cdiv(n_tri, 256)), dim3(256), 0, (hipStream_t)stream, rays_o, rays_d,
                       depth, x1, x2, x3, n_tri, normals);
    NCN_LAUNCH_CHECK("ncn_normals_fwd");
    return 0;
}

int ncn_normals_bwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1, const int64_t* x2,
                    const int64_t* x3, int64_t n_tri, const float* dL_dnormals, const float* term_weights,
                    float* dL_ddepth, void* stream) {
    if (n_tri <= 0) return 0;
    hipLaunchKernelGGL(normals_bwd_kernel, dim3(cdiv(n_tri, 256)), dim3(256), 0, (hipStream_t)stream, rays_o, rays_d,
                       depth, x1, x2, x3, n_tri, dL_dnormals, term_weights, dL_ddepth);
    NCN_LAUNCH_CHECK("ncn_normals_bwd");
    return 0;
}

int ncn_nerf_loss_bwd(const float* rgb, const float* rgb_gt, const float* opacity, int64_t n_rays, float w_opacity,
                      const float* photo_loss, const float* rays_o, const float* rays_d, const float* depth,
                      const float* dL_dnormals, const float* up_total, const float* up_terms, float* dL_drgb,
                      float* dL_dopacity, float* dL_ddepth, void* stream) {
    NCN_REQUIRE(n_rays % 64 == 0, hipErrorInvalidValue, "ncn_nerf_loss_bwd: n_rays=%lld is not whole 8x8 patches",
                (long long)n_rays);
    NCN_REQUIRE((dL_drgb == nullptr) == (dL_dopacity == nullptr), hipErrorInvalidValue,
                "ncn_nerf_loss_bwd: dL_drgb and dL_dopacity are written together (both or neither)");
    if (n_rays <= 0) return 0;
    hipLaunchKernelGGL(nerf_loss_bwd_kernel, dim3(cdiv(n_rays, 256)), dim3(256), 0, (hipStream_t)stream, rgb, rgb_gt,
                       opacity, n_rays, w_opacity, photo_loss, rays_o, rays_d, depth, dL_dnormals, up_total, up_terms,
                       dL_drgb, dL_dopacity, dL_ddepth);
    NCN_LAUNCH_CHECK("ncn_nerf_loss_bwd");
    return 0;
}

#ifdef NCN_DIAG_CL_TIMES
int ncn_diag_cl_times(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ncn_cl_times), sizeof(unsigned long long) * 64);
}
#endif

// Co-residency of the clustering kernel's KM_BLOCKS workgroups (they meet at grid barriers and
// poll each other's partials, so all of them must be resident at once): per-CU occupancy of the
// kernel (registers, LDS, waves) x the CUs left free by `busy_cus` CUs that concurrent work can
// hold entirely (the split step's rgb pass: one workgroup per CU, its LDS takes the CU).
int ncn_cluster_coresidency(int K, int busy_cus, int* capacity) {
    NCN_REQUIRE(K == 10 || K == 20, hipErrorInvalidValue, "ncn_cluster_coresidency: K must be 10 or 20 (got %d)", K);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = K == 20 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cluster_kernel<20>, KM_THREADS, 0)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cluster_kernel<10>, KM_THREADS, 0);
    NCN_REQUIRE(e == hipSuccess, e, "ncn_cluster_coresidency: device query failed (%s)", hipGetErrorString(e));
    const int cap = std::max(0, cus - std::max(0, busy_cus)) * per_cu;
    if (capacity) *capacity = cap;
    NCN_REQUIRE(cap >= KM_BLOCKS, hipErrorCooperativeLaunchTooLarge,
                "ncn_cluster_coresidency: the clustering's %d workgroups cannot all be resident: %d CUs - %d busy "
                "= %d free x %d workgroups per CU = %d", KM_BLOCKS, cus, busy_cus, std::max(0, cus - busy_cus), per_cu,
                cap);
    return 0;
}

int ncn_cluster_loss(const float* normals, int64_t n_tri, int K, int niter, const uint32_t* kmeans_plan, float t_similar,
                     float w_ort, float w_dot, float w_l1, const float* w_dev, const int64_t* step_dev,
                     float sched_start, float sched_grow, const float* photo_loss, float* out_losses,
                     int32_t* out_labels, float* out_centroids, float* dL_dnormals, float* workspace,
                     void* stream) {
    NCN_REQUIRE(n_tri >= 0 && n_tri <= CL_MAX_TRI, hipErrorInvalidValue,
                "ncn_cluster_loss: n_tri=%lld exceeds %d", (long long)n_tri, CL_MAX_TRI);
    // refuse (rather than spin into the barrier timeout) on a device that cannot hold the workgroups
    // at all; checked once per (device, K) — the answer depends on the device and on the kernel
    // instance (K sets its LDS) — and cached in an atomic (0 unknown, 1 resident, 2 refused; a racing
    // first call computes the same answer twice)
    static std::atomic<int> coresident[NCN_MAX_DEVICES][2];
    int dev = 0;
    NCN_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < NCN_MAX_DEVICES, hipErrorInvalidDevice,
                "ncn_cluster_loss: current device %d out of range", dev);
    if (K == 10 || K == 20) {
        std::atomic<int>& c = coresident[dev][K == 20];
        int v = c.load(std::memory_order_relaxed);
        if (v == 0) {
            v = ncn_cluster_coresidency(K, 0, nullptr) == 0 ? 1 : 2;
            c.store(v, std::memory_order_relaxed);
        }
        NCN_REQUIRE(v == 1, hipErrorCooperativeLaunchTooLarge,
                    "ncn_cluster_loss: the device cannot hold the clustering's %d co-resident workgroups", KM_BLOCKS);
    }
    NCN_REQUIRE(niter >= 0 && niter <= 30, hipErrorInvalidValue, "ncn_cluster_loss: niter must be in [0, 30]");
    NCN_REQUIRE(kmeans_plan != nullptr, hipErrorInvalidValue, "ncn_cluster_loss: kmeans_plan required (ncn_kmeans_plan_fill)");
    hipStream_t s = (hipStream_t)stream;
    if (K == 20)
        launch_cluster<20>(normals, (int)n_tri, niter, kmeans_plan, t_similar, w_ort, w_dot, w_l1, w_dev, step_dev, sched_start,
                           sched_grow, photo_loss, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else if (K == 10)
        launch_cluster<10>(normals, (int)n_tri, niter, kmeans_plan, t_similar, w_ort, w_dot, w_l1, w_dev, step_dev, sched_start,
                           sched_grow, photo_loss, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else
        NCN_REQUIRE(false, hipErrorInvalidValue, "ncn_cluster_loss: K must be 10 or 20 (got %d)", K);
    NCN_LAUNCH_CHECK("ncn_cluster_loss");
    return 0;
}

}  // extern "C"
