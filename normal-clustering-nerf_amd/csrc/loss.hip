// Normal-clustering loss path for gfx950:
//  * normals from rendered depth over pixel triangles  (datasets/hypersim_src/utils.py:504-541)
//  * spherical k-means + Manhattan cluster selection + cluster losses and their analytic gradient
//    (losses.py:47-166, 420-478), all inside ONE workgroup so the per-step clustering needs no
//    device->host round trip (the reference copies the normals to the host for faiss, losses.py:434).
#pragma clang fp contract(off)

#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

// ---- normals: P = o + d*depth ; n = normalize(cross(P2-P1, P3-P1)) (F.normalize eps 1e-12) ----
__device__ __forceinline__ void tri_points(const float* __restrict__ o, const float* __restrict__ d,
                                           const float* __restrict__ depth, int64_t i, float P[3]) {
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = o[3 * i + k] + d[3 * i + k] * depth[i];
}

__global__ void normals_fwd_kernel(const float* __restrict__ o, const float* __restrict__ d,
                                   const float* __restrict__ depth, const int64_t* __restrict__ x1,
                                   const int64_t* __restrict__ x2, const int64_t* __restrict__ x3, int64_t T,
                                   float* __restrict__ normals) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
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
__global__ __launch_bounds__(PH_THREADS) void photo_loss_fwd_kernel(const float* __restrict__ rgb,
                                                                    const float* __restrict__ gt,
                                                                    const float* __restrict__ op, int64_t R,
                                                                    float w_op, float* __restrict__ loss) {
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
    const float ga = u[0] * photo[2], gb = u[1] * photo[3];
    const float sa = 2.f / (float)(3 * R);
#pragma unroll
    for (int c = 0; c < 3; c++) drgb[3 * ray + c] = ga == 0.f ? 0.f : ga * sa * (rgb[3 * ray + c] - gt[3 * ray + c]);
    const float oo = op[ray] + 1e-10f;
    dop[ray] = gb == 0.f ? 0.f : gb * w_op * (-(logf(oo) + 1.f)) / (float)R;
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
// Pipeline (one stream, no host round trip, every kernel but prep is KM_BLOCKS workgroups):
//   prep   (1 WG)  : validity filter + ordered compaction (losses.py:427-430), seeded init
//   iter   (niter+1 launches): C_i = update(partials_{i-1}, C_{i-1}) (i>0), assign every valid
//                    point to argmax <x, C_i>, per-workgroup partial sums (x, y, z, count) per
//                    cluster; the last launch (i = niter) is faiss's final search and keeps the
//                    assignment
//   select         : cluster selection (losses.py:75-166) -> label per point, flipped per-cluster
//                    partial sums (losses.py:441-468)
//   sums           : per-cluster partials of x.c, |x-c|_1, sign(x-c)
//   grad           : the three cluster losses, their analytic gradient per point (losses.py:469-478),
//                    labels (-9 invalid) and the zero gradient of every unselected/invalid point
// Every workgroup reduces the same partials in the same fixed order, so all of them hold
// bit-identical centroids/statistics and the result is run-to-run deterministic.
constexpr int CL_THREADS = 1024;     // prep kernel
constexpr int CL_MAX_TRI = 16384;
constexpr int KM_THREADS = 256;      // multi-workgroup kernels
constexpr int KM_BLOCKS = 32;
constexpr int KM_CHUNK_MAX = CL_MAX_TRI / KM_BLOCKS;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x = (x ^ (x >> 16)) * 0x7FEB352Du;
    x = (x ^ (x >> 15)) * 0x846CA68Bu;
    return x ^ (x >> 16);
}

__device__ __forceinline__ bool valid_normal(float a, float b, float c) {
    const bool zero = (fabsf(a) + fabsf(b) + fabsf(c)) == 0.0f;
    const bool bad = isnan(a) || isnan(b) || isnan(c) || isinf(a) || isinf(b) || isinf(c);
    return !(zero || bad);
}

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

// Workspace layout (32-bit words)
struct KmWs {
    int* map;        // [CL_MAX_TRI] compacted valid -> original index
    int* nv;         // [4]
    float* cent;     // [2][K][3]
    float* part;     // [2][KM_BLOCKS][K][4]
    int* asg;        // [CL_MAX_TRI] final assignment (compacted order)
    int* lab;        // [CL_MAX_TRI] selected label +-1..3 / 0 (compacted order)
    float* p2;       // [KM_BLOCKS][12] flipped member sums per selected cluster
    float* p3;       // [KM_BLOCKS][16] x.c, |x-c|_1, sign(x-c) sums per selected cluster
};
__host__ __device__ inline KmWs km_ws(float* base, int K) {
    KmWs w;
    w.map = (int*)base;
    w.nv = (int*)base + CL_MAX_TRI;
    w.cent = base + CL_MAX_TRI + 4;
    w.part = w.cent + 2 * K * 3;
    w.asg = (int*)(w.part + 2 * KM_BLOCKS * K * 4);
    w.lab = w.asg + CL_MAX_TRI;
    w.p2 = (float*)(w.lab + CL_MAX_TRI);
    w.p3 = w.p2 + KM_BLOCKS * 12;
    return w;
}
__host__ __device__ inline int64_t km_ws_words(int K) {
    return CL_MAX_TRI + 4 + 2 * K * 3 + 2 * KM_BLOCKS * K * 4 + 2 * CL_MAX_TRI + KM_BLOCKS * 28;
}

// This workgroup's contiguous chunk of the compacted points.
__device__ __forceinline__ void km_chunk(int nv, int& m0, int& len) {
    const int chunk = (nv + KM_BLOCKS - 1) / KM_BLOCKS;
    m0 = blockIdx.x * chunk;
    len = max(0, min(nv, m0 + chunk) - m0);
}

// Fixed-order segmented sum of NQ values over the chunk held in LDS: thread (q, seg) sums
// val(q, j) over its range of j, then NQ threads add the segments in order.  No serial wave
// reductions, deterministic.  Ends with a barrier; result in out[NQ] (LDS).
template <int NQ, class V>
__device__ __forceinline__ void chunk_sum(int len, float* segbuf /* [KM_THREADS] */, float* out, V val) {
    constexpr int SEGS = KM_THREADS / NQ;
    const int tid = threadIdx.x, q = tid % NQ, seg = tid / NQ;
    if (seg < SEGS) {
        const int lo = (seg * len) / SEGS, hi = ((seg + 1) * len) / SEGS;
        float acc = 0.f;
#pragma unroll 4
        for (int j = lo; j < hi; j++) acc += val(q, j);
        segbuf[seg * NQ + q] = acc;
    }
    __syncthreads();
    if (tid < NQ) {
        float a = 0.f;
#pragma unroll
        for (int sg = 0; sg < SEGS; sg++) a += segbuf[sg * NQ + tid];
        out[tid] = a;
    }
    __syncthreads();
}

// Sum of KM_BLOCKS partial rows (stride `row`) of `nq` values, fixed order, into out (LDS).
__device__ __forceinline__ void sum_partials(const float* __restrict__ p, int row, int nq, float* out) {
    if (threadIdx.x < nq) {
        float a = 0.f;
#pragma unroll 8
        for (int b = 0; b < KM_BLOCKS; b++) a += p[b * row + threadIdx.x];
        out[threadIdx.x] = a;
    }
}

// Centroid update from the per-workgroup partials (called by ALL threads of a workgroup): K*4
// threads sum one (cluster, component) each in fixed workgroup order, K threads form the means, a
// rare empty cluster is split from the largest one (faiss: +-1/1024 on alternating coordinates)
// by thread 0, and K threads L2-normalise (spherical k-means).
template <int K>
struct KmUpdLds {
    float sums[K * 4];
    float nc[K][3];
    float cnt[K];
    int any_empty;
};

template <int K>
__device__ void km_update(const float* __restrict__ part, const float* __restrict__ Cprev, float (*C)[3],
                          KmUpdLds<K>& L) {
    sum_partials(part, K * 4, K * 4, L.sums);
    if (threadIdx.x == 0) L.any_empty = 0;
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        const float n = L.sums[4 * k + 3];
        L.cnt[k] = n;
#pragma unroll
        for (int q = 0; q < 3; q++) L.nc[k][q] = n > 0.f ? L.sums[4 * k + q] / n : Cprev[3 * k + q];
        if (n == 0.f) L.any_empty = 1;
    }
    __syncthreads();
    if (L.any_empty && threadIdx.x == 0) {
        const float EPS = 1.0f / 1024.0f;
        for (int k = 0; k < K; k++) {
            if (L.cnt[k] == 0.f) {
                int j = 0;
                for (int q = 1; q < K; q++)
                    if (L.cnt[q] > L.cnt[j]) j = q;
                for (int q = 0; q < 3; q++) {
                    if (q % 2 == 0) { L.nc[k][q] = L.nc[j][q] * (1 + EPS); L.nc[j][q] = L.nc[j][q] * (1 - EPS); }
                    else { L.nc[k][q] = L.nc[j][q] * (1 - EPS); L.nc[j][q] = L.nc[j][q] * (1 + EPS); }
                }
                const float half = floorf(L.cnt[j] * 0.5f);
                L.cnt[k] = half;
                L.cnt[j] -= half;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        const float nr =
            fmaxf(sqrtf(L.nc[k][0] * L.nc[k][0] + L.nc[k][1] * L.nc[k][1] + L.nc[k][2] * L.nc[k][2]), 1e-30f);
#pragma unroll
        for (int q = 0; q < 3; q++) C[k][q] = L.nc[k][q] / nr;
    }
    __syncthreads();
}

// prep: ordered compaction of the valid normals with one independent load round per thread
// (thread t owns points t, t+1024, ...), ballot/popcount ranks and a 256-entry block scan.
__global__ __launch_bounds__(CL_THREADS) void cluster_prep_kernel(const float* __restrict__ normals, int n_tri,
                                                                  uint32_t seed, int K, float* __restrict__ wsb) {
    constexpr int R_MAX = CL_MAX_TRI / CL_THREADS;  // 16
    constexpr int NW = CL_THREADS / 64;             // 16
    const KmWs ws = km_ws(wsb, K);
    __shared__ int wcnt[R_MAX * NW];
    __shared__ int woff[R_MAX * NW];
    __shared__ int total;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int R = (n_tri + CL_THREADS - 1) / CL_THREADS;
    uint32_t flags = 0;
#pragma unroll
    for (int r = 0; r < R_MAX; r++) {
        const int i = r * CL_THREADS + tid;
        if (r < R && i < n_tri && valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]))
            flags |= 1u << r;
    }
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int rank[R_MAX];
#pragma unroll
    for (int r = 0; r < R_MAX; r++) {
        const uint64_t b = __ballot((flags >> r) & 1u);
        rank[r] = __popcll(b & lt);
        if (lane == 0) wcnt[r * NW + wid] = r < R ? __popcll(b) : 0;
    }
    __syncthreads();
    if (wid == 0) {  // exclusive scan of the R_MAX*NW = 256 counts in (tile, wave) order: 4 per lane
        int v[4], s = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) { v[e] = wcnt[4 * lane + e]; s += v[e]; }
        const int incl = wave_incl_sum_i(s, lane);
        int run = incl - s;
#pragma unroll
        for (int e = 0; e < 4; e++) { woff[4 * lane + e] = run; run += v[e]; }
        if (lane == 63) total = incl;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R_MAX; r++)
        if ((flags >> r) & 1u) ws.map[woff[r * NW + wid] + rank[r]] = r * CL_THREADS + tid;
    const int tot = total;
    if (tid == 0) ws.nv[0] = tot;
    __threadfence_block();
    __syncthreads();
    // init: one seeded pick per stratum (oracle/losses_ref.py:kmeans_init_indices)
    if (tid < K && tot >= K) {
        const int lo = (int)(((int64_t)tid * tot) / K), hi = (int)(((int64_t)(tid + 1) * tot) / K);
        const int span = max(hi - lo, 1);
        const uint32_t h = mix32(seed * 0x9E3779B1u + (uint32_t)tid * 0x85EBCA77u + 1u);
        const int i = ws.map[lo + (int)(h % (uint32_t)span)];
        for (int q = 0; q < 3; q++) ws.cent[3 * tid + q] = normals[3 * i + q];  // buffer 0 = "C_0"
    }
}

// One Lloyd iteration (it < niter) or the final search (it == niter, keeps the assignment).
template <int K>
__global__ __launch_bounds__(KM_THREADS) void kmeans_iter_kernel(const float* __restrict__ normals, int it,
                                                                 int final_pass, float* __restrict__ wsb) {
    constexpr int NQ = K * 4;
    const KmWs ws = km_ws(wsb, K);
    __shared__ float C[K][3];
    __shared__ float pv[4][KM_CHUNK_MAX];  // x, y, z, 1
    __shared__ int pa[KM_CHUNK_MAX];
    __shared__ float segbuf[KM_THREADS];
    __shared__ float outp[NQ];
    __shared__ KmUpdLds<K> upd;
    const int nv = ws.nv[0];
    if (nv < K) return;
    const int tid = threadIdx.x;
    int m0, len;
    km_chunk(nv, m0, len);
    // independent of the centroids: fetch this chunk's normals while the update runs
    for (int j = tid; j < len; j += KM_THREADS) {
        const int i = ws.map[m0 + j];
        pv[0][j] = normals[3 * i];
        pv[1][j] = normals[3 * i + 1];
        pv[2][j] = normals[3 * i + 2];
        pv[3][j] = 1.f;
    }
    // centroid buffer (i & 1) holds C_i; C_0 is the prep kernel's init (buffer 0)
    if (it == 0) {
        if (tid < K * 3) (&C[0][0])[tid] = ws.cent[tid];
        __syncthreads();
    } else {
        km_update<K>(ws.part + ((it - 1) & 1) * KM_BLOCKS * NQ, ws.cent + ((it - 1) & 1) * K * 3, C, upd);
        if (blockIdx.x == 0 && tid < K * 3) ws.cent[(it & 1) * K * 3 + tid] = (&C[0][0])[tid];
    }
    for (int j = tid; j < len; j += KM_THREADS) {
        const int a = nearest<K>(C, pv[0][j], pv[1][j], pv[2][j]);
        pa[j] = a;
        if (final_pass) ws.asg[m0 + j] = a;
    }
    __syncthreads();
    chunk_sum<NQ>(len, segbuf, outp, [&](int q, int j) { return pa[j] == (q >> 2) ? pv[q & 3][j] : 0.f; });
    if (tid < NQ) ws.part[(it & 1) * KM_BLOCKS * NQ + blockIdx.x * NQ + tid] = outp[tid];
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
    if (tid == 0) {
        int c2 = 0;
        for (int j = 1; j < K; j++)
            if (L.cmin[j] < L.cmin[c2]) c2 = j;
        const int c3 = L.cargmin[c2];
        for (int k = 0; k < K; k++) label_map[k] = 0;
        const int cs[3] = {c1, c2, c3};
        for (int q = 0; q < 3; q++)
            for (int k = 0; k < K; k++)
                if (L.sim[cs[q]][k] > t_sim) label_map[k] = q + 1;
        for (int q = 0; q < 3; q++) {  // opposites (losses.py:58-72, 139-163)
            int co = 0;
            for (int k = 1; k < K; k++)
                if (L.sim[cs[q]][k] < L.sim[cs[q]][co]) co = k;
            if (-1.0f * L.sim[cs[q]][co] > t_sim)
                for (int k = 0; k < K; k++)
                    if (L.sim[co][k] > t_sim) label_map[k] = -(q + 1);
        }
    }
    __syncthreads();
}

// Chunk of selected members in LDS: pk = cluster 0..2 (-1 unselected), pv = flip-signed normal.
__device__ __forceinline__ void load_members(const KmWs& ws, const float* __restrict__ normals, int m0, int len,
                                             float (*pv)[KM_CHUNK_MAX], int* pk) {
    for (int j = threadIdx.x; j < len; j += KM_THREADS) {
        const int lb = ws.lab[m0 + j];
        const int i = ws.map[m0 + j];
        const float sg = lb < 0 ? -1.f : 1.f;
        pk[j] = (lb < 0 ? -lb : lb) - 1;
        pv[0][j] = sg * normals[3 * i];
        pv[1][j] = sg * normals[3 * i + 1];
        pv[2][j] = sg * normals[3 * i + 2];
    }
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
__global__ __launch_bounds__(KM_THREADS) void cluster_select_kernel(const float* __restrict__ normals, int niter,
                                                                    float t_sim, float* __restrict__ wsb) {
    const KmWs ws = km_ws(wsb, K);
    __shared__ float C[K][3];
    __shared__ float cnt[K + 4];
    __shared__ int label_map[K];
    __shared__ SelLds<K> sel;
    __shared__ float pv[3][KM_CHUNK_MAX];
    __shared__ int pk[KM_CHUNK_MAX];
    __shared__ float segbuf[KM_THREADS];
    __shared__ float outp[12];
    const int nv = ws.nv[0];
    if (nv < K) return;
    const int tid = threadIdx.x;
    int m0, len;
    km_chunk(nv, m0, len);
    for (int j = tid; j < len; j += KM_THREADS) {
        const int i = ws.map[m0 + j];
        pk[j] = ws.asg[m0 + j];
        pv[0][j] = normals[3 * i];
        pv[1][j] = normals[3 * i + 1];
        pv[2][j] = normals[3 * i + 2];
    }
    if (tid < K * 3) (&C[0][0])[tid] = ws.cent[(niter & 1) * K * 3 + tid];
    if (tid < K) {  // final cluster sizes = count column of the final-search partials
        const float* p = ws.part + (niter & 1) * KM_BLOCKS * K * 4;
        float a = 0.f;
        for (int b = 0; b < KM_BLOCKS; b++) a += p[b * K * 4 + 4 * tid + 3];
        cnt[tid] = a;
    }
    __syncthreads();
    select_clusters<K>(C, cnt, t_sim, sel, label_map);
    for (int j = tid; j < len; j += KM_THREADS) {
        const int lb = label_map[pk[j]];
        ws.lab[m0 + j] = lb;
        const float sg = lb < 0 ? -1.f : 1.f;
        pk[j] = (lb < 0 ? -lb : lb) - 1;
        pv[0][j] *= sg;
        pv[1][j] *= sg;
        pv[2][j] *= sg;
    }
    __syncthreads();
    chunk_sum<12>(len, segbuf, outp, [&](int q, int j) {
        const int c = q >> 2, comp = q & 3;
        return pk[j] != c ? 0.f : (comp < 3 ? pv[comp][j] : 1.f);
    });
    if (tid < 12) ws.p2[blockIdx.x * 12 + tid] = outp[tid];
}

template <int K>
__global__ __launch_bounds__(KM_THREADS) void cluster_sums_kernel(const float* __restrict__ normals,
                                                                  float* __restrict__ wsb) {
    const KmWs ws = km_ws(wsb, K);
    __shared__ ClStats S;
    __shared__ float pv[3][KM_CHUNK_MAX];
    __shared__ int pk[KM_CHUNK_MAX];
    __shared__ float segbuf[KM_THREADS];
    __shared__ float outp[15];
    const int nv = ws.nv[0];
    if (nv < K) return;
    int m0, len;
    km_chunk(nv, m0, len);
    load_members(ws, normals, m0, len, pv, pk);
    cluster_stats(ws, S);
    if (!S.ok) return;
    chunk_sum<15>(len, segbuf, outp, [&](int q, int j) {
        const int c = q / 5, comp = q % 5;
        if (pk[j] != c) return 0.f;
        const float x0 = pv[0][j], x1 = pv[1][j], x2 = pv[2][j];
        if (comp == 0) return x0 * S.cc[c][0] + x1 * S.cc[c][1] + x2 * S.cc[c][2];
        if (comp == 1) return fabsf(x0 - S.cc[c][0]) + fabsf(x1 - S.cc[c][1]) + fabsf(x2 - S.cc[c][2]);
        const float u = pv[comp - 2][j] - S.cc[c][comp - 2];
        return u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
    });
    if (threadIdx.x < 15) ws.p3[blockIdx.x * 16 + threadIdx.x] = outp[threadIdx.x];
}

template <int K>
__global__ __launch_bounds__(KM_THREADS) void cluster_grad_kernel(
    const float* __restrict__ normals, int n_tri, int niter, float w_ort, float w_dot, float w_l1,
    const float* __restrict__ w_dev, const int64_t* __restrict__ step_dev, float sched_start, float sched_grow,
    const float* __restrict__ photo, const float* __restrict__ wsb, float* __restrict__ out_losses,
    int32_t* __restrict__ out_labels, float* __restrict__ out_centroids, float* __restrict__ dn) {
    const KmWs ws = km_ws((float*)wsb, K);
    if (w_dev) { w_ort = w_dev[0]; w_dot = w_dev[1]; w_l1 = w_dev[2]; }
    if (step_dev) {  // losses.py:217: max(0, min(w, (step - start) * (w / grow)))
        const float ds = (float)(*step_dev) - sched_start;
        w_ort = fmaxf(0.f, fminf(w_ort, ds * (w_ort / sched_grow)));
        w_dot = fmaxf(0.f, fminf(w_dot, ds * (w_dot / sched_grow)));
        w_l1 = fmaxf(0.f, fminf(w_l1, ds * (w_l1 / sched_grow)));
    }
    __shared__ ClStats S;
    __shared__ float st3[15];
    __shared__ float G[3][3][3];  // G[term][cluster][xyz]
    __shared__ float pv[3][KM_CHUNK_MAX];
    __shared__ int pk[KM_CHUNK_MAX];
    const int tid = threadIdx.x;
    const int nv = ws.nv[0];
    const int64_t T3 = (int64_t)n_tri * 3;
    // invalid normals (not in the compaction): label -9, zero gradient
    for (int i = blockIdx.x * KM_THREADS + tid; i < n_tri; i += KM_BLOCKS * KM_THREADS) {
        if (!valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2])) {
            out_labels[i] = -9;
#pragma unroll
            for (int q = 0; q < 3; q++) dn[3 * i + q] = dn[T3 + 3 * i + q] = dn[2 * T3 + 3 * i + q] = 0.f;
        }
    }
    int m0, len;
    km_chunk(nv, m0, len);
    const bool clustered = nv >= K;
    if (clustered) {
        load_members(ws, normals, m0, len, pv, pk);
        cluster_stats(ws, S);
        if (S.ok) sum_partials(ws.p3, 16, 15, st3);
        __syncthreads();
    }
    const bool ok = clustered && S.ok;
    if (blockIdx.x == 0 && tid < K * 3) out_centroids[tid] = clustered ? ws.cent[(niter & 1) * K * 3 + tid] : 0.f;
    if (tid == 0) {
        float ort = 0.f, cdot = 0.f, cl1 = 0.f;
        if (ok) {
            const float(*cc)[3] = S.cc;
            const float d12 = cc[0][0] * cc[1][0] + cc[0][1] * cc[1][1] + cc[0][2] * cc[1][2];
            const float d13 = cc[0][0] * cc[2][0] + cc[0][1] * cc[2][1] + cc[0][2] * cc[2][2];
            const float d23 = cc[1][0] * cc[2][0] + cc[1][1] * cc[2][1] + cc[1][2] * cc[2][2];
            ort = (fabsf(d12) + fabsf(d13) + fabsf(d23)) / 3.0f;
            for (int c = 0; c < 3; c++) {
                cdot += 1.0f - st3[5 * c] / S.cnt[c];
                cl1 += st3[5 * c + 1] / S.cnt[c];
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
                    G[0][c][q] = w_ort * go[c];
                    G[1][c][q] = (w_dot / 3.0f) * (-S.cm[c][q]);
                    G[2][c][q] = (w_l1 / 3.0f) * (-st3[5 * c + 2 + q] / S.cnt[c]);
                }
            }
            // project through c = m/|m| : dL/dm = (G - c (c.G)) / |m|, then dm/dx = 1/N
            for (int tm = 0; tm < 3; tm++)
                for (int c = 0; c < 3; c++) {
                    const float cg = cc[c][0] * G[tm][c][0] + cc[c][1] * G[tm][c][1] + cc[c][2] * G[tm][c][2];
                    for (int q = 0; q < 3; q++)
                        G[tm][c][q] = (G[tm][c][q] - cc[c][q] * cg) / (fmaxf(S.cmn[c], 1e-12f) * S.cnt[c]);
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
        const int i = ws.map[m0 + j];
        const int lb = clustered ? ws.lab[m0 + j] : 0;
        out_labels[i] = lb;
        const int c = clustered ? pk[j] : -1;
        if (!ok || c < 0) {
#pragma unroll
            for (int q = 0; q < 3; q++) dn[3 * i + q] = dn[T3 + 3 * i + q] = dn[2 * T3 + 3 * i + q] = 0.f;
            continue;
        }
        const float sg = lb < 0 ? -1.f : 1.f;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float u = pv[q][j] - S.cc[c][q];
            const float su = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
            dn[3 * i + q] = sg * G[0][c][q];
            dn[T3 + 3 * i + q] = sg * ((w_dot / 3.0f) * (-S.cc[c][q] / S.cnt[c]) + G[1][c][q]);
            dn[2 * T3 + 3 * i + q] = sg * ((w_l1 / 3.0f) * (su / S.cnt[c]) + G[2][c][q]);
        }
    }
}

template <int K>
static void launch_cluster(const float* normals, int n_tri, int niter, uint32_t seed, float t_sim, float w_ort,
                           float w_dot, float w_l1, const float* w_dev, const int64_t* step_dev, float sched_start,
                           float sched_grow, const float* photo, float* out_losses, int32_t* out_labels, float* out_centroids,
                           float* dn, float* ws, hipStream_t s) {
    hipLaunchKernelGGL(cluster_prep_kernel, dim3(1), dim3(CL_THREADS), 0, s, normals, n_tri, seed, K, ws);
    for (int it = 0; it <= niter; it++)
        hipLaunchKernelGGL(kmeans_iter_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, it,
                           (int)(it == niter), ws);
    hipLaunchKernelGGL(cluster_select_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, niter, t_sim, ws);
    hipLaunchKernelGGL(cluster_sums_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, ws);
    hipLaunchKernelGGL(cluster_grad_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, n_tri, niter, w_ort,
                       w_dot, w_l1, w_dev, step_dev, sched_start, sched_grow, photo, ws, out_losses, out_labels,
                       out_centroids, dn);
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int64_t ncn_cluster_workspace_words(int K) { return km_ws_words(K); }

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
    if (n_rays <= 0) return 0;
    hipLaunchKernelGGL(nerf_loss_bwd_kernel, dim3(cdiv(n_rays, 256)), dim3(256), 0, (hipStream_t)stream, rgb, rgb_gt,
                       opacity, n_rays, w_opacity, photo_loss, rays_o, rays_d, depth, dL_dnormals, up_total, up_terms,
                       dL_drgb, dL_dopacity, dL_ddepth);
    NCN_LAUNCH_CHECK("ncn_nerf_loss_bwd");
    return 0;
}

int ncn_cluster_loss(const float* normals, int64_t n_tri, int K, int niter, uint32_t seed, float t_similar,
                     float w_ort, float w_dot, float w_l1, const float* w_dev, const int64_t* step_dev,
                     float sched_start, float sched_grow, const float* photo_loss, float* out_losses,
                     int32_t* out_labels, float* out_centroids, float* dL_dnormals, float* workspace,
                     void* stream) {
    NCN_REQUIRE(n_tri >= 0 && n_tri <= CL_MAX_TRI, hipErrorInvalidValue,
                "ncn_cluster_loss: n_tri=%lld exceeds %d", (long long)n_tri, CL_MAX_TRI);
    NCN_REQUIRE(niter >= 0, hipErrorInvalidValue, "ncn_cluster_loss: niter < 0");
    hipStream_t s = (hipStream_t)stream;
    if (K == 20)
        launch_cluster<20>(normals, (int)n_tri, niter, seed, t_similar, w_ort, w_dot, w_l1, w_dev, step_dev, sched_start,
                           sched_grow, photo_loss, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else if (K == 10)
        launch_cluster<10>(normals, (int)n_tri, niter, seed, t_similar, w_ort, w_dot, w_l1, w_dev, step_dev, sched_start,
                           sched_grow, photo_loss, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else
        NCN_REQUIRE(false, hipErrorInvalidValue, "ncn_cluster_loss: K must be 10 or 20 (got %d)", K);
    NCN_LAUNCH_CHECK("ncn_cluster_loss");
    return 0;
}

}  // extern "C"
