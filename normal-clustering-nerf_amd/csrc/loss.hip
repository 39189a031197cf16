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

// d/d depth through P_k = o + d*depth, a = P2-P1, b = P3-P1, c = a x b, n = c / max(|c|, eps)
__global__ void normals_bwd_kernel(const float* __restrict__ o, const float* __restrict__ d,
                                   const float* __restrict__ depth, const int64_t* __restrict__ x1,
                                   const int64_t* __restrict__ x2, const int64_t* __restrict__ x3, int64_t T,
                                   const float* __restrict__ dn, float* __restrict__ ddepth) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const int64_t i1 = x1[t], i2 = x2[t], i3 = x3[t];
    float P1[3], P2[3], P3[3];
    tri_points(o, d, depth, i1, P1);
    tri_points(o, d, depth, i2, P2);
    tri_points(o, d, depth, i3, P3);
    const float a[3] = {P2[0] - P1[0], P2[1] - P1[1], P2[2] - P1[2]};
    const float b[3] = {P3[0] - P1[0], P3[1] - P1[1], P3[2] - P1[2]};
    const float c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    const float len = sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const float g[3] = {dn[3 * t], dn[3 * t + 1], dn[3 * t + 2]};
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
    const float g2 = da[0] * d[3 * i2] + da[1] * d[3 * i2 + 1] + da[2] * d[3 * i2 + 2];
    const float g3 = db[0] * d[3 * i3] + db[1] * d[3 * i3 + 1] + db[2] * d[3 * i3 + 2];
    const float g1 = -((da[0] + db[0]) * d[3 * i1] + (da[1] + db[1]) * d[3 * i1 + 1] + (da[2] + db[2]) * d[3 * i1 + 2]);
    atomicAdd(ddepth + i1, g1);
    atomicAdd(ddepth + i2, g2);
    atomicAdd(ddepth + i3, g3);
}

// ---- clustering ----
// Pipeline (one stream, no host round trip):
//   prep  (1 WG)  : validity filter + ordered compaction (losses.py:427-430), seeded init
//   iter  (NB WGs, niter launches): C_i = update(partials_{i-1}, C_{i-1}) (i>0), assign every valid
//                   point to argmax <x, C_i>, per-workgroup partial sums (x, y, z, count) per cluster
//   final (1 WG)  : C = update(partials_last), final search, cluster selection (losses.py:75-166),
//                   flips, the three cluster losses and their analytic gradient (losses.py:441-478)
// Every workgroup recomputes the centroid update from the same partials in the same fixed order,
// so all of them hold bit-identical centroids.
constexpr int CL_THREADS = 512;      // prep + final kernels
constexpr int CL_WAVES = CL_THREADS / 64;
constexpr int CL_MAX_TRI = 16384;
constexpr int KM_THREADS = 256;      // iteration kernel
constexpr int KM_WAVES = KM_THREADS / 64;
constexpr int KM_BLOCKS = 32;

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

// Block reduction of NV per-thread values into out[NV] (fixed order: lanes, then waves).
template <int NV, int WAVES>
__device__ __forceinline__ void block_reduce(float (&v)[NV], float* red /* [WAVES][NV] */, float* out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; q++) {
        const float s = wave_sum(v[q]);
        if (lane == 0) red[wid * NV + q] = s;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < NV; q += WAVES * 64) {
        float s = 0.f;
        for (int w = 0; w < WAVES; w++) s += red[w * NV + q];
        out[q] = s;
    }
    __syncthreads();
}

// Workspace layout (32-bit words)
struct KmWs {
    int* map;        // [CL_MAX_TRI] compacted valid -> original index
    int* nv;         // [1]
    float* cent;     // [2][K][3]
    float* part;     // [2][KM_BLOCKS][K][4]
};
__host__ __device__ inline KmWs km_ws(float* base, int K) {
    KmWs w;
    w.map = (int*)base;
    w.nv = (int*)base + CL_MAX_TRI;
    w.cent = base + CL_MAX_TRI + 4;
    w.part = w.cent + 2 * K * 3;
    return w;
}
__host__ __device__ inline int64_t km_ws_words(int K) { return CL_MAX_TRI + 4 + 2 * K * 3 + 2 * KM_BLOCKS * K * 4; }

// Centroid update from the per-workgroup partials (called by ALL threads of a workgroup):
// threads sum the partials of one (cluster, component) each in fixed workgroup order, then thread 0
// forms the means, splits empty clusters from the largest (faiss: +-1/1024 on alternating
// coordinates) and L2-normalises (spherical).
template <int K>
__device__ void km_update(const float* __restrict__ part, const float* __restrict__ Cprev, float (*C)[3],
                          float* sums /* LDS [K*8] */) {
    for (int q = threadIdx.x; q < K * 4; q += blockDim.x) {
        float a = 0.f;
        for (int b = 0; b < KM_BLOCKS; b++) a += part[b * K * 4 + q];
        sums[q] = a;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float (*nc)[3] = (float (*)[3])(sums + K * 4);  // LDS scratch [K][3] + [K] after the sums
        float* cnt = sums + K * 7;
        for (int k = 0; k < K; k++) {
            cnt[k] = sums[4 * k + 3];
            for (int q = 0; q < 3; q++) nc[k][q] = cnt[k] > 0.f ? sums[4 * k + q] / cnt[k] : Cprev[3 * k + q];
        }
        const float EPS = 1.0f / 1024.0f;
        for (int k = 0; k < K; k++) {
            if (cnt[k] == 0.f) {
                int j = 0;
                for (int q = 1; q < K; q++)
                    if (cnt[q] > cnt[j]) j = q;
                for (int q = 0; q < 3; q++) {
                    if (q % 2 == 0) { nc[k][q] = nc[j][q] * (1 + EPS); nc[j][q] = nc[j][q] * (1 - EPS); }
                    else { nc[k][q] = nc[j][q] * (1 - EPS); nc[j][q] = nc[j][q] * (1 + EPS); }
                }
                const float half = floorf(cnt[j] * 0.5f);
                cnt[k] = half;
                cnt[j] -= half;
            }
        }
        for (int k = 0; k < K; k++) {
            const float nr = fmaxf(sqrtf(nc[k][0] * nc[k][0] + nc[k][1] * nc[k][1] + nc[k][2] * nc[k][2]), 1e-30f);
            for (int q = 0; q < 3; q++) C[k][q] = nc[k][q] / nr;
        }
    }
    __syncthreads();
}

template <int K>
__global__ __launch_bounds__(CL_THREADS) void cluster_prep_kernel(const float* __restrict__ normals, int n_tri,
                                                                  uint32_t seed, float* __restrict__ wsb) {
    const KmWs ws = km_ws(wsb, K);
    __shared__ int scan_w[CL_WAVES];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ch = (n_tri + CL_THREADS - 1) / CL_THREADS;
    const int b0 = tid * ch, b1 = min(n_tri, b0 + ch);
    int cnt = 0;
    for (int i = b0; i < b1; i++) cnt += valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o2 = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o2;
    }
    if (lane == 63) scan_w[wid] = incl;
    __syncthreads();
    int woff = 0, tot = 0;
    for (int w = 0; w < CL_WAVES; w++) {
        if (w < wid) woff += scan_w[w];
        tot += scan_w[w];
    }
    int pos = woff + incl - cnt;
    for (int i = b0; i < b1; i++)
        if (valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2])) ws.map[pos++] = i;
    if (tid == 0) ws.nv[0] = tot;
    __syncthreads();
    // init: one seeded pick per stratum (oracle/losses_ref.py:kmeans_init_indices)
    if (tid < K && tot >= K) {
        const int lo = (int)(((int64_t)tid * tot) / K), hi = (int)(((int64_t)(tid + 1) * tot) / K);
        const int span = max(hi - lo, 1);
        const uint32_t h = mix32(seed * 0x9E3779B1u + (uint32_t)tid * 0x85EBCA77u + 1u);
        const int i = ws.map[lo + (int)(h % (uint32_t)span)];
        for (int q = 0; q < 3; q++) ws.cent[3 * tid + q] = normals[3 * i + q];  // buffer 0 = "C_{-1}"
    }
}

template <int K>
__global__ __launch_bounds__(KM_THREADS) void kmeans_iter_kernel(const float* __restrict__ normals, int it,
                                                                 float* __restrict__ wsb) {
    const KmWs ws = km_ws(wsb, K);
    __shared__ float C[K][3];
    __shared__ float red[KM_WAVES * K * 4];
    __shared__ float outp[K * 8];
    const int nv = ws.nv[0];
    if (nv < K) return;
    const int tid = threadIdx.x;
    // centroid buffer (i & 1) holds C_i; C_0 is the prep kernel's init (buffer 0)
    if (it == 0) {
        if (tid < K * 3) (&C[0][0])[tid] = ws.cent[tid];
        __syncthreads();
    } else {
        km_update<K>(ws.part + ((it - 1) & 1) * KM_BLOCKS * K * 4, ws.cent + ((it - 1) & 1) * K * 3, C, outp);
        if (blockIdx.x == 0 && tid < K * 3) ws.cent[(it & 1) * K * 3 + tid] = (&C[0][0])[tid];
    }
    const int chunk = (nv + KM_BLOCKS - 1) / KM_BLOCKS;
    const int m0 = blockIdx.x * chunk, m1 = min(nv, m0 + chunk);
    float S[K * 4];
#pragma unroll
    for (int q = 0; q < K * 4; q++) S[q] = 0.f;
    for (int m = m0 + tid; m < m1; m += KM_THREADS) {
        const int i = ws.map[m];
        const float x = normals[3 * i], y = normals[3 * i + 1], z = normals[3 * i + 2];
        const int a = nearest<K>(C, x, y, z);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const bool h = (a == k);
            S[4 * k] += h ? x : 0.f;
            S[4 * k + 1] += h ? y : 0.f;
            S[4 * k + 2] += h ? z : 0.f;
            S[4 * k + 3] += h ? 1.f : 0.f;
        }
    }
    block_reduce<K * 4, KM_WAVES>(S, red, outp);
    float* mypart = ws.part + (it & 1) * KM_BLOCKS * K * 4 + blockIdx.x * K * 4;
    for (int q = tid; q < K * 4; q += KM_THREADS) mypart[q] = outp[q];
}

template <int K>
__global__ __launch_bounds__(CL_THREADS) void cluster_final_kernel(
    const float* __restrict__ normals, int n_tri, int niter, float t_sim, float w_ort, float w_dot, float w_l1,
    const float* __restrict__ wsb, float* __restrict__ out_losses, int32_t* __restrict__ out_labels,
    float* __restrict__ out_centroids, float* __restrict__ dn) {
    const KmWs ws = km_ws((float*)wsb, K);
    __shared__ unsigned char asg[CL_MAX_TRI];
    __shared__ float red[CL_WAVES * K];
    __shared__ float stats[K * 8];
    __shared__ float C[K][3];
    __shared__ int label_map[K];
    __shared__ float cc[3][3], cm[3][3], cmn[3], ccnt[3], G[3][3][3];  // G[term][cluster][xyz]
    __shared__ int ok_s;
    __shared__ float sim[K][K];
    const int tid = threadIdx.x;
    const int nv = ws.nv[0];
    // outputs for every triangle: invalid -> -9, zero gradient everywhere
    for (int i = tid; i < n_tri; i += CL_THREADS) {
        out_labels[i] = valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]) ? 0 : -9;
#pragma unroll
        for (int q = 0; q < 9; q++) dn[(int64_t)(q / 3) * n_tri * 3 + 3 * i + (q % 3)] = 0.f;
    }
    if (tid == 0) {
        out_losses[0] = 0.f; out_losses[1] = 0.f; out_losses[2] = 0.f; out_losses[3] = (float)nv;
        out_losses[4] = 0.f; out_losses[5] = 0.f; out_losses[6] = 0.f;
    }
    if (nv < K) return;  // too few normals to cluster (faiss would refuse); no cluster loss
    if (niter == 0) {
        if (tid < K * 3) (&C[0][0])[tid] = ws.cent[tid];
        __syncthreads();
    } else {
        km_update<K>(ws.part + ((niter - 1) & 1) * KM_BLOCKS * K * 4, ws.cent + ((niter - 1) & 1) * K * 3, C, stats);
    }
    if (tid < K * 3) out_centroids[tid] = (&C[0][0])[tid];
    // final search (losses.py:436) + cluster sizes
    {
        float S[K];
#pragma unroll
        for (int k = 0; k < K; k++) S[k] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = ws.map[m];
            const int a = nearest<K>(C, normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
            asg[m] = (unsigned char)a;
#pragma unroll
            for (int k = 0; k < K; k++) S[k] += (a == k) ? 1.f : 0.f;
        }
        block_reduce<K, CL_WAVES>(S, red, stats);
    }
    // cluster selection (losses.py:75-166) -> label of every original cluster
    if (tid == 0) {
        for (int i = 0; i < K; i++)
            for (int j = 0; j < K; j++) sim[i][j] = C[i][0] * C[j][0] + C[i][1] * C[j][1] + C[i][2] * C[j][2];
        int c1 = 0;
        for (int k = 1; k < K; k++)
            if (stats[k] > stats[c1]) c1 = k;
        float best = 0.f;
        int c2 = -1, c3 = -1;
        for (int j = 0; j < K; j++) {  // criteria[i][j] = |s(i,c1)| + |s(c1,j)| + |s(i,j)|
            float mn = 0.f;
            int mi = -1;
            for (int i = 0; i < K; i++) {
                const float cr = fabsf(sim[i][c1]) + fabsf(sim[c1][j]) + fabsf(sim[i][j]);
                if (mi < 0 || cr < mn) { mn = cr; mi = i; }
            }
            if (c2 < 0 || mn < best) { best = mn; c2 = j; c3 = mi; }
        }
        int* lab = label_map;
        for (int k = 0; k < K; k++) lab[k] = 0;
        const int cs[3] = {c1, c2, c3};
        for (int q = 0; q < 3; q++)
            for (int k = 0; k < K; k++)
                if (sim[cs[q]][k] > t_sim) lab[k] = q + 1;
        for (int q = 0; q < 3; q++) {  // opposites (losses.py:58-72, 139-163)
            int co = 0;
            for (int k = 1; k < K; k++)
                if (sim[cs[q]][k] < sim[cs[q]][co]) co = k;
            if (-1.0f * sim[cs[q]][co] > t_sim)
                for (int k = 0; k < K; k++)
                    if (sim[co][k] > t_sim) lab[k] = -(q + 1);
        }
    }
    __syncthreads();
    // flipped members, per-cluster means (losses.py:441-468)
    {
        float S[12];
#pragma unroll
        for (int q = 0; q < 12; q++) S[q] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = ws.map[m];
            const int lb = label_map[asg[m]];
            out_labels[i] = lb;
            const float sg = lb < 0 ? -1.f : 1.f;
            const int k = lb < 0 ? -lb : lb;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const bool h = (k == c + 1);
                S[4 * c] += h ? sg * normals[3 * i] : 0.f;
                S[4 * c + 1] += h ? sg * normals[3 * i + 1] : 0.f;
                S[4 * c + 2] += h ? sg * normals[3 * i + 2] : 0.f;
                S[4 * c + 3] += h ? 1.f : 0.f;
            }
        }
        block_reduce<12, CL_WAVES>(S, red, stats);
    }
    if (tid == 0) {
        int ok = 1;
        for (int c = 0; c < 3; c++) {
            ccnt[c] = stats[4 * c + 3];
            if (ccnt[c] == 0.f) ok = 0;  // mean of an empty cluster is NaN -> every term filtered (losses.py:246-262)
            for (int q = 0; q < 3; q++) cm[c][q] = ccnt[c] > 0.f ? stats[4 * c + q] / ccnt[c] : 0.f;
            const float nr = sqrtf(cm[c][0] * cm[c][0] + cm[c][1] * cm[c][1] + cm[c][2] * cm[c][2]);
            cmn[c] = nr;
            for (int q = 0; q < 3; q++) cc[c][q] = cm[c][q] / fmaxf(nr, 1e-12f);
        }
        ok_s = ok;
    }
    __syncthreads();
    if (!ok_s) return;
    // per-cluster sums of x.c, |x-c|_1 and sign(x-c)
    {
        float S[15];
#pragma unroll
        for (int q = 0; q < 15; q++) S[q] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = ws.map[m];
            const int lb = label_map[asg[m]];
            if (lb == 0) continue;
            const float sg = lb < 0 ? -1.f : 1.f;
            const int k = (lb < 0 ? -lb : lb) - 1;
            const float x[3] = {sg * normals[3 * i], sg * normals[3 * i + 1], sg * normals[3 * i + 2]};
#pragma unroll
            for (int c = 0; c < 3; c++) {
                if (c != k) continue;
                float dot = 0.f, l1 = 0.f;
#pragma unroll
                for (int q = 0; q < 3; q++) {
                    dot += x[q] * cc[c][q];
                    const float u = x[q] - cc[c][q];
                    l1 += fabsf(u);
                    S[5 * c + 2 + q] += u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
                }
                S[5 * c] += dot;
                S[5 * c + 1] += l1;
            }
        }
        block_reduce<15, CL_WAVES>(S, red, stats);
    }
    if (tid == 0) {
        const float d12 = cc[0][0] * cc[1][0] + cc[0][1] * cc[1][1] + cc[0][2] * cc[1][2];
        const float d13 = cc[0][0] * cc[2][0] + cc[0][1] * cc[2][1] + cc[0][2] * cc[2][2];
        const float d23 = cc[1][0] * cc[2][0] + cc[1][1] * cc[2][1] + cc[1][2] * cc[2][2];
        const float ort = (fabsf(d12) + fabsf(d13) + fabsf(d23)) / 3.0f;
        float cdot = 0.f, cl1 = 0.f;
        for (int c = 0; c < 3; c++) {
            cdot += 1.0f - stats[5 * c] / ccnt[c];
            cl1 += stats[5 * c + 1] / ccnt[c];
        }
        cdot /= 3.0f;
        cl1 /= 3.0f;
        out_losses[0] = ort; out_losses[1] = cdot; out_losses[2] = cl1;
        out_losses[4] = w_ort * ort; out_losses[5] = w_dot * cdot; out_losses[6] = w_l1 * cl1;
        // upstream gradient w.r.t. each centroid c_k, per term
        const float s12 = d12 > 0.f ? 1.f : (d12 < 0.f ? -1.f : 0.f);
        const float s13 = d13 > 0.f ? 1.f : (d13 < 0.f ? -1.f : 0.f);
        const float s23 = d23 > 0.f ? 1.f : (d23 < 0.f ? -1.f : 0.f);
        for (int q = 0; q < 3; q++) {
            const float go[3] = {(s12 * cc[1][q] + s13 * cc[2][q]) / 3.0f, (s12 * cc[0][q] + s23 * cc[2][q]) / 3.0f,
                                 (s13 * cc[0][q] + s23 * cc[1][q]) / 3.0f};
            for (int c = 0; c < 3; c++) {
                G[0][c][q] = w_ort * go[c];
                G[1][c][q] = (w_dot / 3.0f) * (-cm[c][q]);
                G[2][c][q] = (w_l1 / 3.0f) * (-stats[5 * c + 2 + q] / ccnt[c]);
            }
        }
        // project through c = m/|m| : dL/dm = (G - c (c.G)) / |m|, then dm/dx = 1/N
        for (int tm = 0; tm < 3; tm++)
            for (int c = 0; c < 3; c++) {
                const float cg = cc[c][0] * G[tm][c][0] + cc[c][1] * G[tm][c][1] + cc[c][2] * G[tm][c][2];
                for (int q = 0; q < 3; q++)
                    G[tm][c][q] = (G[tm][c][q] - cc[c][q] * cg) / (fmaxf(cmn[c], 1e-12f) * ccnt[c]);
            }
    }
    __syncthreads();
    // per-normal gradient (direct terms + through the centroid), times the flip sign
    for (int m = tid; m < nv; m += CL_THREADS) {
        const int i = ws.map[m];
        const int lb = label_map[asg[m]];
        if (lb == 0) continue;
        const float sg = lb < 0 ? -1.f : 1.f;
        const int c = (lb < 0 ? -lb : lb) - 1;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float x = sg * normals[3 * i + q];
            const float u = x - cc[c][q];
            const float su = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
            dn[3 * i + q] = sg * G[0][c][q];
            dn[(int64_t)n_tri * 3 + 3 * i + q] = sg * ((w_dot / 3.0f) * (-cc[c][q] / ccnt[c]) + G[1][c][q]);
            dn[(int64_t)n_tri * 6 + 3 * i + q] = sg * ((w_l1 / 3.0f) * (su / ccnt[c]) + G[2][c][q]);
        }
    }
}

template <int K>
static void launch_cluster(const float* normals, int n_tri, int niter, uint32_t seed, float t_sim, float w_ort,
                           float w_dot, float w_l1, float* out_losses, int32_t* out_labels, float* out_centroids,
                           float* dn, float* ws, hipStream_t s) {
    hipLaunchKernelGGL(cluster_prep_kernel<K>, dim3(1), dim3(CL_THREADS), 0, s, normals, n_tri, seed, ws);
    for (int it = 0; it < niter; it++)
        hipLaunchKernelGGL(kmeans_iter_kernel<K>, dim3(KM_BLOCKS), dim3(KM_THREADS), 0, s, normals, it, ws);
    hipLaunchKernelGGL(cluster_final_kernel<K>, dim3(1), dim3(CL_THREADS), 0, s, normals, n_tri, niter, t_sim, w_ort,
                       w_dot, w_l1, ws, out_losses, out_labels, out_centroids, dn);
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int64_t ncn_cluster_workspace_words(int K) { return km_ws_words(K); }

int ncn_normals_fwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1, const int64_t* x2,
                    const int64_t* x3, int64_t n_tri, float* normals, void* stream) {
    if (n_tri <= 0) return 0;
    hipLaunchKernelGGL(normals_fwd_kernel, dim3(cdiv(n_tri, 256)), dim3(256), 0, (hipStream_t)stream, rays_o, rays_d,
                       depth, x1, x2, x3, n_tri, normals);
    NCN_LAUNCH_CHECK("ncn_normals_fwd");
    return 0;
}

int ncn_normals_bwd(const float* rays_o, const float* rays_d, const float* depth, const int64_t* x1, const int64_t* x2,
                    const int64_t* x3, int64_t n_tri, const float* dL_dnormals, float* dL_ddepth, void* stream) {
    if (n_tri <= 0) return 0;
    hipLaunchKernelGGL(normals_bwd_kernel, dim3(cdiv(n_tri, 256)), dim3(256), 0, (hipStream_t)stream, rays_o, rays_d,
                       depth, x1, x2, x3, n_tri, dL_dnormals, dL_ddepth);
    NCN_LAUNCH_CHECK("ncn_normals_bwd");
    return 0;
}

int ncn_cluster_loss(const float* normals, int64_t n_tri, int K, int niter, uint32_t seed, float t_similar,
                     float w_ort, float w_dot, float w_l1, float* out_losses, int32_t* out_labels,
                     float* out_centroids, float* dL_dnormals, float* workspace, void* stream) {
    NCN_REQUIRE(n_tri >= 0 && n_tri <= CL_MAX_TRI, hipErrorInvalidValue,
                "ncn_cluster_loss: n_tri=%lld exceeds %d", (long long)n_tri, CL_MAX_TRI);
    NCN_REQUIRE(niter >= 0, hipErrorInvalidValue, "ncn_cluster_loss: niter < 0");
    hipStream_t s = (hipStream_t)stream;
    if (K == 20)
        launch_cluster<20>(normals, (int)n_tri, niter, seed, t_similar, w_ort, w_dot, w_l1, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else if (K == 10)
        launch_cluster<10>(normals, (int)n_tri, niter, seed, t_similar, w_ort, w_dot, w_l1, out_losses, out_labels,
                           out_centroids, dL_dnormals, workspace, s);
    else
        NCN_REQUIRE(false, hipErrorInvalidValue, "ncn_cluster_loss: K must be 10 or 20 (got %d)", K);
    NCN_LAUNCH_CHECK("ncn_cluster_loss");
    return 0;
}

}  // extern "C"
