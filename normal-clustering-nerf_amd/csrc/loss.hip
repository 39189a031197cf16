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
constexpr int CL_THREADS = 512;
constexpr int CL_WAVES = CL_THREADS / 64;
constexpr int CL_MAX_TRI = 16384;

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

// Block reduction of NV per-thread values into out[NV] (fixed order: lanes, then waves 0..15).
template <int NV>
__device__ __forceinline__ void block_reduce(float (&v)[NV], float* red /* [CL_WAVES][NV] */, float* out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; q++) {
        const float s = wave_sum(v[q]);
        if (lane == 0) red[wid * NV + q] = s;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < NV; q += CL_THREADS) {
        float s = 0.f;
        for (int w = 0; w < CL_WAVES; w++) s += red[w * NV + q];
        out[q] = s;
    }
    __syncthreads();
}

template <int K>
__global__ __launch_bounds__(CL_THREADS) void cluster_loss_kernel(
    const float* __restrict__ normals, int n_tri, int niter, uint32_t seed, float t_sim, float w_ort, float w_dot,
    float w_l1, float* __restrict__ out_losses, int32_t* __restrict__ out_labels, float* __restrict__ out_centroids,
    float* __restrict__ dn) {
    __shared__ int map[CL_MAX_TRI];
    __shared__ unsigned char asg[CL_MAX_TRI];
    __shared__ float red[CL_WAVES * K * 4];
    __shared__ float stats[K * 4];
    __shared__ float C[K][3];
    __shared__ int scan_w[CL_WAVES];
    __shared__ int label_map[K];
    __shared__ float cc[3][3], cm[3][3], cmn[3], ccnt[3], G[3][3][3];  // G[term][cluster][xyz]
    __shared__ int ok_s;
    __shared__ float sim[K][K], nc[K][3], cntk[K];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // 1. ordered compaction of valid normals (losses.py:427-430)
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
    for (int i = b0; i < b1; i++) {
        const bool v = valid_normal(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
        out_labels[i] = v ? 0 : -9;
#pragma unroll
        for (int q = 0; q < 9; q++) dn[(int64_t)(q / 3) * n_tri * 3 + 3 * i + (q % 3)] = 0.f;
        if (v) map[pos++] = i;
    }
    const int nv = tot;
    if (tid == 0) {
        out_losses[0] = 0.f; out_losses[1] = 0.f; out_losses[2] = 0.f; out_losses[3] = (float)nv;
    }
    __syncthreads();
    if (nv < K) return;  // too few normals to cluster (faiss would refuse); no cluster loss

    // 2. init: one seeded pick per stratum (oracle/losses_ref.py:kmeans_init_indices)
    if (tid < K) {
        const int lo = (int)(((int64_t)tid * nv) / K), hi = (int)(((int64_t)(tid + 1) * nv) / K);
        const int span = max(hi - lo, 1);
        const uint32_t h = mix32(seed * 0x9E3779B1u + (uint32_t)tid * 0x85EBCA77u + 1u);
        const int i = map[lo + (int)(h % (uint32_t)span)];
        C[tid][0] = normals[3 * i]; C[tid][1] = normals[3 * i + 1]; C[tid][2] = normals[3 * i + 2];
    }
    __syncthreads();

    // 3. Lloyd iterations (assign by max inner product, mean, split empties, L2-normalise)
    for (int it = 0; it < niter; it++) {
        float S[K * 4];
#pragma unroll
        for (int q = 0; q < K * 4; q++) S[q] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = map[m];
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
        block_reduce<K * 4>(S, red, stats);
        if (tid == 0) {
            for (int k = 0; k < K; k++) {
                cntk[k] = stats[4 * k + 3];
                for (int q = 0; q < 3; q++) nc[k][q] = cntk[k] > 0.f ? stats[4 * k + q] / cntk[k] : C[k][q];
            }
            const float EPS = 1.0f / 1024.0f;
            for (int k = 0; k < K; k++) {
                if (cntk[k] == 0.f) {
                    int j = 0;
                    for (int q = 1; q < K; q++)
                        if (cntk[q] > cntk[j]) j = q;
                    for (int q = 0; q < 3; q++) {
                        if (q % 2 == 0) { nc[k][q] = nc[j][q] * (1 + EPS); nc[j][q] = nc[j][q] * (1 - EPS); }
                        else { nc[k][q] = nc[j][q] * (1 - EPS); nc[j][q] = nc[j][q] * (1 + EPS); }
                    }
                    const float half = floorf(cntk[j] * 0.5f);
                    cntk[k] = half;
                    cntk[j] -= half;
                }
            }
            for (int k = 0; k < K; k++) {
                const float nr = fmaxf(sqrtf(nc[k][0] * nc[k][0] + nc[k][1] * nc[k][1] + nc[k][2] * nc[k][2]), 1e-30f);
                for (int q = 0; q < 3; q++) C[k][q] = nc[k][q] / nr;
            }
        }
        __syncthreads();
    }
    // final search (losses.py:436) + cluster sizes
    {
        float S[K];
#pragma unroll
        for (int k = 0; k < K; k++) S[k] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = map[m];
            const int a = nearest<K>(C, normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
            asg[m] = (unsigned char)a;
#pragma unroll
            for (int k = 0; k < K; k++) S[k] += (a == k) ? 1.f : 0.f;
        }
        block_reduce<K>(S, red, stats);
    }
    // 4. cluster selection (losses.py:75-166) -> per original cluster label
    if (tid == 0) {
        for (int i = 0; i < K; i++)
            for (int j = 0; j < K; j++) sim[i][j] = C[i][0] * C[j][0] + C[i][1] * C[j][1] + C[i][2] * C[j][2];
        int c1 = 0;
        for (int k = 1; k < K; k++)
            if (stats[k] > stats[c1]) c1 = k;
        // criteria[i][j] = |s(i,c1)| + |s(c1,j)| + |s(i,j)| ; mins over i (first), argmin over j (first)
        float best = 0.f;
        int c2 = -1, c3 = -1;
        for (int j = 0; j < K; j++) {
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
        for (int k = 0; k < K; k++)
            for (int q = 0; q < 3; q++) out_centroids[3 * k + q] = C[k][q];
    }
    __syncthreads();
    // 5. flipped members, per-cluster means (losses.py:441-468)
    {
        float S[12];
#pragma unroll
        for (int q = 0; q < 12; q++) S[q] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = map[m];
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
        block_reduce<12>(S, red, stats);
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
    // 6. per-cluster sums of x.c, |x-c|_1 and sign(x-c)
    {
        float S[15];
#pragma unroll
        for (int q = 0; q < 15; q++) S[q] = 0.f;
        for (int m = tid; m < nv; m += CL_THREADS) {
            const int i = map[m];
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
        block_reduce<15>(S, red, stats);
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
        // upstream gradient w.r.t. each centroid c_k
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
    // 7. per-normal gradient (direct terms + through the centroid), times the flip sign
    for (int m = tid; m < nv; m += CL_THREADS) {
        const int i = map[m];
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

}  // namespace ncn

using namespace ncn;

extern "C" {

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
                     float* out_centroids, float* dL_dnormals, void* stream) {
    NCN_REQUIRE(n_tri >= 0 && n_tri <= CL_MAX_TRI, hipErrorInvalidValue,
                "ncn_cluster_loss: n_tri=%lld exceeds the single-workgroup limit %d", (long long)n_tri, CL_MAX_TRI);
    NCN_REQUIRE(niter >= 0, hipErrorInvalidValue, "ncn_cluster_loss: niter < 0");
    hipStream_t s = (hipStream_t)stream;
    if (K == 20)
        hipLaunchKernelGGL(cluster_loss_kernel<20>, dim3(1), dim3(CL_THREADS), 0, s, normals, (int)n_tri, niter, seed,
                           t_similar, w_ort, w_dot, w_l1, out_losses, out_labels, out_centroids, dL_dnormals);
    else if (K == 10)
        hipLaunchKernelGGL(cluster_loss_kernel<10>, dim3(1), dim3(CL_THREADS), 0, s, normals, (int)n_tri, niter, seed,
                           t_similar, w_ort, w_dot, w_l1, out_losses, out_labels, out_centroids, dL_dnormals);
    else
        NCN_REQUIRE(false, hipErrorInvalidValue, "ncn_cluster_loss: K must be 10 or 20 (got %d)", K);
    NCN_LAUNCH_CHECK("ncn_cluster_loss");
    return 0;
}

}  // extern "C"
