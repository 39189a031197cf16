// NGPMT field for gfx950: multires hash-grid encoding (tiny-cuda-nn Grid/Hash semantics) fused
// with sigma_net (32->64->16), TruncExp, and rgb_net (cat[d/|d|, h] 19->64->64->3, Sigmoid).
// Replaces tcnn Encoding + two FullyFusedMLPs (reference models/ngp_mt.py:70-113, 157-229) and
// TruncExp (models/custom_functions.py:162-173).
//
// Layout ("transposed activations"): every layer is computed as  Y^T = W . X^T  with
// v_mfma_f32_16x16x16_f16, samples on the MFMA column (lane & 15) and features on the rows.
// The accumulator of one layer (lane (g,r) holds rows 4g..4g+3 of column r) is *exactly* the
// B-operand layout of a K=16 step of the next layer, so activations never leave registers.
// A wave owns 16 samples per step; lane (g = lane>>4, r = lane&15) encodes hash levels
// {2g, 2g+1, 8+2g, 9+2g} of sample r — i.e. the two K=16 steps of layer 1 — and in the backward
// scatters the gradient of exactly those levels.  Weights live in LDS as pre-packed fp16 MFMA
// fragments (ncn_field_pack_weights), 8 bytes per lane per fragment (ds_read_b64).
// Numerics: fp32 hash table + fp32 trilinear interpolation, fp16 MFMA operands, fp32 accumulate.
#include <algorithm>
#include <cstring>
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4_t mfma16(half4_t a, half4_t b, float4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ half4_t to_h4(float4_t v) {
    half4_t h;
    h[0] = (_Float16)v[0]; h[1] = (_Float16)v[1]; h[2] = (_Float16)v[2]; h[3] = (_Float16)v[3];
    return h;
}
__device__ __forceinline__ half4_t relu_h4(float4_t v) {
    half4_t h;
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = (_Float16)fmaxf(v[i], 0.0f);
    return h;
}
__device__ __forceinline__ float4_t zero4() { return float4_t{0.f, 0.f, 0.f, 0.f}; }

// ---- packed weight fragment table (units: fragments of 64 lanes x 4 halves = 512 B) ----
// forward (A = W, rows = out, K = in)
constexpr int F_L1 = 0;    // [t 0..3][ks 0..1]     W1[16t+r][16ks+4g+j]
constexpr int F_L2 = 8;    // [ks 0..3]             W2[r][16ks+4g+j]
constexpr int F_L3 = 12;   // [t 0..3][ks 0..1]     ks0: W3[16t+r][3+4g+j] (h), ks1: g==0&&j<3 ? W3[16t+r][j] (d)
constexpr int F_L4 = 20;   // [t 0..3][ks 0..3]     W4[16t+r][16ks+4g+j]
constexpr int F_L5 = 36;   // [ks 0..3]             r<3 ? W5[r][16ks+4g+j]
constexpr int N_FWD_FRAGS = 40;
// backward (A = W^T, rows = in, K = out)
constexpr int B_L5 = 40;   // [t 0..3]              4g+j<3 ? W5[4g+j][16t+r]
constexpr int B_L4 = 44;   // [t 0..3][ks 0..3]     W4[16ks+4g+j][16t+r]
constexpr int B_L3 = 60;   // [ks 0..3]             W3[16ks+4g+j][3+r]       (rows = h only)
constexpr int B_L2 = 64;   // [t 0..3]              W2[4g+j][16t+r]
constexpr int B_L1 = 68;   // [t 0..1][ks 0..3]     W1[16ks+4g+j][16t+r]
constexpr int N_FRAGS = 76;
static_assert(N_FRAGS * 256 == NCN_FIELD_PACKED_HALVES, "packed size");

// master weight offsets (floats) inside the concatenated fp32 buffer
constexpr int W1_OFF = 0, W2_OFF = W1_OFF + 64 * 32, W3_OFF = W2_OFF + 16 * 64, W4_OFF = W3_OFF + 64 * 19,
              W5_OFF = W4_OFF + 64 * 64, W_TOTAL = W5_OFF + 3 * 64;
static_assert(W_TOTAL == NCN_FIELD_NW, "weights size");

__device__ float frag_value(const float* __restrict__ W, int f, int lane, int j) {
    const int g = lane >> 4, r = lane & 15;
    const int k4 = 4 * g + j;
    if (f < F_L2) { const int t = (f - F_L1) >> 1, ks = (f - F_L1) & 1; return W[W1_OFF + (16 * t + r) * 32 + 16 * ks + k4]; }
    if (f < F_L3) { const int ks = f - F_L2; return W[W2_OFF + r * 64 + 16 * ks + k4]; }
    if (f < F_L4) {
        const int t = (f - F_L3) >> 1, ks = (f - F_L3) & 1;
        if (ks == 0) return W[W3_OFF + (16 * t + r) * 19 + 3 + k4];
        return (g == 0 && j < 3) ? W[W3_OFF + (16 * t + r) * 19 + j] : 0.f;
    }
    if (f < F_L5) { const int t = (f - F_L4) >> 2, ks = (f - F_L4) & 3; return W[W4_OFF + (16 * t + r) * 64 + 16 * ks + k4]; }
    if (f < B_L5) { const int ks = f - F_L5; return r < 3 ? W[W5_OFF + r * 64 + 16 * ks + k4] : 0.f; }
    if (f < B_L4) { const int t = f - B_L5; return k4 < 3 ? W[W5_OFF + k4 * 64 + 16 * t + r] : 0.f; }
    if (f < B_L3) { const int t = (f - B_L4) >> 2, ks = (f - B_L4) & 3; return W[W4_OFF + (16 * ks + k4) * 64 + 16 * t + r]; }
    if (f < B_L2) { const int ks = f - B_L3; return W[W3_OFF + (16 * ks + k4) * 19 + 3 + r]; }
    if (f < B_L1) { const int t = f - B_L2; return W[W2_OFF + k4 * 64 + 16 * t + r]; }
    const int t = (f - B_L1) >> 2, ks = (f - B_L1) & 3;
    return W[W1_OFF + (16 * ks + k4) * 32 + 16 * t + r];
}

__global__ void pack_weights_kernel(const float* __restrict__ W, _Float16* __restrict__ out) {
    const int f = blockIdx.x, lane = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; j++) out[(f * 64 + lane) * 4 + j] = (_Float16)frag_value(W, f, lane, j);
}

// ---- hash grid ----
struct LevelTable {
    float scale[16];
    uint32_t res[16], params[16], offset[16];
};

// tiny-cuda-nn grid_index (dense stride while it fits, else coherent prime hash) % params
__device__ __forceinline__ uint32_t grid_index(uint32_t params, uint32_t res, uint32_t x, uint32_t y, uint32_t z) {
    uint32_t stride = 1, index = 0;
    if (stride <= params) { index += x * stride; stride *= res; }
    if (stride <= params) { index += y * stride; stride *= res; }
    if (stride <= params) { index += z * stride; stride *= res; }
    if (params < stride) index = x ^ (y * 2654435761u) ^ (z * 805459861u);
    return index % params;
}

struct LevelPos {
    uint32_t px, py, pz;
    float fx, fy, fz;
};
__device__ __forceinline__ LevelPos level_pos(float scale, float x, float y, float z) {
    LevelPos p;
    float a = fmaf(scale, x, 0.5f), b = fmaf(scale, y, 0.5f), c = fmaf(scale, z, 0.5f);
    const float fa = floorf(a), fb = floorf(b), fc = floorf(c);
    p.px = (uint32_t)(int)fa; p.py = (uint32_t)(int)fb; p.pz = (uint32_t)(int)fc;
    p.fx = a - fa; p.fy = b - fb; p.fz = c - fc;
    return p;
}

// trilinear interpolation of one level (tcnn kernel_grid: corner bit d -> +1 along dim d)
__device__ __forceinline__ float2 encode_level(const float2* __restrict__ tab, const LevelTable& L, int l, float x,
                                               float y, float z) {
    const LevelPos p = level_pos(L.scale[l], x, y, z);
    const uint32_t params = L.params[l], res = L.res[l], off = L.offset[l];
    float2 v[8];
    float w[8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const uint32_t cx = p.px + (c & 1), cy = p.py + ((c >> 1) & 1), cz = p.pz + ((c >> 2) & 1);
        v[c] = tab[off + grid_index(params, res, cx, cy, cz)];
        float wt = 1.0f;
        wt *= (c & 1) ? p.fx : 1.0f - p.fx;
        wt *= (c & 2) ? p.fy : 1.0f - p.fy;
        wt *= (c & 4) ? p.fz : 1.0f - p.fz;
        w[c] = wt;
    }
    float2 acc = make_float2(0.f, 0.f);
#pragma unroll
    for (int c = 0; c < 8; c++) {
        acc.x = fmaf(w[c], v[c].x, acc.x);
        acc.y = fmaf(w[c], v[c].y, acc.y);
    }
    return acc;
}

// Backward scatter of one level for the 16 samples of a lane group (lanes 16g..16g+15 hold 16
// consecutive samples, i.e. mostly consecutive points of one ray).
//  1. Runs: lanes whose samples fall in the same base cell form runs; a segmented suffix sum over
//     each run (4 doubling steps with DPP row shifts inside the 16-lane row) leaves the run total in
//     its head lane.  At the coarse levels a group usually shares one cell: up to 16x fewer atomics
//     on the few thousand hot entries.
//  2. Coalescing: the two corners that differ only in x (tcnn's hash multiplies x by 1, so their
//     entries are adjacent for dense levels and share a 64-B line 7/8 of the time for hashed ones)
//     x 2 features = 16 contiguous bytes.  A quad of lanes takes one source lane's 4 values
//     (quad_perm broadcast), so each f32-atomic instruction touches ~16 lines instead of 64:
//     scattered single-lane atomics run ~17x below the coalesced atomic rate on MI355X.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_ROW_SL(int k) { return 0x100 + k; }  // dst[r] = src[r+k] inside a 16-lane row
constexpr int DPP_ROW_SR(int k) { return 0x110 + k; }  // dst[r] = src[r-k]
constexpr int DPP_QUAD_BCAST(int t) { return t * 0x55; }  // quad_perm [t,t,t,t]

template <int K>
__device__ __forceinline__ void run_sum(float& v, const int (&link)[4]) {
    const float t = dppf<DPP_ROW_SL(1 << K)>(v);
    if (link[K]) v += t;
}

template <int T>
__device__ __forceinline__ void quad_atomics(float* __restrict__ grad, int j, bool head, const float (&V)[4],
                                             uint32_t i0, uint32_t i1) {
    const int bh = dppi<DPP_QUAD_BCAST(T)>((int)head);
    const float b0 = dppf<DPP_QUAD_BCAST(T)>(V[0]), b1 = dppf<DPP_QUAD_BCAST(T)>(V[1]);
    const float b2 = dppf<DPP_QUAD_BCAST(T)>(V[2]), b3 = dppf<DPP_QUAD_BCAST(T)>(V[3]);
    const uint32_t e0 = (uint32_t)dppi<DPP_QUAD_BCAST(T)>((int)i0), e1 = (uint32_t)dppi<DPP_QUAD_BCAST(T)>((int)i1);
    const float val = j == 0 ? b0 : (j == 1 ? b1 : (j == 2 ? b2 : b3));
    const uint32_t e = j < 2 ? e0 : e1;
    if (bh) atomicAdd(grad + 2 * (size_t)e + (j & 1), val);
}

__device__ __forceinline__ void scatter_level(float* __restrict__ grad, const LevelTable& L, int l, float x, float y,
                                              float z, float g0, float g1, bool valid, int r, int lane) {
    const LevelPos p = level_pos(L.scale[l], x, y, z);
    const uint32_t params = L.params[l], res = L.res[l], off = L.offset[l];
    // run structure from the base cell (a sample outside [0,n) gets a key no valid sample has)
    const int key = valid ? (int)(p.px + res * (p.py + res * p.pz)) : (int)(0xFFFFFFF0u - (uint32_t)r);
    const int key_next = dppi<DPP_ROW_SL(1)>(key);
    const int key_prev = dppi<DPP_ROW_SR(1)>(key);
    int link[4];
    link[0] = (r < 15) && (key_next == key);
    link[1] = link[0] && dppi<DPP_ROW_SL(1)>(link[0]);
    link[2] = link[1] && dppi<DPP_ROW_SL(2)>(link[1]);
    link[3] = link[2] && dppi<DPP_ROW_SL(4)>(link[2]);
    const bool head = valid && (r == 0 || key_prev != key);
    const int j = lane & 3;
#pragma unroll
    for (int cp = 0; cp < 4; cp++) {  // corner pair: (x, x+1) at (y + (cp&1), z + (cp>>1))
        const uint32_t cy = p.py + (cp & 1), cz = p.pz + (cp >> 1);
        const float wy = (cp & 1) ? p.fy : 1.0f - p.fy;
        const float wz = (cp & 2) ? p.fz : 1.0f - p.fz;
        const float w0 = ((1.0f - p.fx) * wy) * wz, w1 = (p.fx * wy) * wz;
        float V[4] = {valid ? w0 * g0 : 0.f, valid ? w0 * g1 : 0.f, valid ? w1 * g0 : 0.f, valid ? w1 * g1 : 0.f};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            run_sum<0>(V[q], link);
            run_sum<1>(V[q], link);
            run_sum<2>(V[q], link);
            run_sum<3>(V[q], link);
        }
        const uint32_t i0 = off + grid_index(params, res, p.px, cy, cz);
        const uint32_t i1 = off + grid_index(params, res, p.px + 1, cy, cz);
        quad_atomics<0>(grad, j, head, V, i0, i1);
        quad_atomics<1>(grad, j, head, V, i0, i1);
        quad_atomics<2>(grad, j, head, V, i0, i1);
        quad_atomics<3>(grad, j, head, V, i0, i1);
    }
}

__device__ __forceinline__ half4_t frag(const half4_t* __restrict__ lds_frags, int f, int lane) {
    return lds_frags[f * 64 + lane];
}

// Shared per-group forward (16 samples).  Produces every intermediate the backward needs.
struct FwdState {
    half4_t x2[4];     // relu(H1) tiles (B operands of L2)
    float4_t h;        // sigma_net output tile (rows 4g..4g+3)
    half4_t x3h, x3d;  // L3 B operands (h tile, d tile)
    half4_t x4[4];     // relu(G1)
    half4_t x5[4];     // relu(G2)
    float4_t out;      // rgb pre-activation tile (rows 0..2 valid on g==0)
    uint32_t m1, m3, m4;  // relu masks: bit (4t+i)
};

__device__ __forceinline__ void mlp_sigma(const half4_t* F, int lane, half4_t e0, half4_t e1, FwdState& st) {
    st.m1 = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
        acc = mfma16(frag(F, F_L1 + 2 * t, lane), e0, acc);
        acc = mfma16(frag(F, F_L1 + 2 * t + 1, lane), e1, acc);
        st.x2[t] = relu_h4(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) st.m1 |= (acc[i] > 0.f ? 1u : 0u) << (4 * t + i);
    }
    float4_t h = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ks++) h = mfma16(frag(F, F_L2 + ks, lane), st.x2[ks], h);
    st.h = h;
}

__device__ __forceinline__ void mlp_rgb(const half4_t* F, int lane, float dnx, float dny, float dnz, FwdState& st) {
    const int g = lane >> 4;
    st.x3h = to_h4(st.h);
    half4_t xd;
    xd[0] = (_Float16)(g == 0 ? dnx : 0.f);
    xd[1] = (_Float16)(g == 0 ? dny : 0.f);
    xd[2] = (_Float16)(g == 0 ? dnz : 0.f);
    xd[3] = (_Float16)0.f;
    st.x3d = xd;
    st.m3 = 0;
    st.m4 = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
        acc = mfma16(frag(F, F_L3 + 2 * t, lane), st.x3h, acc);
        acc = mfma16(frag(F, F_L3 + 2 * t + 1, lane), st.x3d, acc);
        st.x4[t] = relu_h4(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) st.m3 |= (acc[i] > 0.f ? 1u : 0u) << (4 * t + i);
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
#pragma unroll
        for (int ks = 0; ks < 4; ks++) acc = mfma16(frag(F, F_L4 + 4 * t + ks, lane), st.x4[ks], acc);
        st.x5[t] = relu_h4(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) st.m4 |= (acc[i] > 0.f ? 1u : 0u) << (4 * t + i);
    }
    float4_t o = zero4();
#pragma unroll
    for (int ks = 0; ks < 4; ks++) o = mfma16(frag(F, F_L5 + ks, lane), st.x5[ks], o);
    st.out = o;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ void load_levels(LevelTable& Ls, const LevelTable& La) {
    if (threadIdx.x < 16) {
        const int l = threadIdx.x;
        Ls.scale[l] = La.scale[l];
        Ls.res[l] = La.res[l];
        Ls.params[l] = La.params[l];
        Ls.offset[l] = La.offset[l];
    }
}

// ---------------------------------------------------------------------------------------------
// Forward: grid-stride over 16-sample groups, one group per wave per step.
__global__ __launch_bounds__(256) void field_fwd_kernel(const float* __restrict__ xyzs, const float* __restrict__ dirs,
                                                        int64_t n, const float2* __restrict__ table, LevelTable Lt,
                                                        float xyz_min, float xyz_extent,
                                                        const half4_t* __restrict__ wpacked, int mode,
                                                        float* __restrict__ sigmas, float* __restrict__ rgbs,
                                                        half4_t* __restrict__ enc_cache) {
    __shared__ half4_t F[N_FWD_FRAGS * 64];
    __shared__ LevelTable L;
    for (int i = threadIdx.x; i < N_FWD_FRAGS * 64; i += 256) F[i] = wpacked[i];
    load_levels(L, Lt);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
    const int64_t n_groups = (n + 15) / 16;
    const int64_t wave0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
        const int64_t s = grp * 16 + r;
        const bool valid = s < n;
        float x = 0.f, y = 0.f, z = 0.f;
        if (valid) {
            x = (xyzs[3 * s] - xyz_min) / xyz_extent;
            y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
            z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
        }
        const float2 e00 = encode_level(table, L, 2 * g, x, y, z);
        const float2 e01 = encode_level(table, L, 2 * g + 1, x, y, z);
        const float2 e10 = encode_level(table, L, 8 + 2 * g, x, y, z);
        const float2 e11 = encode_level(table, L, 9 + 2 * g, x, y, z);
        half4_t b0, b1;
        b0[0] = (_Float16)e00.x; b0[1] = (_Float16)e00.y; b0[2] = (_Float16)e01.x; b0[3] = (_Float16)e01.y;
        b1[0] = (_Float16)e10.x; b1[1] = (_Float16)e10.y; b1[2] = (_Float16)e11.x; b1[3] = (_Float16)e11.y;
        if (enc_cache) {
            enc_cache[(grp * 2 + 0) * 64 + lane] = b0;
            enc_cache[(grp * 2 + 1) * 64 + lane] = b1;
        }
        FwdState st;
        mlp_sigma(F, lane, b0, b1, st);
        if (g == 0 && valid) sigmas[s] = __expf(st.h[0]);  // TruncExp forward = exp
        if (mode == 1) continue;
        float dx = 0.f, dy = 0.f, dz = 0.f;
        if (valid) {
            dx = dirs[3 * s]; dy = dirs[3 * s + 1]; dz = dirs[3 * s + 2];
            const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
            dx /= nrm; dy /= nrm; dz /= nrm;
        }
        mlp_rgb(F, lane, dx, dy, dz, st);
        if (g == 0 && valid) {
            rgbs[3 * s] = sigmoidf_(st.out[0]);
            rgbs[3 * s + 1] = sigmoidf_(st.out[1]);
            rgbs[3 * s + 2] = sigmoidf_(st.out[2]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Backward.  Per 16-sample group: recompute the MLP forward from the cached encoding, back-
// propagate through the five layers (transposed products with the W^T fragments), scatter the
// encoding gradient of this lane's four levels into the fp32 table gradient with no-return f32
// atomics, and accumulate dW = sum_s dY_s X_s^T over the wave's groups in 40 register tiles.
// The dW MFMAs need samples on K: each C-layout tile is transposed through a wave-private
// 512-byte LDS slot (4 x ds_write_b16, 1 x ds_read_b64).  At the end the four waves reduce their
// tiles into LDS and the workgroup writes one fp32 slab row (reduced in a fixed order later).
constexpr int BWD_THREADS = 256;

struct WGrad {
    float4_t w1[4][2], w2[4], w3[4][2], w4[4][4], w5[4];
};

__device__ __forceinline__ half4_t transpose_tile(_Float16* slot, int lane, float4_t v) {
    const int g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; i++) slot[(4 * g + i) * 16 + r] = (_Float16)v[i];
    __builtin_amdgcn_wave_barrier();
    const half4_t out = *(const half4_t*)(slot + r * 16 + 4 * g);
    __builtin_amdgcn_wave_barrier();
    return out;
}
__device__ __forceinline__ half4_t transpose_tile_h(_Float16* slot, int lane, half4_t v) {
    const int g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; i++) slot[(4 * g + i) * 16 + r] = v[i];
    __builtin_amdgcn_wave_barrier();
    const half4_t out = *(const half4_t*)(slot + r * 16 + 4 * g);
    __builtin_amdgcn_wave_barrier();
    return out;
}

__global__ __launch_bounds__(BWD_THREADS) void field_bwd_kernel(
    const float* __restrict__ xyzs, const float* __restrict__ dirs, int64_t n, LevelTable Lt, float xyz_min,
    float xyz_extent, const half4_t* __restrict__ wpacked, const half4_t* __restrict__ enc_cache,
    const float* __restrict__ dL_dsig, const float* __restrict__ dL_drgb, float* __restrict__ grad_table,
    float* __restrict__ slab) {
    // One LDS arena: [fragments | transpose slots] during the loop, reused as the fp32 dW
    // reduction buffer afterwards (43 KB total -> several workgroups per CU).
    constexpr int FRAG_BYTES = N_FRAGS * 64 * 8, SLOT_BYTES = 4 * 2 * 256 * 2;
    static_assert(FRAG_BYTES + SLOT_BYTES >= NCN_FIELD_NW * 4, "arena too small for the dW reduction");
    __shared__ __attribute__((aligned(16))) char arena[FRAG_BYTES + SLOT_BYTES];
    __shared__ LevelTable L;
    half4_t* F = (half4_t*)arena;
    _Float16* tslots = (_Float16*)(arena + FRAG_BYTES);
    float* red = (float*)arena;
    for (int i = threadIdx.x; i < N_FRAGS * 64; i += BWD_THREADS) F[i] = wpacked[i];
    load_levels(L, Lt);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15, wid = threadIdx.x >> 6;
    _Float16* sA = tslots + wid * 512;
    _Float16* sB = tslots + wid * 512 + 256;
    WGrad acc;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        acc.w2[a] = zero4(); acc.w5[a] = zero4();
#pragma unroll
        for (int b = 0; b < 2; b++) { acc.w1[a][b] = zero4(); acc.w3[a][b] = zero4(); }
#pragma unroll
        for (int b = 0; b < 4; b++) acc.w4[a][b] = zero4();
    }
    const int64_t n_groups = (n + 15) / 16;
    const int64_t wave0 = (int64_t)blockIdx.x * 4 + wid;
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
        const int64_t s = grp * 16 + r;
        const bool valid = s < n;
        const half4_t e0 = enc_cache[(grp * 2 + 0) * 64 + lane];
        const half4_t e1 = enc_cache[(grp * 2 + 1) * 64 + lane];
        float dx = 0.f, dy = 0.f, dz = 0.f, dsig = 0.f, dr0 = 0.f, dr1 = 0.f, dr2 = 0.f;
        if (valid) {
            dx = dirs[3 * s]; dy = dirs[3 * s + 1]; dz = dirs[3 * s + 2];
            const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
            dx /= nrm; dy /= nrm; dz /= nrm;
            dsig = dL_dsig ? dL_dsig[s] : 0.f;
            if (dL_drgb) { dr0 = dL_drgb[3 * s]; dr1 = dL_drgb[3 * s + 1]; dr2 = dL_drgb[3 * s + 2]; }
        }
        FwdState st;
        mlp_sigma(F, lane, e0, e1, st);
        mlp_rgb(F, lane, dx, dy, dz, st);
        // dY5: d(pre-sigmoid) = drgb * s(1-s), rows 0..2 on g==0
        float4_t dy5 = zero4();
        if (g == 0) {
            const float s0 = sigmoidf_(st.out[0]), s1 = sigmoidf_(st.out[1]), s2 = sigmoidf_(st.out[2]);
            dy5[0] = dr0 * s0 * (1.f - s0);
            dy5[1] = dr1 * s1 * (1.f - s1);
            dy5[2] = dr2 * s2 * (1.f - s2);
        }
        const half4_t dy5h = to_h4(dy5);
        // L5 backward -> dG2, masked -> dD4
        float4_t dD4[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            float4_t v = mfma16(frag(F, B_L5 + t, lane), dy5h, zero4());
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = ((st.m4 >> (4 * t + i)) & 1u) ? v[i] : 0.f;
            dD4[t] = v;
        }
        half4_t dD4h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) dD4h[t] = to_h4(dD4[t]);
        // L4 backward -> dG1 -> dD3
        float4_t dD3[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            float4_t v = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ks++) v = mfma16(frag(F, B_L4 + 4 * t + ks, lane), dD4h[ks], v);
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = ((st.m3 >> (4 * t + i)) & 1u) ? v[i] : 0.f;
            dD3[t] = v;
        }
        half4_t dD3h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) dD3h[t] = to_h4(dD3[t]);
        // L3 backward -> dh (rgb path) ; + TruncExp backward on h[0]
        float4_t dh = zero4();
#pragma unroll
        for (int ks = 0; ks < 4; ks++) dh = mfma16(frag(F, B_L3 + ks, lane), dD3h[ks], dh);
        if (g == 0) dh[0] += dsig * __expf(fminf(fmaxf(st.h[0], -15.f), 15.f));
        const half4_t dhh = to_h4(dh);
        // L2 backward -> dH1 -> dD1
        half4_t dD1h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            float4_t v = mfma16(frag(F, B_L2 + t, lane), dhh, zero4());
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = ((st.m1 >> (4 * t + i)) & 1u) ? v[i] : 0.f;
            dD1h[t] = to_h4(v);
        }
        // L1 backward -> dE (tile t holds levels 8t+2g, 8t+2g+1)
        float4_t dE[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            float4_t v = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ks++) v = mfma16(frag(F, B_L1 + 4 * t + ks, lane), dD1h[ks], v);
            dE[t] = v;
        }
        {
            float x = 0.f, y = 0.f, z = 0.f;
            if (valid) {
                x = (xyzs[3 * s] - xyz_min) / xyz_extent;
                y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
                z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
            }
            scatter_level(grad_table, L, 2 * g, x, y, z, dE[0][0], dE[0][1], valid, r, lane);
            scatter_level(grad_table, L, 2 * g + 1, x, y, z, dE[0][2], dE[0][3], valid, r, lane);
            scatter_level(grad_table, L, 8 + 2 * g, x, y, z, dE[1][0], dE[1][1], valid, r, lane);
            scatter_level(grad_table, L, 9 + 2 * g, x, y, z, dE[1][2], dE[1][3], valid, r, lane);
        }
        // ---- weight gradients: dW[out][in] += sum_s dY[out][s] X[in][s] ----
        // A operand = dY^T rows (out, lane r) over K = samples; B operand = X over K = samples.
        {   // L5: dY = dy5 (1 out tile), X = x5 (4 in tiles)
            const half4_t A = transpose_tile(sA, lane, dy5);
#pragma unroll
            for (int b = 0; b < 4; b++) acc.w5[b] = mfma16(A, transpose_tile_h(sB, lane, st.x5[b]), acc.w5[b]);
        }
        {   // L4: dY = dD4 (4 out tiles), X = x4 (4 in tiles)
            half4_t Xt[4];
#pragma unroll
            for (int b = 0; b < 4; b++) Xt[b] = transpose_tile_h(sB, lane, st.x4[b]);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile(sA, lane, dD4[a]);
#pragma unroll
                for (int b = 0; b < 4; b++) acc.w4[a][b] = mfma16(A, Xt[b], acc.w4[a][b]);
            }
        }
        {   // L3: dY = dD3 (4 out tiles), X = [d | h] : in tile 0 = d (cols 0..2), tile 1 = h (cols 3..18)
            const half4_t Xd = transpose_tile_h(sB, lane, st.x3d);
            const half4_t Xh = transpose_tile_h(sB, lane, st.x3h);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile(sA, lane, dD3[a]);
                acc.w3[a][0] = mfma16(A, Xd, acc.w3[a][0]);
                acc.w3[a][1] = mfma16(A, Xh, acc.w3[a][1]);
            }
        }
        {   // L2: dY = dh (1 out tile), X = x2 (4 in tiles)
            const half4_t A = transpose_tile(sA, lane, dh);
#pragma unroll
            for (int b = 0; b < 4; b++) acc.w2[b] = mfma16(A, transpose_tile_h(sB, lane, st.x2[b]), acc.w2[b]);
        }
        {   // L1: dY = dD1 (4 out tiles), X = e (2 in tiles)
            const half4_t X0 = transpose_tile_h(sB, lane, e0);
            const half4_t X1 = transpose_tile_h(sB, lane, e1);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile_h(sA, lane, dD1h[a]);
                acc.w1[a][0] = mfma16(A, X0, acc.w1[a][0]);
                acc.w1[a][1] = mfma16(A, X1, acc.w1[a][1]);
            }
        }
    }
    // ---- workgroup reduction of the 40 tiles into LDS (C layout: row 4g+i, col r) ----
    __syncthreads();  // every wave is done with the fragments / slots: reuse the arena
    for (int i = threadIdx.x; i < NCN_FIELD_NW; i += BWD_THREADS) red[i] = 0.f;
    __syncthreads();
    // W1 [64][32]
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) atomicAdd(&red[W1_OFF + (16 * a + 4 * g + i) * 32 + 16 * b + r], acc.w1[a][b][i]);
    // W2 [16][64]
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
        for (int i = 0; i < 4; i++) atomicAdd(&red[W2_OFF + (4 * g + i) * 64 + 16 * b + r], acc.w2[b][i]);
    // W3 [64][19]: in tile 0 -> cols 0..2 (d), in tile 1 -> cols 3..18 (h)
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (r < 3) atomicAdd(&red[W3_OFF + (16 * a + 4 * g + i) * 19 + r], acc.w3[a][0][i]);
            atomicAdd(&red[W3_OFF + (16 * a + 4 * g + i) * 19 + 3 + r], acc.w3[a][1][i]);
        }
    // W4 [64][64]
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) atomicAdd(&red[W4_OFF + (16 * a + 4 * g + i) * 64 + 16 * b + r], acc.w4[a][b][i]);
    // W5 [3][64]
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (4 * g + i < 3) atomicAdd(&red[W5_OFF + (4 * g + i) * 64 + 16 * b + r], acc.w5[b][i]);
    __syncthreads();
    float* out = slab + (int64_t)blockIdx.x * NCN_FIELD_NW;
    for (int i = threadIdx.x; i < NCN_FIELD_NW; i += BWD_THREADS) out[i] = red[i];
}

// Sum of the per-workgroup dW slabs: blockIdx.y takes a chunk of slabs (coalesced 1 KB rows),
// chunk partials are added with f32 atomics (gw accumulates, like every .grad).
constexpr int WRED_CHUNK = 16;
__global__ void reduce_wgrad_kernel(const float* __restrict__ slab, int nb, float* __restrict__ gw) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= NCN_FIELD_NW) return;
    const int b0 = blockIdx.y * WRED_CHUNK, b1 = min(nb, b0 + WRED_CHUNK);
    float s = 0.f;
    for (int b = b0; b < b1; b++) s += slab[(int64_t)b * NCN_FIELD_NW + i];
    atomicAdd(gw + i, s);
}

static LevelTable make_table(const uint32_t* levels) {
    LevelTable t;
    for (int l = 0; l < 16; l++) {
        memcpy(&t.scale[l], &levels[4 * l], 4);
        t.res[l] = levels[4 * l + 1];
        t.params[l] = levels[4 * l + 2];
        t.offset[l] = levels[4 * l + 3];
    }
    return t;
}

static int fwd_grid(int64_t n) {
    const int64_t groups = (n + 15) / 16;
    return (int)std::min<int64_t>(std::max<int64_t>((groups + 3) / 4, 1), 4096);
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int ncn_field_pack_weights(const float* w_master, uint16_t* weights_packed, void* stream) {
    hipLaunchKernelGGL(pack_weights_kernel, dim3(N_FRAGS), dim3(64), 0, (hipStream_t)stream, w_master,
                       (_Float16*)weights_packed);
    NCN_LAUNCH_CHECK("ncn_field_pack_weights");
    return 0;
}

// `levels` is a HOST array of 16 x {scale f32 bits, resolution, params, offset}.
int ncn_field_fwd(const float* xyzs, const float* dirs, int64_t n, const float* table, const uint32_t* levels,
                  float xyz_min, float xyz_extent, const uint16_t* weights_packed, int mode, float* sigmas,
                  float* rgbs, uint16_t* enc_cache, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(mode == 0 || mode == 1, hipErrorInvalidValue, "ncn_field_fwd: mode must be 0 or 1");
    NCN_REQUIRE(((uintptr_t)table & 7) == 0 && ((uintptr_t)enc_cache & 7) == 0, hipErrorInvalidValue,
                "ncn_field_fwd: table / enc_cache must be 8-byte aligned");
    const LevelTable Lt = make_table(levels);
    hipLaunchKernelGGL(field_fwd_kernel, dim3(fwd_grid(n)), dim3(256), 0, (hipStream_t)stream, xyzs, dirs, n,
                       (const float2*)table, Lt, xyz_min, xyz_extent, (const half4_t*)weights_packed, mode, sigmas,
                       rgbs, (half4_t*)enc_cache);
    NCN_LAUNCH_CHECK("ncn_field_fwd");
    return 0;
}

int ncn_field_bwd_blocks(int64_t n) {
    const int64_t groups = (n + 15) / 16;
    // 2 workgroups per CU on 256 CUs; at least ~4 groups per wave
    return (int)std::max<int64_t>(1, std::min<int64_t>(512, (groups + 15) / 16));
}

int ncn_field_bwd(const float* xyzs, const float* dirs, int64_t n, const uint32_t* levels, float xyz_min,
                  float xyz_extent, const uint16_t* weights_packed, const uint16_t* enc_cache,
                  const float* dL_dsigmas, const float* dL_drgbs, float* grad_table, float* slab, void* stream) {
    if (n <= 0) return 0;
    const LevelTable Lt = make_table(levels);
    hipLaunchKernelGGL(field_bwd_kernel, dim3(ncn_field_bwd_blocks(n)), dim3(BWD_THREADS), 0, (hipStream_t)stream,
                       xyzs, dirs, n, Lt, xyz_min, xyz_extent, (const half4_t*)weights_packed,
                       (const half4_t*)enc_cache, dL_dsigmas, dL_drgbs, grad_table, slab);
    NCN_LAUNCH_CHECK("ncn_field_bwd");
    return 0;
}

int ncn_field_reduce_wgrad(const float* slab, int n_blocks, float* grad_w, void* stream) {
    if (n_blocks <= 0) return 0;
    hipLaunchKernelGGL(reduce_wgrad_kernel, dim3(cdiv(NCN_FIELD_NW, 256), cdiv(n_blocks, WRED_CHUNK)), dim3(256), 0,
                       (hipStream_t)stream, slab, n_blocks, grad_w);
    NCN_LAUNCH_CHECK("ncn_field_reduce_wgrad");
    return 0;
}

}  // extern "C"
