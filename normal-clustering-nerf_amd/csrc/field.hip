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
// ReLU backward on a gradient tile: keep v where the saved fp16 activation is > 0, as fp16
__device__ __forceinline__ half4_t relu_mask_h4(float4_t v, half4_t x) {
    half4_t h;
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = x[i] > (_Float16)0.0f ? (_Float16)v[i] : (_Float16)0.0f;
    return h;
}

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
    // index % params without a 32-bit division: a hashed level always has params = 2^log2_T (a
    // power of two), a dense level has index < res^3 <= params.  Same result as the modulo.
    if ((params & (params - 1)) == 0) return index & (params - 1);
    return index < params ? index : index % params;
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

// DPP helpers (16-lane rows)
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

template <int K>
__device__ __forceinline__ void run_sum(float& v, const int (&link)[4]) {
    const float t = dppf<DPP_ROW_SL(1 << K)>(v);
    if (link[K]) v += t;
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
};

__device__ __forceinline__ void mlp_sigma(const half4_t* F, int lane, half4_t e0, half4_t e1, FwdState& st) {
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
        acc = mfma16(frag(F, F_L1 + 2 * t, lane), e0, acc);
        acc = mfma16(frag(F, F_L1 + 2 * t + 1, lane), e1, acc);
        st.x2[t] = relu_h4(acc);
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
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
        acc = mfma16(frag(F, F_L3 + 2 * t, lane), st.x3h, acc);
        acc = mfma16(frag(F, F_L3 + 2 * t + 1, lane), st.x3d, acc);
        st.x4[t] = relu_h4(acc);
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
        float4_t acc = zero4();
#pragma unroll
        for (int ks = 0; ks < 4; ks++) acc = mfma16(frag(F, F_L4 + 4 * t + ks, lane), st.x4[ks], acc);
        st.x5[t] = relu_h4(acc);
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
                                                        int64_t n, const int32_t* __restrict__ n_dev,
                                                        const float2* __restrict__ table, LevelTable Lt,
                                                        float xyz_min, float xyz_extent,
                                                        const half4_t* __restrict__ wpacked, int mode,
                                                        float* __restrict__ sigmas, float* __restrict__ rgbs,
                                                        half4_t* __restrict__ enc_cache) {
    __shared__ half4_t F[N_FWD_FRAGS * 64];
    __shared__ LevelTable L;
    if (n_dev) n = min<int64_t>(n, *n_dev);  // device-resident count (static-capacity buffers)
    for (int i = threadIdx.x; i < N_FWD_FRAGS * 64; i += 256) F[i] = wpacked[i];
    load_levels(L, Lt);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
    const int64_t n_groups = (n + 15) / 16;
    const int64_t wave0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
        const half4_t* Fl = F + opaque_zero();  // fragments re-read from LDS every group (not hoisted)
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
        mlp_sigma(Fl, lane, b0, b1, st);
        if (g == 0 && valid) sigmas[s] = __expf(st.h[0]);  // TruncExp forward = exp
        if (mode == 1) continue;
        float dx = 0.f, dy = 0.f, dz = 0.f;
        if (valid) {
            dx = dirs[3 * s]; dy = dirs[3 * s + 1]; dz = dirs[3 * s + 2];
            const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
            dx /= nrm; dy /= nrm; dz /= nrm;
        }
        mlp_rgb(Fl, lane, dx, dy, dz, st);
        if (g == 0 && valid) {
            rgbs[3 * s] = sigmoidf_(st.out[0]);
            rgbs[3 * s + 1] = sigmoidf_(st.out[1]);
            rgbs[3 * s + 2] = sigmoidf_(st.out[2]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Backward, MLP pass.  Per 16-sample group (inputs prefetched one group ahead): recompute the MLP
// forward from the cached encoding, back-propagate through the five layers (transposed products
// with the W^T fragments, re-read from LDS every group), write the encoding gradient level-major
// for the scatter pass, and accumulate dW = sum_s dY_s X_s^T over the wave's groups in 40
// register tiles, each layer's right after its output gradient exists.  The dW MFMAs need the
// samples on K: a C-layout tile is transposed by one MFMA with the identity (transpose_tile).
// At the end the four waves reduce their tiles into LDS and the workgroup writes one fp32 slab
// row (reduced in a fixed order later).
constexpr int BWD_THREADS = 256;

struct WGrad {
    float4_t w1[4][2], w2[4], w3[4][2], w4[4][4], w5[4];
};

// Tile transpose by MFMA: a C-layout tile (lane (g,r) = [feature 4g+i][sample r]) fed as the A
// operand of A.I (I = 16x16 identity B fragment) comes back as [sample 4g+i][feature r], i.e. with
// the samples on K as the dW products need.  Exact (products with 1, sums of zeros), one MFMA
// instead of an LDS round trip.
__device__ __forceinline__ half4_t identity_frag(int lane) {
    const int g = lane >> 4, r = lane & 15;
    half4_t I;
#pragma unroll
    for (int j = 0; j < 4; j++) I[j] = (_Float16)((4 * g + j == r) ? 1.0f : 0.0f);
    return I;
}
__device__ __forceinline__ half4_t transpose_tile_h(half4_t I, half4_t v) { return to_h4(mfma16(v, I, zero4())); }
__device__ __forceinline__ half4_t transpose_tile(half4_t I, float4_t v) { return transpose_tile_h(I, to_h4(v)); }

// Per-group inputs of the backward (prefetched one group ahead).
struct BwdIn {
    half4_t e0, e1;
    float dx, dy, dz, dsig, dr0, dr1, dr2;
};
__device__ __forceinline__ void bwd_load(BwdIn& in, int64_t grp, int64_t n, int lane, const half4_t* __restrict__ enc,
                                         const float* __restrict__ dirs, const float* __restrict__ dL_dsig,
                                         const float* __restrict__ dL_drgb) {
    const int64_t s = grp * 16 + (lane & 15);
    const bool valid = s < n;
    in.e0 = enc[(grp * 2 + 0) * 64 + lane];
    in.e1 = enc[(grp * 2 + 1) * 64 + lane];
    in.dx = in.dy = in.dz = in.dsig = in.dr0 = in.dr1 = in.dr2 = 0.f;
    if (valid) {
        in.dx = dirs[3 * s]; in.dy = dirs[3 * s + 1]; in.dz = dirs[3 * s + 2];
        in.dsig = dL_dsig ? dL_dsig[s] : 0.f;
        if (dL_drgb) { in.dr0 = dL_drgb[3 * s]; in.dr1 = dL_drgb[3 * s + 1]; in.dr2 = dL_drgb[3 * s + 2]; }
    }
}

__global__ __launch_bounds__(BWD_THREADS) void field_bwd_kernel(
    const float* __restrict__ dirs, int64_t n, const int32_t* __restrict__ n_dev, const half4_t* __restrict__ wpacked,
    const half4_t* __restrict__ enc_cache, const float* __restrict__ dL_dsig, const float* __restrict__ dL_drgb,
    float* __restrict__ dE_out, float* __restrict__ slab) {
    const int64_t n_stride = n;  // dE layout [16][n_stride]
    if (n_dev) n = min<int64_t>(n, *n_dev);
    // LDS: the weight fragments during the loop, reused as the fp32 dW reduction buffer afterwards.
    constexpr int FRAG_BYTES = N_FRAGS * 64 * 8;
    static_assert(FRAG_BYTES >= NCN_FIELD_NW * 4, "arena too small for the dW reduction");
    __shared__ __attribute__((aligned(16))) char arena[FRAG_BYTES];
    half4_t* F = (half4_t*)arena;
    float* red = (float*)arena;
    for (int i = threadIdx.x; i < N_FRAGS * 64; i += BWD_THREADS) F[i] = wpacked[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15, wid = threadIdx.x >> 6;
    const half4_t Iden = identity_frag(lane);
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
    BwdIn nxt;
    if (wave0 < n_groups) bwd_load(nxt, wave0, n, lane, enc_cache, dirs, dL_dsig, dL_drgb);
    for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
        const int64_t s = grp * 16 + r;
        const bool valid = s < n;
        const half4_t* Fl = F + opaque_zero();  // fragments re-read from LDS every group (not hoisted)
        const BwdIn cur = nxt;  // the next group's loads go out before this group's math
        if (grp + n_waves < n_groups) bwd_load(nxt, grp + n_waves, n, lane, enc_cache, dirs, dL_dsig, dL_drgb);
        const half4_t e0 = cur.e0, e1 = cur.e1;
        float dx = cur.dx, dy = cur.dy, dz = cur.dz;
        const float dsig = cur.dsig, dr0 = cur.dr0, dr1 = cur.dr1, dr2 = cur.dr2;
        if (valid) {
            const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
            dx /= nrm; dy /= nrm; dz /= nrm;
        }
        FwdState st;
        mlp_sigma(Fl, lane, e0, e1, st);
        mlp_rgb(Fl, lane, dx, dy, dz, st);
        // Backward through the five layers with each layer's weight gradient accumulated as soon as
        // its output gradient exists (dW[out][in] += sum_s dY[out][s] X[in][s]: A = dY with the
        // samples on K, B = X with the samples on K, both via transpose_tile), so every activation
        // tile dies right after its last use.  ReLU masks come from the saved fp16 activations.
        // dY5: d(pre-sigmoid) = drgb * s(1-s), rows 0..2 on g==0
        float4_t dy5 = zero4();
        if (g == 0) {
            const float s0 = sigmoidf_(st.out[0]), s1 = sigmoidf_(st.out[1]), s2 = sigmoidf_(st.out[2]);
            dy5[0] = dr0 * s0 * (1.f - s0);
            dy5[1] = dr1 * s1 * (1.f - s1);
            dy5[2] = dr2 * s2 * (1.f - s2);
        }
        const half4_t dy5h = to_h4(dy5);
        {   // dW5: dY = dy5 (1 out tile), X = x5 (4 in tiles)
            const half4_t A = transpose_tile_h(Iden, dy5h);
#pragma unroll
            for (int b = 0; b < 4; b++) acc.w5[b] = mfma16(A, transpose_tile_h(Iden, st.x5[b]), acc.w5[b]);
        }
        // L5 backward -> dG2, ReLU(x5) mask -> dD4
        half4_t dD4h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) dD4h[t] = relu_mask_h4(mfma16(frag(Fl, B_L5 + t, lane), dy5h, zero4()), st.x5[t]);
        {   // dW4: dY = dD4 (4 out tiles), X = x4 (4 in tiles)
            half4_t Xt[4];
#pragma unroll
            for (int b = 0; b < 4; b++) Xt[b] = transpose_tile_h(Iden, st.x4[b]);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile_h(Iden, dD4h[a]);
#pragma unroll
                for (int b = 0; b < 4; b++) acc.w4[a][b] = mfma16(A, Xt[b], acc.w4[a][b]);
            }
        }
        // L4 backward -> dG1, ReLU(x4) mask -> dD3
        half4_t dD3h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            float4_t v = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ks++) v = mfma16(frag(Fl, B_L4 + 4 * t + ks, lane), dD4h[ks], v);
            dD3h[t] = relu_mask_h4(v, st.x4[t]);
        }
        {   // dW3: dY = dD3 (4 out tiles), X = [d | h] : in tile 0 = d (cols 0..2), tile 1 = h (cols 3..18)
            const half4_t Xd = transpose_tile_h(Iden, st.x3d);
            const half4_t Xh = transpose_tile_h(Iden, st.x3h);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile_h(Iden, dD3h[a]);
                acc.w3[a][0] = mfma16(A, Xd, acc.w3[a][0]);
                acc.w3[a][1] = mfma16(A, Xh, acc.w3[a][1]);
            }
        }
        // L3 backward -> dh (rgb path) ; + TruncExp backward on h[0]
        float4_t dh = zero4();
#pragma unroll
        for (int ks = 0; ks < 4; ks++) dh = mfma16(frag(Fl, B_L3 + ks, lane), dD3h[ks], dh);
        if (g == 0) dh[0] += dsig * __expf(fminf(fmaxf(st.h[0], -15.f), 15.f));
        const half4_t dhh = to_h4(dh);
        {   // dW2: dY = dh (1 out tile), X = x2 (4 in tiles)
            const half4_t A = transpose_tile_h(Iden, dhh);
#pragma unroll
            for (int b = 0; b < 4; b++) acc.w2[b] = mfma16(A, transpose_tile_h(Iden, st.x2[b]), acc.w2[b]);
        }
        // L2 backward -> dH1, ReLU(x2) mask -> dD1
        half4_t dD1h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) dD1h[t] = relu_mask_h4(mfma16(frag(Fl, B_L2 + t, lane), dhh, zero4()), st.x2[t]);
        {   // dW1: dY = dD1 (4 out tiles), X = e (2 in tiles)
            const half4_t X0 = transpose_tile_h(Iden, e0);
            const half4_t X1 = transpose_tile_h(Iden, e1);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                const half4_t A = transpose_tile_h(Iden, dD1h[a]);
                acc.w1[a][0] = mfma16(A, X0, acc.w1[a][0]);
                acc.w1[a][1] = mfma16(A, X1, acc.w1[a][1]);
            }
        }
        // L1 backward -> dE (tile t holds levels 8t+2g, 8t+2g+1)
        float4_t dE[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            float4_t v = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ks++) v = mfma16(frag(Fl, B_L1 + 4 * t + ks, lane), dD1h[ks], v);
            dE[t] = v;
        }
        // encoding gradient -> level-major [16][n] float2 for the scatter pass
        if (valid) {
            float2* o = (float2*)dE_out;
            o[(int64_t)(2 * g) * n_stride + s] = make_float2(dE[0][0], dE[0][1]);
            o[(int64_t)(2 * g + 1) * n_stride + s] = make_float2(dE[0][2], dE[0][3]);
            o[(int64_t)(8 + 2 * g) * n_stride + s] = make_float2(dE[1][0], dE[1][1]);
            o[(int64_t)(9 + 2 * g) * n_stride + s] = make_float2(dE[1][2], dE[1][3]);
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

// ---------------------------------------------------------------------------------------------
// Scatter of the encoding gradient into the fp32 table gradient (tcnn kernel_grid_backward).
// Hash-grid gradients are extremely local: the rays of a patch re-touch the same few entries per
// level hundreds of times, so a workgroup owns one span of consecutive samples
// (~1/4 patch) and, level by level, aggregates every contribution in an LDS hash table before
// anything reaches memory (6144 slots, 4-way set associative: 24 KB keys + 96 KB int64 sums):
//  1. consecutive samples (lanes) in the same base cell are merged first with DPP run sums inside
//     each 16-lane row (all 8 corners shared);
//  2. run heads look up their 8 corners (one ds_read_b128 of the set per corner, ds_cmpst_b32 to
//     claim an empty way) and add with ds_add_u64 into 64-bit FIXED-POINT sums: on gfx950 an LDS f32 atomic
//     costs ~3 cycles per active lane (193 cycles per wave-instruction, tools/lds_atomic_bench),
//     an LDS u64 atomic add ~13 cycles per wave-instruction.  The fixed point is exact integer
//     arithmetic (order-independent, reproducible): per (workgroup, level) the scale is 2^k with
//     k = 46 - e, max|dE| < 2^e, so a value within 2^23 of the level's maximum converts exactly
//     and the LDS sum (< 2^15 contributions) cannot overflow;
//  3. at the end of a level (or when half of the slots are taken) the table is flushed: two
//     lanes per slot, each converts its sum back to f32 and issues one f32 global atomic.
// A contribution whose set is full of other entries goes straight to a global atomic, as
// does a whole level whose gradient is not finite (NaN/Inf propagate as in the f32 path).
#ifdef NCN_DIAG_PHASES
__device__ unsigned long long ncn_sc_phase[8];
#define SC_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define SC_ACC(i, a, b) ph[i] += (b) - (a)
#else
#define SC_T(v)
#define SC_ACC(i, a, b)
#endif
constexpr int SC_THREADS = 1024;
#ifndef SC_SETS
#define SC_SETS 1536
#endif
#ifndef SC_FLUSH_FRAC
#define SC_FLUSH_FRAC 2
#endif
constexpr int SC_WAYS = 4;                  // 4-way set associative: one ds_read_b128 per lookup
constexpr int SC_TS = SC_SETS * SC_WAYS;    // 6144 slots: 24 KB keys + 96 KB sums + 12 KB claim list
constexpr uint32_t SC_EMPTY = 0xFFFFFFFFu;
#ifndef SC_MERGE_LEVELS
#define SC_MERGE_LEVELS 16
#endif

__device__ __forceinline__ uint32_t sc_set(uint32_t e) { return __umulhi(e * 0x9E3779B1u, (uint32_t)SC_SETS); }

// round(v * 2^k) as int64 for |v * 2^k| < 2^46 without f64: split at 2^23 into two exact int32s
__device__ __forceinline__ long long sc_fix(float v, int k) {
    const float x = ldexpf(v, k - 23);   // |x| < 2^23
    const float hi = truncf(x);          // exact
    const float lo = ldexpf(x - hi, 23); // exact fraction, |lo| < 2^23
    return ((long long)(int)hi << 23) + (long long)(int)rintf(lo);
}

// Flush: only the slots claimed since the last flush (the `used` list), two lanes per slot (x and
// y of one entry are adjacent floats: 8-B pieces per atomic instruction), one f32 global atomic per
// non-zero sum; then exactly those slots are reset.  Cost proportional to the entries, not the table.
__device__ __forceinline__ void sc_flush(uint32_t* keys, long long* valx, long long* valy,
                                         const uint16_t* used, int* fill, float* __restrict__ grad, uint32_t off,
                                         int k) {
    const int nf = *fill;
    for (int i = threadIdx.x; i < 2 * nf; i += SC_THREADS) {
        const int slot = used[i >> 1];
        const uint32_t key = keys[slot];
        const long long q = (i & 1) ? valy[slot] : valx[slot];
#ifdef NCN_DIAG_SC_NO_GATOMIC
        if (q == 12345) grad[2 * (size_t)(off + key) + (i & 1)] = 1.f;
#else
        if (q != 0) atomicAdd(grad + 2 * (size_t)(off + key) + (i & 1), (float)ldexp((double)q, -k));
#endif
    }
    __syncthreads();  // every lane has read its slots
    for (int i = threadIdx.x; i < nf; i += SC_THREADS) {
        const int slot = used[i];
        keys[slot] = SC_EMPTY;
        valx[slot] = 0;
        valy[slot] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) *fill = 0;
    __syncthreads();
}

__device__ __forceinline__ int64_t scatter_span_of(int64_t n) {
    // ~one span per CU: n/256 samples, at least 1024, a multiple of 64; at most 2^16 so that the
    // fixed-point sums keep their headroom (each sample adds at most once to an entry)
    int64_t sp = min<int64_t>(65536, max<int64_t>(1024, (n + 255) / 256));
    return (sp + 63) / 64 * 64;
}

__global__ __launch_bounds__(SC_THREADS) void field_scatter_kernel(const float* __restrict__ xyzs, int64_t n_stride,
                                                                   const int32_t* __restrict__ n_dev, LevelTable Lt,
                                                                   float xyz_min, float xyz_extent,
                                                                   const float2* __restrict__ dE,
                                                                   float* __restrict__ grad) {
    __shared__ __attribute__((aligned(16))) uint32_t keys[SC_TS];
    __shared__ long long valx[SC_TS], valy[SC_TS];
    __shared__ uint16_t used[SC_TS];  // slots claimed since the last flush, in claim order
    __shared__ int fill;              // == number of entries in `used`
    __shared__ float wmax[SC_THREADS / 64][16];
    __shared__ float lmax[16];
    for (int i = threadIdx.x; i < SC_TS; i += SC_THREADS) {
        keys[i] = SC_EMPTY;
        valx[i] = 0;
        valy[i] = 0;
    }
    if (threadIdx.x == 0) fill = 0;
    const int lane = threadIdx.x & 63, r = lane & 15, wid = threadIdx.x >> 6;
    const int64_t n = n_dev ? min<int64_t>(n_stride, *n_dev) : n_stride;
    const int64_t span = scatter_span_of(n), nspans = (n + span - 1) / span;
    for (int64_t sp = blockIdx.x; sp < nspans; sp += gridDim.x) {
    const int64_t s0 = sp * span, s1 = min(n, s0 + span);
    // fixed-point scale per level: max |dE| over the span, all 16 levels in one load round
    {
        float m[16];
#pragma unroll
        for (int l = 0; l < 16; l++) m[l] = 0.f;
        for (int64_t s = s0 + threadIdx.x; s < s1; s += SC_THREADS) {
#pragma unroll
            for (int l = 0; l < 16; l++) {
                const float2 g = dE[(int64_t)l * n_stride + s];
                const float a = fmaxf(fabsf(g.x), fabsf(g.y));
                m[l] = (isfinite(g.x) && isfinite(g.y)) ? fmaxf(m[l], a) : INFINITY;
            }
        }
#pragma unroll
        for (int l = 0; l < 16; l++) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) m[l] = fmaxf(m[l], __shfl_xor(m[l], o, 64));
        }
        if (lane < 16) {
            float v = m[0];
#pragma unroll
            for (int l = 1; l < 16; l++) v = lane == l ? m[l] : v;
            wmax[wid][lane] = v;
        }
        __syncthreads();
        if (threadIdx.x < 16) {
            float v = 0.f;
            for (int w = 0; w < SC_THREADS / 64; w++) v = fmaxf(v, wmax[w][threadIdx.x]);
            lmax[threadIdx.x] = v;
        }
        __syncthreads();
    }
    // the span is cut into nchunk EQUAL chunks (<= SC_THREADS samples each) so that no chunk
    // leaves most waves idle at its barrier
    const int nchunk = (int)((s1 - s0 + SC_THREADS - 1) / SC_THREADS);
    const int64_t len = s1 - s0;
    const int total = 16 * max(nchunk, 0);
    // software pipeline over (level, chunk): the next item's loads are in flight while this one
    // is aggregated
    auto load = [&](int it, float& x, float& y, float& z, float2& g) {
        const int l = it / nchunk, ch = it - l * nchunk;
        const int64_t c0 = s0 + len * ch / nchunk, c1 = s0 + len * (ch + 1) / nchunk;
        const int64_t s = c0 + threadIdx.x;
        x = y = z = 0.f;
        g = make_float2(0.f, 0.f);
        if (s < c1) {
            x = xyzs[3 * s];
            y = xyzs[3 * s + 1];
            z = xyzs[3 * s + 2];
            g = dE[(int64_t)l * n_stride + s];
        }
    };
    float nx, ny, nz;
    float2 ng;
    if (total > 0) load(0, nx, ny, nz, ng);
#ifdef NCN_DIAG_PHASES
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    for (int it = 0; it < total; it++) {
        SC_T(t0);
        const int l = it / nchunk, ch = it - l * nchunk;
#ifdef NCN_DIAG_SC_LEVELS_MASK
        const float m = ((NCN_DIAG_SC_LEVELS_MASK >> l) & 1) ? lmax[l] : 0.f;
#else
        const float m = lmax[l];
#endif
        if (m == 0.f) {  // uniform: nothing at this level; keep the pipeline moving
            if (it + 1 < total) load(it + 1, nx, ny, nz, ng);
            continue;
        }
        const float scale = Lt.scale[l];
        const uint32_t res = Lt.res[l], params = Lt.params[l], off = Lt.offset[l];
        const bool dense = (uint64_t)res * res * res <= params;  // tcnn: stride stays <= params
        const bool direct = !isfinite(m);
        int e2 = 0;
        (void)frexpf(direct ? 1.f : m, &e2);  // m < 2^e2
        const int k = 46 - e2;
        const int64_t c1 = s0 + len * (ch + 1) / nchunk;
        const int64_t s = s0 + len * ch / nchunk + threadIdx.x;
        const float x = (nx - xyz_min) / xyz_extent, y = (ny - xyz_min) / xyz_extent, z = (nz - xyz_min) / xyz_extent;
        const float2 gv = ng;
        if (it + 1 < total) load(it + 1, nx, ny, nz, ng);
        const bool valid = s < c1 && ((gv.x != 0.f) || (gv.y != 0.f));
        const LevelPos p = level_pos(scale, x, y, z);
        // corner weights in the forward's association ((wx * wy) * wz) and entry indices without
        // per-corner grid_index branches: dense = base + dx + dy*res + dz*res^2, hashed =
        // ((x+dx) ^ (y+dy)*P1 ^ (z+dz)*P2) & (params-1) (params is 2^19 on every hashed level)
        const float wx[2] = {1.0f - p.fx, p.fx}, wy[2] = {1.0f - p.fy, p.fy}, wz[2] = {1.0f - p.fz, p.fz};
        uint32_t e[8];
        if (dense) {
            const uint32_t b0 = p.px + res * p.py + res * res * p.pz;
#pragma unroll
            for (int c = 0; c < 8; c++) {
                e[c] = b0 + (c & 1) + ((c >> 1) & 1) * res + ((c >> 2) & 1) * res * res;
                e[c] = e[c] < params ? e[c] : e[c] % params;  // as grid_index (boundary corner)
            }
        } else {
            const uint32_t hy0 = p.py * 2654435761u, hy1 = (p.py + 1) * 2654435761u;
            const uint32_t hz0 = p.pz * 805459861u, hz1 = (p.pz + 1) * 805459861u;
#pragma unroll
            for (int c = 0; c < 8; c++)
                e[c] = ((p.px + (c & 1)) ^ ((c & 2) ? hy1 : hy0) ^ ((c & 4) ? hz1 : hz0)) & (params - 1);
        }
        // runs of lanes in the same base cell, merged with DPP suffix sums inside each 16-lane row
        // (an inactive lane gets a key nobody else has).  Coarse levels only: from level
        // SC_MERGE_LEVELS on most lanes head their own run and the merge would cost more VALU
        // than the LDS traffic it saves.
        bool head = valid;
        float v0[8], v1[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
            v0[c] = valid ? w * gv.x : 0.f;
            v1[c] = valid ? w * gv.y : 0.f;
        }
        if (l < SC_MERGE_LEVELS) {
            const int key = valid ? (int)(p.px + res * (p.py + res * p.pz)) : (int)(0xFFFFFFF0u - (uint32_t)r);
            const int key_next = dppi<DPP_ROW_SL(1)>(key);
            const int key_prev = dppi<DPP_ROW_SR(1)>(key);
            int link[4];
            link[0] = (r < 15) && (key_next == key);
            link[1] = link[0] && dppi<DPP_ROW_SL(1)>(link[0]);
            link[2] = link[1] && dppi<DPP_ROW_SL(2)>(link[1]);
            link[3] = link[2] && dppi<DPP_ROW_SL(4)>(link[2]);
            head = valid && (r == 0 || key_prev != key);
#pragma unroll
            for (int c = 0; c < 8; c++) {
                run_sum<0>(v0[c], link); run_sum<0>(v1[c], link);
                run_sum<1>(v0[c], link); run_sum<1>(v1[c], link);
                run_sum<2>(v0[c], link); run_sum<2>(v1[c], link);
                run_sum<3>(v0[c], link); run_sum<3>(v1[c], link);
            }
        }
        uint32_t newmask = 0;  // corners whose slot this lane claimed
        int slot[8];
        if (head && direct) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                atomicAdd(grad + 2 * (size_t)(off + e[c]), v0[c]);
                atomicAdd(grad + 2 * (size_t)(off + e[c]) + 1, v1[c]);
            }
        }
        SC_T(t1);
        if (head && !direct) {
            uint4 kk[8];
#pragma unroll
            for (int c = 0; c < 8; c++) kk[c] = *(const uint4*)&keys[SC_WAYS * sc_set(e[c])];
            int claim[8];
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const int p0 = SC_WAYS * sc_set(e[c]);
                const uint32_t k0 = kk[c].x, k1 = kk[c].y, k2 = kk[c].z, k3 = kk[c].w;
                slot[c] = k0 == e[c] ? p0 : k1 == e[c] ? p0 + 1 : k2 == e[c] ? p0 + 2 : k3 == e[c] ? p0 + 3 : -1;
                // claim the first way of the set seen empty
                claim[c] = slot[c] >= 0 ? -1
                         : k0 == SC_EMPTY ? p0 : k1 == SC_EMPTY ? p0 + 1 : k2 == SC_EMPTY ? p0 + 2
                         : k3 == SC_EMPTY ? p0 + 3 : -1;
            }
            uint32_t got[8];
#pragma unroll
            for (int c = 0; c < 8; c++) got[c] = claim[c] >= 0 ? atomicCAS(&keys[claim[c]], SC_EMPTY, e[c]) : 0u;
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if (claim[c] >= 0) {
                    if (got[c] == SC_EMPTY) { slot[c] = claim[c]; newmask |= 1u << c; }
                    else if (got[c] == e[c]) slot[c] = claim[c];
                }
            }
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if (slot[c] >= 0) {
                    atomicAdd((unsigned long long*)&valx[slot[c]], (unsigned long long)sc_fix(v0[c], k));
                    atomicAdd((unsigned long long*)&valy[slot[c]], (unsigned long long)sc_fix(v1[c], k));
                } else {
#ifdef NCN_DIAG_SC_NO_FALLBACK
                    if (v0[c] == 1234.5f) grad[c] = v1[c];
#else
                    atomicAdd(grad + 2 * (size_t)(off + e[c]), v0[c]);
                    atomicAdd(grad + 2 * (size_t)(off + e[c]) + 1, v1[c]);
#endif
                }
            }
        }
        SC_T(t2);
        {   // append the claimed slots to `used`: one LDS atomic per wave
            const int mine = __builtin_popcount(newmask);
            const float incl = wave_incl_sum_dpp((float)mine);
            const int wtot = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
            int base = 0;
            if (wtot) {
                if (lane == 0) base = atomicAdd(&fill, wtot);
                base = __builtin_amdgcn_readfirstlane(base);
                int pos = base + (int)incl - mine;
#pragma unroll
                for (int c = 0; c < 8; c++)
                    if (newmask & (1u << c)) used[pos++] = (uint16_t)slot[c];
            }
        }
        __syncthreads();
        SC_T(t3);
        if (ch == nchunk - 1 || fill > SC_TS / SC_FLUSH_FRAC) sc_flush(keys, valx, valy, used, &fill, grad, off, k);
        SC_T(t4);
        SC_ACC(0, t0, t1);
        SC_ACC(1, t1, t2);
        SC_ACC(2, t2, t3);
        SC_ACC(3, t3, t4);
    }
#ifdef NCN_DIAG_PHASES
    if (threadIdx.x == 0 && blockIdx.x == 7)
        for (int i = 0; i < 4; i++) ncn_sc_phase[i] = ph[i];
#endif
    __syncthreads();  // lmax / wmax are rewritten by the next span
    }
}

static int scatter_grid(int64_t n_cap) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(256, (n_cap + 1023) / 1024));  // one per CU
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
int ncn_field_fwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const float* table,
                  const uint32_t* levels,
                  float xyz_min, float xyz_extent, const uint16_t* weights_packed, int mode, float* sigmas,
                  float* rgbs, uint16_t* enc_cache, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(mode == 0 || mode == 1, hipErrorInvalidValue, "ncn_field_fwd: mode must be 0 or 1");
    NCN_REQUIRE(((uintptr_t)table & 7) == 0 && ((uintptr_t)enc_cache & 7) == 0, hipErrorInvalidValue,
                "ncn_field_fwd: table / enc_cache must be 8-byte aligned");
    const LevelTable Lt = make_table(levels);
    hipLaunchKernelGGL(field_fwd_kernel, dim3(fwd_grid(n)), dim3(256), 0, (hipStream_t)stream, xyzs, dirs, n, n_dev,
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

int64_t ncn_field_bwd_dE_floats(int64_t n) { return n > 0 ? 32 * n : 0; }

int ncn_field_bwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const uint32_t* levels,
                  float xyz_min,
                  float xyz_extent, const uint16_t* weights_packed, const uint16_t* enc_cache,
                  const float* dL_dsigmas, const float* dL_drgbs, float* grad_table, float* slab, float* dE_ws,
                  void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(((uintptr_t)dE_ws & 7) == 0, hipErrorInvalidValue, "ncn_field_bwd: dE_ws must be 8-byte aligned");
    const LevelTable Lt = make_table(levels);
    hipLaunchKernelGGL(field_bwd_kernel, dim3(ncn_field_bwd_blocks(n)), dim3(BWD_THREADS), 0, (hipStream_t)stream,
                       dirs, n, n_dev, (const half4_t*)weights_packed, (const half4_t*)enc_cache, dL_dsigmas,
                       dL_drgbs, dE_ws, slab);
    NCN_LAUNCH_CHECK("ncn_field_bwd");
    hipLaunchKernelGGL(field_scatter_kernel, dim3(scatter_grid(n)), dim3(SC_THREADS), 0, (hipStream_t)stream, xyzs, n,
                       n_dev, Lt, xyz_min, xyz_extent, (const float2*)dE_ws, grad_table);
    NCN_LAUNCH_CHECK("ncn_field_bwd (scatter)");
    return 0;
}

#ifdef NCN_DIAG_PHASES
int ncn_diag_read_phases(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ncn_sc_phase), 8 * sizeof(unsigned long long));
}
#endif

int ncn_field_reduce_wgrad(const float* slab, int n_blocks, float* grad_w, void* stream) {
    if (n_blocks <= 0) return 0;
    hipLaunchKernelGGL(reduce_wgrad_kernel, dim3(cdiv(NCN_FIELD_NW, 256), cdiv(n_blocks, WRED_CHUNK)), dim3(256), 0,
                       (hipStream_t)stream, slab, n_blocks, grad_w);
    NCN_LAUNCH_CHECK("ncn_field_reduce_wgrad");
    return 0;
}

}  // extern "C"
