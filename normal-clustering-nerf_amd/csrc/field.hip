// NGPMT field for gfx950: multires hash-grid encoding (tiny-cuda-nn Grid/Hash semantics) fused
// with sigma_net (32->64->16), TruncExp, and rgb_net, replacing tcnn Encoding + two FullyFusedMLPs
// (reference models/ngp_mt.py:70-113, 157-229) and TruncExp (models/custom_functions.py:162-173).
// rgb_net is tcnn's network as built by the reference: `tcnn.Network(n_input_dims=19, ...)` wraps
// an Identity encoding that pads the 19 inputs cat[d/|d|, h] to the FullyFusedMLP's 16-alignment
// (32) with the value 1.0 (a learned bias in the padded columns), and pads the 3 outputs to 16:
// W3 is 64x32, W5 16x64 (rgb_net.params = 7168, sigma_net.params = 3072, as tcnn).
//
// Layout ("transposed activations"): every layer is computed as  Y^T = W . X^T  with the gfx950
// v_mfma_f32_16x16x32_{f16,bf16} (K = 32 per instruction), samples on the MFMA column (lane & 15),
// features on the rows.  The accumulator of a layer (lane (g,r) holds rows 4g..4g+3 of column r)
// is the B operand of the next layer with no data movement: two 16-row accumulator tiles side by
// side form a K = 32 operand whose element j of lane group g is feature phi(g,j) = 4g+j (j < 4, the
// first tile) or 16+4g+j-4 (the second), and the A fragments (weights) are packed in the same
// permuted K order.  A wave owns 16 samples per step; lane (g,r) encodes hash levels
// {2g, 2g+1, 8+2g, 9+2g} of sample r — exactly features phi(g, 0..7) of the encoding, i.e. the
// layer-1 B operand — and in the backward scatters the gradient of those levels.  Weights live in
// LDS as pre-packed MFMA fragments (ncn_field_pack_weights, 16 B per lane per K=32 fragment).
// Operand precision is a template parameter: fp16 (tcnn's FullyFusedMLP precision) or bf16
// (config #3); fp32 hash table + fp32 trilinear interpolation, fp32 accumulation either way.
#include <algorithm>
#include <type_traits>
#include <cstring>
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

typedef float float4_t __attribute__((ext_vector_type(4)));
typedef short short4_t __attribute__((ext_vector_type(4)));

// MFMA operand traits: T = _Float16 or __bf16; v4 = one K=16 / half a K=32 fragment, v8 = K=32.
template <typename T> struct Mfma;
template <> struct Mfma<_Float16> {
    static constexpr bool f16 = true;
    typedef _Float16 v4 __attribute__((ext_vector_type(4)));
    typedef _Float16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ float4_t k32(v8 a, v8 b, float4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ float4_t k16(v4 a, v4 b, float4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma<__bf16> {
    static constexpr bool f16 = false;
    typedef __bf16 v4 __attribute__((ext_vector_type(4)));
    typedef __bf16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ float4_t k32(v8 a, v8 b, float4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ float4_t k16(v4 a, v4 b, float4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
    }
};

__device__ __forceinline__ float4_t zero4() { return float4_t{0.f, 0.f, 0.f, 0.f}; }
template <typename T>
__device__ __forceinline__ typename Mfma<T>::v4 cvt4(float4_t v) {  // round to the operand type (RNE)
    typename Mfma<T>::v4 h;
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = (T)v[i];
    return h;
}
template <typename T>
__device__ __forceinline__ typename Mfma<T>::v4 relu4(float4_t v) {
    typename Mfma<T>::v4 h;
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = (T)fmaxf(v[i], 0.0f);
    return h;
}
// ReLU backward on a gradient tile: keep v where the saved (rounded) activation is > 0
template <typename T>
__device__ __forceinline__ typename Mfma<T>::v4 relu_mask4(float4_t v, typename Mfma<T>::v4 x) {
    typename Mfma<T>::v4 h;
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = (float)x[i] > 0.0f ? (T)v[i] : (T)0.0f;
    return h;
}
template <typename V8, typename V4>
__device__ __forceinline__ V8 cat8(V4 a, V4 b) {
    return V8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// ---- packed weight fragments ----
// K=32 fragments (64 lanes x 8 values = 1 KB; lane (g,r) element j = A[row r][k phi(g,j)])
// forward (A = W, rows = out, K = in)
constexpr int F_L1 = 0;    // [t 0..3]          W1[16t+r][phi]
constexpr int F_L2 = 4;    // [s 0..1]          W2[r][32s+phi]
constexpr int F_L3 = 6;    // [t 0..3]          W3[16t+r][psi]   (psi: the padded-input order, below)
constexpr int F_L4 = 10;   // [t 0..3][s 0..1]  W4[16t+r][32s+phi]
constexpr int F_L5 = 18;   // [s 0..1]          W5[r][32s+phi]   (all 16 padded output rows)
constexpr int N_FWD32 = 20;
// backward (A = W^T, rows = in, K = out)
constexpr int B_L4 = 20;   // [t 0..3][s 0..1]  W4[32s+phi][16t+r]
constexpr int B_L3 = 28;   // [s 0..1]          W3[32s+phi][3+r]   (rows = h only)
constexpr int B_L1 = 30;   // [t 0..1][s 0..1]  W1[32s+phi][16t+r]
constexpr int N_FRAG32 = 34;
// K=16 fragments (64 lanes x 4 values = 512 B; lane (g,r) element j = A[row r][k 4g+j]) of the two
// products whose K is a 16-wide layer output (the K=32 form would be half zeros)
constexpr int B_L5 = 0;    // [t 0..3]          W5[4g+j][16t+r]
constexpr int B_L2 = 4;    // [t 0..3]          W2[4g+j][16t+r]
constexpr int N_FRAG16 = 8;
constexpr int PACKED_HALVES = N_FRAG32 * 512 + N_FRAG16 * 256;
static_assert(PACKED_HALVES == NCN_FIELD_PACKED_HALVES, "packed size");

// master weight offsets (floats) inside the concatenated fp32 buffer (tcnn's padded shapes)
constexpr int W1_OFF = 0, W2_OFF = W1_OFF + 64 * 32, W3_OFF = W2_OFF + 16 * 64, W4_OFF = W3_OFF + 64 * 32,
              W5_OFF = W4_OFF + 64 * 64, W_TOTAL = W5_OFF + 16 * 64;
static_assert(W_TOTAL == NCN_FIELD_NW, "weights size");

__host__ __device__ constexpr int phi(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }
// rgb_net input index of K element (g,j) of the layer-3 B operand [h tile | d,pad tile]:
// j < 4: h feature 4g+j = input 3+4g+j; j >= 4: q = 4g+j-4, input q (d, q < 3) or 16+q (padding)
__host__ __device__ constexpr int psi(int g, int j) {
    return j < 4 ? 3 + 4 * g + j : ((4 * g + j - 4) < 3 ? (4 * g + j - 4) : 16 + (4 * g + j - 4));
}

// index into the concatenated master weights of packed element (f, lane, j)
__host__ __device__ constexpr int frag32_index(int f, int lane, int j) {
    const int g = lane >> 4, r = lane & 15, k = phi(g, j);
    if (f < F_L2) return W1_OFF + (16 * (f - F_L1) + r) * 32 + k;
    if (f < F_L3) return W2_OFF + r * 64 + 32 * (f - F_L2) + k;
    if (f < F_L4) return W3_OFF + (16 * (f - F_L3) + r) * 32 + psi(g, j);
    if (f < F_L5) return W4_OFF + (16 * ((f - F_L4) >> 1) + r) * 64 + 32 * ((f - F_L4) & 1) + k;
    if (f < B_L4) return W5_OFF + r * 64 + 32 * (f - F_L5) + k;
    if (f < B_L3) return W4_OFF + (32 * ((f - B_L4) & 1) + k) * 64 + 16 * ((f - B_L4) >> 1) + r;
    if (f < B_L1) return W3_OFF + (32 * (f - B_L3) + k) * 32 + 3 + r;
    return W1_OFF + (32 * ((f - B_L1) & 1) + k) * 32 + 16 * ((f - B_L1) >> 1) + r;
}
__host__ __device__ constexpr int frag16_index(int f, int lane, int j) {
    const int g = lane >> 4, r = lane & 15, k = 4 * g + j;
    return f < B_L2 ? W5_OFF + k * 64 + 16 * (f - B_L5) + r : W2_OFF + k * 64 + 16 * (f - B_L2) + r;
}
__device__ float frag32_value(const float* __restrict__ W, int f, int lane, int j) { return W[frag32_index(f, lane, j)]; }
__device__ float frag16_value(const float* __restrict__ W, int f, int lane, int j) { return W[frag16_index(f, lane, j)]; }

// packed position -> master weight index (ncn_field_pack_map)
__global__ void pack_map_kernel(int32_t* __restrict__ src) {
    const int f = blockIdx.x, lane = threadIdx.x;
    if (f < N_FRAG32) {
        for (int j = 0; j < 8; j++) src[(f * 64 + lane) * 8 + j] = frag32_index(f, lane, j);
    } else {
        const int f16 = f - N_FRAG32;
        for (int j = 0; j < 4; j++) src[N_FRAG32 * 512 + (f16 * 64 + lane) * 4 + j] = frag16_index(f16, lane, j);
    }
}

template <typename T>
__global__ void pack_weights_kernel(const float* __restrict__ W, T* __restrict__ out) {
    const int f = blockIdx.x, lane = threadIdx.x;
    if (f < N_FRAG32) {
#pragma unroll
        for (int j = 0; j < 8; j++) out[(f * 64 + lane) * 8 + j] = (T)frag32_value(W, f, lane, j);
    } else {
        const int f16 = f - N_FRAG32;
#pragma unroll
        for (int j = 0; j < 4; j++) out[N_FRAG32 * 512 + (f16 * 64 + lane) * 4 + j] = (T)frag16_value(W, f16, lane, j);
    }
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

// trilinear interpolation of one level (tcnn kernel_grid: corner bit d -> +1 along dim d).  Entry
// indices without per-corner grid_index branches: a dense level (res^3 <= params: tcnn's stride
// never exceeds params) is base + dx + dy*res + dz*res^2 (mod params only at the boundary corner
// res^3 == params can't reach: kept as in grid_index), a hashed one ((x+dx) ^ (y+dy)*P1 ^
// (z+dz)*P2) & (params-1) with the four products formed once (params is 2^19 on every hashed
// level).  Corner weights in the association ((wx * wy) * wz) of the reference loop.
__device__ __forceinline__ float2 encode_level(const float2* __restrict__ tab, const LevelTable& L, int l, float x,
                                               float y, float z) {
    const LevelPos p = level_pos(L.scale[l], x, y, z);
    const uint32_t params = L.params[l], res = L.res[l], off = L.offset[l];
    uint32_t e[8];
    if ((uint64_t)res * res * res <= params) {
        const uint32_t b0 = p.px + res * p.py + res * res * p.pz;
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const uint32_t i = b0 + (c & 1) + ((c >> 1) & 1) * res + ((c >> 2) & 1) * res * res;
            e[c] = i < params ? i : i % params;
        }
    } else {
        const uint32_t hy0 = p.py * 2654435761u, hy1 = (p.py + 1) * 2654435761u;
        const uint32_t hz0 = p.pz * 805459861u, hz1 = (p.pz + 1) * 805459861u;
        const uint32_t mask = params - 1;
#pragma unroll
        for (int c = 0; c < 8; c++) e[c] = ((p.px + (c & 1)) ^ ((c & 2) ? hy1 : hy0) ^ ((c & 4) ? hz1 : hz0)) & mask;
    }
    float2 v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = tab[off + e[c]];
    const float wx[2] = {1.0f - p.fx, p.fx}, wy[2] = {1.0f - p.fy, p.fy}, wz[2] = {1.0f - p.fz, p.fz};
    float2 acc = make_float2(0.f, 0.f);
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
        acc.x = fmaf(w, v[c].x, acc.x);
        acc.y = fmaf(w, v[c].y, acc.y);
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

// LDS fragment tables: K=32 fragments as v8 per lane, then the K=16 ones as v4 per lane
template <typename T>
struct Frags {
    typedef typename Mfma<T>::v4 v4;
    typedef typename Mfma<T>::v8 v8;
    const v8* f32;
    const v4* f16;
    __device__ __forceinline__ v8 a32(int f, int lane) const { return f32[f * 64 + lane]; }
    __device__ __forceinline__ v4 a16(int f, int lane) const { return f16[f * 64 + lane]; }
};
// The sigma_net fragments alone (the split backward's sigma pass, compact LDS): F_L1, F_L2 at
// their indices, B_L1 packed right behind them; B_L2 as the only fp16 fragments.
template <typename T>
struct FragsSigma : Frags<T> {
    __device__ __forceinline__ typename Mfma<T>::v8 a32(int f, int lane) const {
        return this->f32[(f >= B_L1 ? f - (B_L1 - F_L3) : f) * 64 + lane];
    }
    __device__ __forceinline__ typename Mfma<T>::v4 a16(int f, int lane) const {
        return this->f16[(f - B_L2) * 64 + lane];
    }
};
constexpr int N_SIG32 = F_L3 + 4, N_SIG16 = 4;  // F_L1, F_L2, B_L1 / B_L2

// Shared per-group forward (16 samples).  Produces every intermediate the backward needs.
template <typename T>
struct FwdState {
    typedef typename Mfma<T>::v4 v4;
    v4 x2[4];       // relu(H1) tiles (B operands of L2)
    float4_t h;     // sigma_net output tile (rows 4g..4g+3)
    v4 x3h, x3d;    // L3 B operand halves: h tile, [d, 1-padding] tile
    v4 x4[4];       // relu(G1)
    v4 x5[4];       // relu(G2)
    float4_t out;   // rgb pre-activation tile (rows 0..2 valid on g==0)
};

template <typename T, typename FR>
__device__ __forceinline__ void mlp_sigma(const FR& F, int lane, typename Mfma<T>::v8 e, FwdState<T>& st) {
    typedef Mfma<T> M;
    typedef typename M::v8 v8;
#pragma unroll
    for (int t = 0; t < 4; t++) st.x2[t] = relu4<T>(M::k32(F.a32(F_L1 + t, lane), e, zero4()));
    float4_t h = M::k32(F.a32(F_L2, lane), cat8<v8>(st.x2[0], st.x2[1]), zero4());
    st.h = M::k32(F.a32(F_L2 + 1, lane), cat8<v8>(st.x2[2], st.x2[3]), h);
}

template <typename T>
__device__ __forceinline__ void mlp_rgb(const Frags<T>& F, int lane, float dnx, float dny, float dnz, FwdState<T>& st) {
    typedef Mfma<T> M;
    typedef typename M::v8 v8;
    const int g = lane >> 4;
    st.x3h = cvt4<T>(st.h);
    // [d, 1-padding]: element i of lane group g is padded-input q = 4g+i: d[q] for q < 3, else 1.0
    st.x3d = cvt4<T>(float4_t{g == 0 ? dnx : 1.f, g == 0 ? dny : 1.f, g == 0 ? dnz : 1.f, 1.f});
    const v8 b3 = cat8<v8>(st.x3h, st.x3d);
#pragma unroll
    for (int t = 0; t < 4; t++) st.x4[t] = relu4<T>(M::k32(F.a32(F_L3 + t, lane), b3, zero4()));
    const v8 b4a = cat8<v8>(st.x4[0], st.x4[1]), b4b = cat8<v8>(st.x4[2], st.x4[3]);
#pragma unroll
    for (int t = 0; t < 4; t++)
        st.x5[t] = relu4<T>(M::k32(F.a32(F_L4 + 2 * t + 1, lane), b4b, M::k32(F.a32(F_L4 + 2 * t, lane), b4a, zero4())));
    const float4_t o = M::k32(F.a32(F_L5, lane), cat8<v8>(st.x5[0], st.x5[1]), zero4());
    st.out = M::k32(F.a32(F_L5 + 1, lane), cat8<v8>(st.x5[2], st.x5[3]), o);
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
// Processing order of the training step's samples (ncn_field_sort_windows).  The marcher packs
// samples ray by ray (the compositors need each ray's segment contiguous); the field does not care
// about order, and the table scatter of its backward aggregates the gradients of samples that share
// hash-grid corners — which, across the ~60 neighbouring rays of a patch, are samples at the same
// place in space, far apart in ray order.  So every window of SORT_W consecutive samples is sorted
// by the 30-bit Morton code of its normalised positions (10 bits per axis, the finest hash level's
// resolution): `order[p]` is the sample processed at position p.  The forward evaluates samples in
// that order (neighbouring lanes gather neighbouring table entries), the MLP backward writes the
// encoding gradient in it, and the scatter's units (one window) see long runs of equal cells on
// every level.  Keys carry the in-window index (unique keys, bitonic sort in LDS): the order is a
// deterministic function of the positions.
constexpr int SORT_W = 4096, SORT_THREADS = 1024;
__device__ __forceinline__ uint32_t sort_spread10(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
__device__ __forceinline__ uint32_t sort_q10(float v, float mn, float inv) {
    const float q = (v - mn) * inv * 1024.0f;
    return (uint32_t)(int)fminf(fmaxf(q, 0.0f), 1023.0f);  // (NaN -> 0)
}
__global__ __launch_bounds__(SORT_THREADS) void sort_windows_kernel(const float* __restrict__ xyzs, int64_t n,
                                                                    const int32_t* __restrict__ n_dev, float mn,
                                                                    float inv, int32_t* __restrict__ order) {
    __shared__ unsigned long long k[SORT_W];
    if (n_dev) n = min<int64_t>(n, *n_dev);
    const int64_t base = (int64_t)blockIdx.x * SORT_W;
    if (base >= n) return;  // (uniform)
    const int cnt = (int)min<int64_t>(SORT_W, n - base);
    for (int i = threadIdx.x; i < SORT_W; i += SORT_THREADS) {
        unsigned long long key = ~0ull;  // empty slots sort last
        if (i < cnt) {
            const float* x = xyzs + 3 * (base + i);
            const uint32_t m = sort_spread10(sort_q10(x[0], mn, inv)) | (sort_spread10(sort_q10(x[1], mn, inv)) << 1) |
                               (sort_spread10(sort_q10(x[2], mn, inv)) << 2);
            key = ((unsigned long long)m << 12) | (unsigned long long)i;
        }
        k[i] = key;
    }
    __syncthreads();
    for (int size = 2; size <= SORT_W; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < SORT_W / 2; t += SORT_THREADS) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;  // pair (lo, hi), lo's bit `stride` clear
                const bool up = (lo & size) == 0;
                const unsigned long long a = k[lo], b = k[hi];
                if ((a > b) == up) { k[lo] = b; k[hi] = a; }
            }
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < cnt; i += SORT_THREADS) order[base + i] = (int32_t)(base + (int64_t)(k[i] & 0xFFFull));
}

// ---------------------------------------------------------------------------------------------
// Forward: grid-stride over 16-sample groups, one group per wave per step.
// (Round 3 measured 4 waves/SIMD at 101 us and spills at 5-6; round 5 took the register pressure
// out of the encoding instead — two levels' gathers in flight, below — and at 72 VGPRs the kernel
// runs 7 waves/SIMD: 84 us.  The waves_per_eu hint keeps the allocation in that range: without it
// the compiler's choice left 5 waves.)
// DENSITY: the grid refresh's mode 2 (encodings from encode_xcd_kernel's scratch, sigma only) as its
// own instantiation — the training forward's loop then carries no trace of it (with the scratch read
// inside the shared loop the training kernel took 136 registers, 3 waves/SIMD, and ran ~10 % slower).
template <typename T, bool DENSITY>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void field_fwd_kernel(const float* __restrict__ xyzs, const float* __restrict__ dirs,
                                                        int64_t n, const int32_t* __restrict__ n_dev,
                                                        const float2* __restrict__ table, LevelTable Lt,
                                                        float xyz_min, float xyz_extent,
                                                        const typename Mfma<T>::v8* __restrict__ wpacked, int mode,
                                                        float* __restrict__ sigmas, float* __restrict__ rgbs,
                                                        typename Mfma<T>::v8* __restrict__ enc_cache,
                                                        const int32_t* __restrict__ order) {
    typedef typename Mfma<T>::v8 v8;
    __shared__ v8 Fs[N_FWD32 * 64];
    __shared__ LevelTable L;
    const int64_t n16 = (n + 15) & ~(int64_t)15;  // (mode 2, level-major scratch) per-level stride
    if (n_dev) n = min<int64_t>(n, *n_dev);  // device-resident count (static-capacity buffers)
    for (int i = threadIdx.x; i < N_FWD32 * 64; i += 256) Fs[i] = wpacked[i];
    load_levels(L, Lt);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
    const int64_t n_groups = (n + 15) / 16;
    // (Tried: an XCD-aware renumbering (common.h xcd_block) giving each L2 whole ray patches:
    // 88 -> 109 us — the CUs of one XCD then gather the same fine-level entries at once.)
    const int64_t wave0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
        Frags<T> F;
        F.f32 = Fs + opaque_zero();  // fragments re-read from LDS every group (not hoisted)
        F.f16 = nullptr;
        const int64_t pos = grp * 16 + r;  // processing position; s = the sample it evaluates
        const bool valid = pos < n;
        const int64_t s = valid && order ? (int64_t)order[pos] : pos;
        v8 e;
        if constexpr (DENSITY) {  // the encodings of encode_xcd_kernel (mode 2: density only)
            typedef T t2 __attribute__((ext_vector_type(2)));
            const t2* el = (const t2*)enc_cache + pos;  // levels 2g, 2g+1 | 8+2g, 9+2g of sample pos
            const t2 a0 = el[(2 * g) * n16], a1 = el[(2 * g + 1) * n16];
            const t2 b0 = el[(8 + 2 * g) * n16], b1 = el[(9 + 2 * g) * n16];
            e = v8{a0[0], a0[1], a1[0], a1[1], b0[0], b0[1], b1[0], b1[1]};
        } else {
            float x = 0.f, y = 0.f, z = 0.f;
            if (valid) {
                x = (xyzs[3 * s] - xyz_min) / xyz_extent;
                y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
                z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
            }
            const float2 e00 = encode_level(table, L, 2 * g, x, y, z);
            const float2 e01 = encode_level(table, L, 2 * g + 1, x, y, z);
            // The last two levels' positions wait for the first two's results (an empty asm that
            // reads them), so only two levels' 16 gathers are in flight per lane, not all 32: the
            // kernel then needs 72 VGPRs instead of 120 and runs 7 waves per SIMD instead of 4 —
            // 100 -> 84 us on the bench batch (round 5, tools/field_probe.py; one level at a time:
            // 85; the pairs of an x-edge as one 16-B load: 90-98, the cache-line count does not
            // bound it; buffer loads: 90).
            asm volatile("; encode: levels 8+ after 0-7 %1 %2" : "+v"(x) : "v"(e00.x), "v"(e01.x));
            const float2 e10 = encode_level(table, L, 8 + 2 * g, x, y, z);
            const float2 e11 = encode_level(table, L, 9 + 2 * g, x, y, z);
            e = v8{(T)e00.x, (T)e00.y, (T)e01.x, (T)e01.y, (T)e10.x, (T)e10.y, (T)e11.x, (T)e11.y};
            if (enc_cache) enc_cache[grp * 64 + lane] = e;
        }
        FwdState<T> st;
        mlp_sigma<T>(F, lane, e, st);
        if (g == 0 && valid) sigmas[s] = __expf(st.h[0]);  // TruncExp forward = exp
        if (DENSITY || mode != 0) continue;
        float dx = 0.f, dy = 0.f, dz = 0.f;
        if (valid) {
            dx = dirs[3 * s]; dy = dirs[3 * s + 1]; dz = dirs[3 * s + 2];
            const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
            dx /= nrm; dy /= nrm; dz /= nrm;
        }
        mlp_rgb<T>(F, lane, dx, dy, dz, st);
        if (g == 0 && valid) {
            rgbs[3 * s] = sigmoidf_(st.out[0]);
            rgbs[3 * s + 1] = sigmoidf_(st.out[1]);
            rgbs[3 * s + 2] = sigmoidf_(st.out[2]);
        }
    }
}

// The hash-grid encoding of the density pass (grid refresh: ~1 M points, one per hit cell, with no
// ray coherence) split by level over the XCDs: block b runs on XCD b % 8 (dispatch round-robin — a
// placement hint, nothing depends on it) and XCD x encodes levels x and 15 - x of every point, so each
// 4 MB L2 holds at most two levels' tables instead of serving all 16 (45.8 MB) from the Infinity
// Cache, and every XCD pairs a cheap coarse level with a costly fine one (round 6: x and x + 8 left
// XCDs 5-7 with levels 13-15 and the rest waiting: 225.6 -> 214.5 us for the pass on the bench grid's
// 706 K cells, profiles/round6/density_probe_pairing.log) (the sample-major forward on Morton-ordered grid points: 436 us; with every hashed level
// reading one table: 206 us — tools/field_probe.py).  Output: a level-major scratch [16][n16] of T
// pairs (172 vs 179 us for the pass with the forward's fragment-order layout, tools/density_probe.py), each level's pairs written by its own block; field_fwd_kernel mode 2
// gathers lane (g, r)'s levels {2g, 2g+1 | 8+2g, 9+2g} from it and runs sigma_net.  Same
// encode_level and operand rounding as the sample-major forward: bit-identical sigmas.
template <typename T>
__global__ __launch_bounds__(256) void encode_xcd_kernel(const float* __restrict__ xyzs, int64_t n,
                                                         const int32_t* __restrict__ n_dev,
                                                         const float2* __restrict__ table, LevelTable Lt,
                                                         float xyz_min, float xyz_extent, int nb,
                                                         T* __restrict__ enc) {
    __shared__ LevelTable L;
    load_levels(L, Lt);
    __syncthreads();
    const int64_t n16 = (n + 15) & ~(int64_t)15;  // per-level stride of the level-major scratch
    if (n_dev) n = min<int64_t>(n, *n_dev);
    const int x8 = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int l = j < nb ? x8 : 15 - x8, blk = j < nb ? j : j - nb;
    const int64_t s = (int64_t)blk * 256 + threadIdx.x;
    if (s >= n) return;
    const float x = (xyzs[3 * s] - xyz_min) / xyz_extent;
    const float y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
    const float z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
    const float2 a = encode_level(table, L, l, x, y, z);
    typedef T t2 __attribute__((ext_vector_type(2)));
    // level-major scratch [16][n16] of T pairs: a workgroup's 256 points of one level are one
    // contiguous 1 KB store (a fragment-order layout scattered 4-byte pieces of 64-byte records over
    // 16 workgroups on 8 XCDs: 179 vs 172 us for the pass; round 5: non-temporal point loads and
    // scratch stores, to keep the streamed data from evicting the level's table in L2 — no change)
    ((t2*)enc)[(int64_t)l * n16 + s] = t2{(T)a.x, (T)a.y};
}

// ---------------------------------------------------------------------------------------------
// Backward, MLP pass.  A workgroup of 8 waves (one per CU: 2 waves per SIMD) takes 8 groups of 16
// samples per step.  Phase 1, every wave on its own group (inputs prefetched one step ahead):
// recompute the MLP forward from the cached encoding, back-propagate through the five layers
// (transposed products with the W^T fragments from LDS), write the encoding gradient level-major
// for the scatter pass, and put the 30 operand tiles of the weight gradient (dY and X tiles of
// every layer, transposed so that the samples are on K) into an LDS exchange area.  Phase 2,
// after a barrier: wave w owns 5 of the 40 dW tiles and accumulates them over the step's groups
// straight from the exchange area, two groups (32 samples) per K=32 MFMA.  So no wave holds all
// of dW, the two waves of a SIMD overlap their MFMA chains, and every tile is written once per
// workgroup into its slab row at the end.
constexpr int DE_HEADER_FLOATS = 4;  // the dE workspace's header (ncn_field_bwd_dE_floats)
// (the scatter's sample layout, defined with the scatter below: the rgb / one-pass MLP pass writes
// the positions in it, DE_POS_READY in the header)
__host__ __device__ constexpr int64_t sc_perm_stride(int64_t n_stride);
__device__ __forceinline__ int64_t sc_perm(int64_t s, int cls);
constexpr int DE_POS_FLAG = 2;  // header float: the mask of unit classes whose permuted positions the workspace holds
// The table scatter's unit queue at the end of the workspace: per level_lo of a launch, a grab counter
// and a departure counter (field_scatter_kernel); zeroed by the MLP pass that writes the header, and
// left zero by every scatter launch (its last workgroup out resets them).
constexpr int SC_QUEUE_WORDS = 32;
__host__ __device__ int64_t de_queue_offset(int64_t e_stride);
// The MLP pass writes the coarse classes' positions only: the coarse units' strided loads cost
// 16-20 us per unit, the fine units' grabs measured no faster from permuted positions (round 6,
// profiles/round6/scatter_probe_perm.log), and the writes run beside the clustering.
constexpr int DE_POS_MLP_CLASSES = 2;
// The pass that writes them: the rgb pass, beside the clustering (round 6 A/B against the sigma pass
// after the join: 14.28 / 14.29 M rays/s alike).
constexpr int DE_POS_PART = 1;  // BWD_RGB
constexpr int BWD_WAVES = 8;
constexpr int BWD_THREADS = 64 * BWD_WAVES;
// exchange tiles per group: dW operands, A = dY^T, B = X^T (16 features x 16 samples)
constexpr int XA5 = 0, XB5 = 1, XA4 = 5, XB4 = 9, XA3 = 13, XB3D = 17, XB3H = 18, XA2 = 19, XB2 = 20, XA1 = 24,
              XB1 = 28, N_XFRAG = 30;

// dW operands through LDS images: a C-layout tile (lane (g,r) holds [feature 4g+i][sample r]) is
// stored as a [sample][feature] image (16 rows of 32 B; lane (g,r) writes 8 B at row r, chunk g,
// chunks XOR-swizzled by row>>2 against write bank conflicts) and read back with the gfx950
// transposed read ds_read_b64_tr_b16: lane 4q+p of group g addresses row 4g+q, chunk p, and lane
// (g,i) receives column i of rows 4g..4g+3, i.e. [feature i][samples 4g..4g+3] — half of the A/B
// fragment of a product that sums over samples (the two halves of a K=32 fragment are the images
// of two groups).  (EXEC must be all ones at the read.)
template <typename V>
__device__ __forceinline__ void x_put(uint16_t* tile, int lane, V v) {
    const int g = lane >> 4, r = lane & 15;
    *(V*)(tile + r * 16 + 4 * (g ^ (r >> 2))) = v;
}
template <typename V>
__device__ __forceinline__ V x_get(const uint16_t* tile, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) short4_t*)(tile + (4 * g + q) * 16 + 4 * (p ^ g)));
    return __builtin_bit_cast(V, v);
}

// Per-group inputs of the backward (prefetched one step ahead).
// Backward parts (the split MLP pass of the training step, ncn_field_bwd_mlp_part): BWD_RGB = the
// rgb_net path alone (needs only dL/drgb: it can run while the clustering still computes the depth
// gradient) — dW3..dW5 and the rgb part of dL/dh, stashed; BWD_SIGMA = the rest: dL/dh = stash +
// TruncExp'(h0) dL/dsigma, then sigma_net and the encoding gradient, dW1, dW2.  BWD_ALL = both.
enum { BWD_RGB = 1, BWD_SIGMA = 2, BWD_ALL = 3 };
template <typename T>
struct BwdIn {
    typename Mfma<T>::v8 e;
    float dx, dy, dz, dsig, dr0, dr1, dr2;
    float px, py, pz;  // (rgb / one pass, with positions out) the sample's position
    typename Mfma<T>::v4 dq;  // (BWD_SIGMA) the stashed rgb part of dL/dh of this lane's tile, as operands
    float h0;                 // (BWD_SIGMA, g = 0) its row-0 element in fp32 (TruncExp's term is added to it)
};
template <typename T, int PART>
__device__ __forceinline__ void bwd_load(BwdIn<T>& in, int64_t grp, int64_t n, int lane,
                                         const typename Mfma<T>::v8* __restrict__ enc, const float* __restrict__ dirs,
                                         const float* __restrict__ dL_dsig, const float* __restrict__ dL_dsig2,
                                         const float* __restrict__ dL_drgb,
                                         const typename Mfma<T>::v4* __restrict__ stq, const float* __restrict__ sth0,
                                         const int32_t* __restrict__ order, float S, const float* __restrict__ xyzs) {
    const int64_t pos = grp * 16 + (lane & 15);  // processing position (enc_cache / dE order)
    const bool valid = pos < n;
    in.e = enc[grp * 64 + lane];
    in.dx = in.dy = in.dz = in.dsig = in.dr0 = in.dr1 = in.dr2 = 0.f;
    in.px = in.py = in.pz = 0.f;
    if constexpr ((PART & DE_POS_PART) != 0) {
        if (xyzs && valid) { in.px = xyzs[3 * pos]; in.py = xyzs[3 * pos + 1]; in.pz = xyzs[3 * pos + 2]; }
    }
    if constexpr (PART == BWD_SIGMA) {
        in.dq = stq[grp * 64 + lane];
        in.h0 = (lane >> 4) == 0 ? sth0[grp * 16 + (lane & 15)] : 0.f;
    }
    if (valid) {
        const int64_t s = order ? (int64_t)order[pos] : pos;
        if constexpr ((PART & BWD_RGB) != 0) {
            in.dx = dirs[3 * s]; in.dy = dirs[3 * s + 1]; in.dz = dirs[3 * s + 2];
            if (dL_drgb) { in.dr0 = dL_drgb[3 * s] * S; in.dr1 = dL_drgb[3 * s + 1] * S; in.dr2 = dL_drgb[3 * s + 2] * S; }
        }
        if constexpr ((PART & BWD_SIGMA) != 0) {
            const float ds = (dL_dsig ? dL_dsig[s] : 0.f) + (dL_dsig2 ? dL_dsig2[s] : 0.f);
            in.dsig = ds * S;
        }
    }
}

// Phase 1 for one group: forward recompute, backward through the layers, dE out, dW operands out.
__device__ __forceinline__ float lmax_upd(float m, float a, float b) {  // non-finite -> INF
    return (isfinite(a) && isfinite(b)) ? fmaxf(m, fmaxf(fabsf(a), fabsf(b))) : INFINITY;
}
// exchange tiles a pass keeps per group: the sigma pass only XA2..XB1+1 (compact layout, origin XA2)
template <int PART> constexpr int x_count() { return PART == BWD_SIGMA ? N_XFRAG - XA2 : N_XFRAG; }
template <int PART> constexpr int x_origin() { return PART == BWD_SIGMA ? XA2 : 0; }

template <typename T, int PART, typename FR>
__device__ __forceinline__ void bwd_group(const FR& F, uint16_t* Xw, const BwdIn<T>& cur, int64_t grp,
                                          int64_t n, int64_t n_stride, int lane, float* __restrict__ dE_out,
                                          float (&lm)[4], float inv_S, typename Mfma<T>::v4* __restrict__ stq,
                                          float* __restrict__ sth0) {
    typedef Mfma<T> M;
    typedef typename M::v4 v4;
    typedef typename M::v8 v8;
    const int g = lane >> 4, r = lane & 15;
    const int64_t s = grp * 16 + r;
    const bool valid = s < n;
    FwdState<T> st;
    mlp_sigma<T>(F, lane, cur.e, st);
    float4_t dh;
    if constexpr ((PART & BWD_RGB) != 0) {
    float dx = cur.dx, dy = cur.dy, dz = cur.dz;
    if (valid) {
        const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
        dx /= nrm; dy /= nrm; dz /= nrm;
    }
    mlp_rgb<T>(F, lane, dx, dy, dz, st);
    // dY5: d(pre-sigmoid) = drgb * s(1-s), rows 0..2 on g==0 (the padded output rows get zero)
    float4_t dy5 = zero4();
    if (g == 0) {
        const float s0 = sigmoidf_(st.out[0]), s1 = sigmoidf_(st.out[1]), s2 = sigmoidf_(st.out[2]);
        dy5[0] = cur.dr0 * s0 * (1.f - s0);
        dy5[1] = cur.dr1 * s1 * (1.f - s1);
        dy5[2] = cur.dr2 * s2 * (1.f - s2);
    }
    const v4 dy5h = cvt4<T>(dy5);
    x_put(Xw + XA5 * 256, lane, dy5h);
#pragma unroll
    for (int b = 0; b < 4; b++) x_put(Xw + (XB5 + b) * 256, lane, st.x5[b]);
    // L5 backward -> dG2, ReLU(x5) mask -> dD4
    v4 dD4[4];
#pragma unroll
    for (int t = 0; t < 4; t++) dD4[t] = relu_mask4<T>(M::k16(F.a16(B_L5 + t, lane), dy5h, zero4()), st.x5[t]);
#pragma unroll
    for (int t = 0; t < 4; t++) {
        x_put(Xw + (XA4 + t) * 256, lane, dD4[t]);
        x_put(Xw + (XB4 + t) * 256, lane, st.x4[t]);
    }
    // L4 backward -> dG1, ReLU(x4) mask -> dD3
    const v8 d4a = cat8<v8>(dD4[0], dD4[1]), d4b = cat8<v8>(dD4[2], dD4[3]);
    v4 dD3[4];
#pragma unroll
    for (int t = 0; t < 4; t++)
        dD3[t] = relu_mask4<T>(M::k32(F.a32(B_L4 + 2 * t + 1, lane), d4b, M::k32(F.a32(B_L4 + 2 * t, lane), d4a, zero4())),
                                st.x4[t]);
#pragma unroll
    for (int t = 0; t < 4; t++) x_put(Xw + (XA3 + t) * 256, lane, dD3[t]);
    x_put(Xw + XB3D * 256, lane, st.x3d);
    x_put(Xw + XB3H * 256, lane, st.x3h);
    // L3 backward -> dh (rgb path) ; + TruncExp backward on h[0]
    dh = M::k32(F.a32(B_L3, lane), cat8<v8>(dD3[0], dD3[1]), zero4());
    dh = M::k32(F.a32(B_L3 + 1, lane), cat8<v8>(dD3[2], dD3[3]), dh);
    if constexpr (PART == BWD_RGB) {  // the sigma part follows in its own pass (BWD_SIGMA)
        // stash: the operand-rounded tile (what the sigma pass converts it to anyway) and, for the
        // row-0 element that TruncExp's term is added to first, its fp32 value: 36 B per sample
        stq[grp * 64 + lane] = cvt4<T>(dh);
        if (g == 0) sth0[grp * 16 + r] = dh[0];
        return;
    }
    }
    v4 dhh;
    const float tex = __expf(fminf(fmaxf(st.h[0], -15.f), 15.f));
    if constexpr (PART == BWD_SIGMA) {  // (the same explicit fma and rounding as below: bit-identical)
        dhh = cur.dq;
        if (g == 0) dhh[0] = (T)fmaf(cur.dsig, tex, cur.h0);
    } else {  // (the split passes' order: the whole tile rounded as the rgb pass stashes it, then the
              // row-0 element recomputed with the TruncExp term — keeps the two forms bit-identical)
        dhh = cvt4<T>(dh);
        if (g == 0) dhh[0] = (T)fmaf(cur.dsig, tex, dh[0]);
    }
    constexpr int XO = x_origin<PART>();
    x_put(Xw + (XA2 - XO) * 256, lane, dhh);
#pragma unroll
    for (int b = 0; b < 4; b++) x_put(Xw + (XB2 - XO + b) * 256, lane, st.x2[b]);
    // L2 backward -> dH1, ReLU(x2) mask -> dD1
    v4 dD1[4];
#pragma unroll
    for (int t = 0; t < 4; t++) dD1[t] = relu_mask4<T>(M::k16(F.a16(B_L2 + t, lane), dhh, zero4()), st.x2[t]);
#pragma unroll
    for (int t = 0; t < 4; t++) x_put(Xw + (XA1 - XO + t) * 256, lane, dD1[t]);
    const v4 e0 = v4{cur.e[0], cur.e[1], cur.e[2], cur.e[3]}, e1 = v4{cur.e[4], cur.e[5], cur.e[6], cur.e[7]};
    x_put(Xw + (XB1 - XO) * 256, lane, e0);
    x_put(Xw + (XB1 - XO + 1) * 256, lane, e1);
    // L1 backward -> dE (tile t holds levels 8t+2g, 8t+2g+1)
    const v8 d1a = cat8<v8>(dD1[0], dD1[1]), d1b = cat8<v8>(dD1[2], dD1[3]);
    float4_t dE[2];
#pragma unroll
    for (int t = 0; t < 2; t++)
        dE[t] = M::k32(F.a32(B_L1 + 2 * t + 1, lane), d1b, M::k32(F.a32(B_L1 + 2 * t, lane), d1a, zero4()));
    // The encoding gradient leaves in the MLP operand type, as tcnn hands its network's input gradient
    // (type T) to the grid backward: fp16 at the chain's scale S (the scatter divides by S), bf16
    // unscaled — level-major [16][n_stride] pairs behind the workspace header (dE_pairs), half the
    // bytes of f32 pairs.  fp16 overflow gives inf: the level's max is then non-finite, the scatter
    // adds it straight to the gradient and the GradScaler skips the step, as tcnn's would.
    typedef T t2 __attribute__((ext_vector_type(2)));
    const t2 q[4] = {t2{(T)dE[0][0], (T)dE[0][1]}, t2{(T)dE[0][2], (T)dE[0][3]}, t2{(T)dE[1][0], (T)dE[1][1]},
                     t2{(T)dE[1][2], (T)dE[1][3]}};
    // per-level max |dE| of this lane's levels (2g, 2g+1, 8+2g, 9+2g), of the stored values (loss
    // scale off: an exact power of two): the scatter's fixed-point scale
#pragma unroll
    for (int j = 0; j < 4; j++) lm[j] = lmax_upd(lm[j], (float)q[j][0] * inv_S, (float)q[j][1] * inv_S);
    if (valid) {
        t2* o = (t2*)dE_out;
        o[(int64_t)(2 * g) * n_stride + s] = q[0];
        o[(int64_t)(2 * g + 1) * n_stride + s] = q[1];
        o[(int64_t)(8 + 2 * g) * n_stride + s] = q[2];
        o[(int64_t)(9 + 2 * g) * n_stride + s] = q[3];
    }
}

// Phase 2: the dW tiles owned by wave `wid`, accumulated over the exchange tiles of `ng` groups,
// two groups per K=32 MFMA (an odd last group is paired with zeros).  Ownership (5 tiles each):
// waves 0-3: W4 row-block a = wid (4 tiles) + W5 column block wid; waves 4-5: W3 row-blocks
// 2(wid-4), +1 (d/pad and h tiles) + W2 block wid-4; waves 6-7: W1 row-blocks 2(wid-6), +1 (two K
// tiles) + W2 block wid-4.
template <typename T, int NX = N_XFRAG, int XO = 0>
__device__ __forceinline__ typename Mfma<T>::v8 x_pair(const uint16_t* X, int q, int ng, int tile, int lane) {
    typedef typename Mfma<T>::v4 v4;
    const v4 a = x_get<v4>(X + (q * NX + tile - XO) * 256, lane);
    const v4 b = q + 1 < ng ? x_get<v4>(X + ((q + 1) * NX + tile - XO) * 256, lane) : v4{0, 0, 0, 0};
    return cat8<typename Mfma<T>::v8>(a, b);
}
template <typename T, int PART>
__device__ __forceinline__ void bwd_dw(const uint16_t* X, int ng, int wid, int lane, float4_t (&acc)[5]) {
    typedef Mfma<T> M;
    typedef typename M::v8 v8;
    constexpr bool RGB = (PART & BWD_RGB) != 0, SIG = (PART & BWD_SIGMA) != 0;
    if constexpr (PART == BWD_SIGMA) {  // 12 tiles: W1 (4 row x 2 col blocks) one per wave, W2 on waves 0-3
        constexpr int NX = x_count<PART>(), XO = x_origin<PART>();
        for (int q = 0; q < ng; q += 2) {
            acc[0] = M::k32(x_pair<T, NX, XO>(X, q, ng, XA1 + (wid >> 1), lane),
                            x_pair<T, NX, XO>(X, q, ng, XB1 + (wid & 1), lane), acc[0]);
            if (wid < 4)
                acc[1] = M::k32(x_pair<T, NX, XO>(X, q, ng, XA2, lane), x_pair<T, NX, XO>(X, q, ng, XB2 + wid, lane),
                                acc[1]);
        }
        return;
    }
    if constexpr (PART == BWD_RGB) {  // 28 tiles: W4 on waves 0-3 (4 each), W3 row block + W5 on waves 4-7
        for (int q = 0; q < ng; q += 2) {
            if (wid < 4) {
                const v8 A4 = x_pair<T>(X, q, ng, XA4 + wid, lane);
#pragma unroll
                for (int b = 0; b < 4; b++) acc[b] = M::k32(A4, x_pair<T>(X, q, ng, XB4 + b, lane), acc[b]);
            } else {
                const v8 A3 = x_pair<T>(X, q, ng, XA3 + wid - 4, lane);
                acc[0] = M::k32(A3, x_pair<T>(X, q, ng, XB3D, lane), acc[0]);
                acc[1] = M::k32(A3, x_pair<T>(X, q, ng, XB3H, lane), acc[1]);
                acc[4] = M::k32(x_pair<T>(X, q, ng, XA5, lane), x_pair<T>(X, q, ng, XB5 + wid - 4, lane), acc[4]);
            }
        }
        return;
    }
    for (int q = 0; q < ng; q += 2) {
        if (wid < 4) {
            if constexpr (RGB) {
                const v8 A4 = x_pair<T>(X, q, ng, XA4 + wid, lane);
#pragma unroll
                for (int b = 0; b < 4; b++) acc[b] = M::k32(A4, x_pair<T>(X, q, ng, XB4 + b, lane), acc[b]);
                acc[4] = M::k32(x_pair<T>(X, q, ng, XA5, lane), x_pair<T>(X, q, ng, XB5 + wid, lane), acc[4]);
            }
        } else if (wid < 6) {
            if constexpr (RGB) {
                const v8 Bd = x_pair<T>(X, q, ng, XB3D, lane), Bh = x_pair<T>(X, q, ng, XB3H, lane);
#pragma unroll
                for (int aa = 0; aa < 2; aa++) {
                    const v8 A3 = x_pair<T>(X, q, ng, XA3 + 2 * (wid - 4) + aa, lane);
                    acc[2 * aa] = M::k32(A3, Bd, acc[2 * aa]);
                    acc[2 * aa + 1] = M::k32(A3, Bh, acc[2 * aa + 1]);
                }
            }
            if constexpr (SIG)
                acc[4] = M::k32(x_pair<T>(X, q, ng, XA2, lane), x_pair<T>(X, q, ng, XB2 + wid - 4, lane), acc[4]);
        } else {
            if constexpr (SIG) {
                const v8 B0 = x_pair<T>(X, q, ng, XB1, lane), B1 = x_pair<T>(X, q, ng, XB1 + 1, lane);
#pragma unroll
                for (int aa = 0; aa < 2; aa++) {
                    const v8 A1 = x_pair<T>(X, q, ng, XA1 + 2 * (wid - 6) + aa, lane);
                    acc[2 * aa] = M::k32(A1, B0, acc[2 * aa]);
                    acc[2 * aa + 1] = M::k32(A1, B1, acc[2 * aa + 1]);
                }
                acc[4] = M::k32(x_pair<T>(X, q, ng, XA2, lane), x_pair<T>(X, q, ng, XB2 + wid - 4, lane), acc[4]);
            }
        }
    }
}

// The owned tiles (C layout: lane (g,r) = rows 4g+i, column r) into the workgroup's slab row.
// W3 columns: the h tile's column r is input 3+r; the [d, pad] tile's column q is input q (d) or
// 16+q (the 13 constant-1 padding inputs, whose gradient is the plain sum of dY).
// (A split pass stores only its own tiles: the other pass writes the rest of the same slab row.)
template <int PART>
__device__ __forceinline__ void bwd_store_dw(float* __restrict__ out, int wid, int lane, float4_t (&acc)[5], float inv_S) {
    constexpr bool RGB = (PART & BWD_RGB) != 0, SIG = (PART & BWD_SIGMA) != 0;
    const int g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int t = 0; t < 5; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) acc[t][i] *= inv_S;
    if constexpr (PART == BWD_SIGMA) {  // (bwd_dw's split-pass tile ownership)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = 4 * g + i;
            out[W1_OFF + (16 * (wid >> 1) + row) * 32 + 16 * (wid & 1) + r] = acc[0][i];
            if (wid < 4) out[W2_OFF + row * 64 + 16 * wid + r] = acc[1][i];
        }
        return;
    }
    if constexpr (PART == BWD_RGB) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = 4 * g + i;
            if (wid < 4) {
#pragma unroll
                for (int b = 0; b < 4; b++) out[W4_OFF + (16 * wid + row) * 64 + 16 * b + r] = acc[b][i];
            } else {
                const int orow = 16 * (wid - 4) + row;
                out[W3_OFF + orow * 32 + (r < 3 ? r : 16 + r)] = acc[0][i];
                out[W3_OFF + orow * 32 + 3 + r] = acc[1][i];
                out[W5_OFF + row * 64 + 16 * (wid - 4) + r] = acc[4][i];
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int row = 4 * g + i;
        if (wid < 4) {
            if constexpr (RGB) {
#pragma unroll
                for (int b = 0; b < 4; b++) out[W4_OFF + (16 * wid + row) * 64 + 16 * b + r] = acc[b][i];
                out[W5_OFF + row * 64 + 16 * wid + r] = acc[4][i];
            }
        } else if (wid < 6) {
            if constexpr (RGB) {
#pragma unroll
                for (int aa = 0; aa < 2; aa++) {
                    const int orow = 16 * (2 * (wid - 4) + aa) + row;
                    out[W3_OFF + orow * 32 + (r < 3 ? r : 16 + r)] = acc[2 * aa][i];
                    out[W3_OFF + orow * 32 + 3 + r] = acc[2 * aa + 1][i];
                }
            }
            if constexpr (SIG) out[W2_OFF + row * 64 + 16 * (wid - 4) + r] = acc[4][i];
        } else {
            if constexpr (SIG) {
#pragma unroll
                for (int aa = 0; aa < 2; aa++) {
                    const int orow = 16 * (2 * (wid - 6) + aa) + row;
                    out[W1_OFF + orow * 32 + r] = acc[2 * aa][i];
                    out[W1_OFF + orow * 32 + 16 + r] = acc[2 * aa + 1][i];
                }
                out[W2_OFF + row * 64 + 16 * (wid - 4) + r] = acc[4][i];
            }
        }
    }
}

// one 8-wave workgroup per CU on 256 CUs; at least ~4 steps of 8 groups each
__host__ __device__ inline int bwd_blocks_of(int64_t n) {
    const int64_t groups = (n + 15) / 16;
    const int64_t b = (groups + 31) / 32;
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

template <typename T, int PART = BWD_ALL>
__global__ __launch_bounds__(BWD_THREADS) void field_bwd_kernel(
    const float* __restrict__ dirs, int64_t n, const int32_t* __restrict__ n_dev, const uint16_t* __restrict__ wpacked,
    const typename Mfma<T>::v8* __restrict__ enc_cache, const float* __restrict__ dL_dsig,
    const float* __restrict__ dL_drgb, const float* __restrict__ loss_scale, float* __restrict__ dE_out,
    float* __restrict__ slab, float* __restrict__ level_max, const int32_t* __restrict__ order,
    const float* __restrict__ dL_dsig2 = nullptr, float* __restrict__ stash = nullptr,
    const float* __restrict__ xyzs = nullptr) {
    typedef typename Mfma<T>::v4 v4;
    // AMP loss scale (GradScaler of the reference's precision=16 run) times tcnn's fp16 module loss
    // scale (128): the fp16 chain sees the upstream gradients times S (a power of two), dE and dW
    // leave it divided by S.  bf16 (fp32's exponent range) runs unscaled, as tcnn's non-fp16 modules.
    const float S = loss_scale ? *loss_scale * (Mfma<T>::f16 ? NCN_TCNN_LOSS_SCALE : 1.f) : 1.f, inv_S = 1.f / S;
    typedef typename Mfma<T>::v8 v8;
    const int64_t n_stride = (n + 3) & ~(int64_t)3;  // dE layout [16][n_stride] (16-B aligned rows)
    // dE workspace: a 16-B header {1 / S, operand type (0 fp16, 1 bf16)} then the pairs
    float* const dE_pairs = dE_out ? dE_out + DE_HEADER_FLOATS : nullptr;
    if (PART != BWD_RGB && dE_out && blockIdx.x == 0 && threadIdx.x < SC_QUEUE_WORDS) {
        if (threadIdx.x == 0) {
            dE_out[0] = inv_S;
            dE_out[1] = Mfma<T>::f16 ? 0.f : 1.f;
        }
        ((unsigned*)(dE_out + de_queue_offset(n_stride)))[threadIdx.x] = 0u;  // the scatter's unit queue
    }
    // (rgb / one pass) the sample positions in the scatter's per-class load order (sc_perm), behind
    // the encoding gradient: lane (g, r) writes sample r's position into class g's array.  In the
    // processing order of `order` the scatter gathers them itself (no positions written).
    const float* pos_src = ((PART & DE_POS_PART) != 0 && dE_out && !order) ? xyzs : nullptr;
    float* const pos_out = pos_src ? dE_out + DE_HEADER_FLOATS + 16 * n_stride : nullptr;
    const int64_t pos_stride = sc_perm_stride(n_stride);
    if ((PART & DE_POS_PART) != 0 && dE_out && blockIdx.x == 0 && threadIdx.x == 0)
        dE_out[DE_POS_FLAG] = pos_out ? (float)((1 << DE_POS_MLP_CLASSES) - 1) : 0.f;
    const int lm_rows = bwd_blocks_of(n);            // level_max rows the scatter reads
    // split passes' stash (ncn_field_bwd_stash_floats): [groups][64] operand tiles, then [groups][16]
    // fp32 row-0 elements (capacity groups: the layout does not depend on the device count)
    v4* stq = (v4*)stash;
    float* sth0 = stash ? stash + ((n + 15) / 16) * 128 : nullptr;
    if (n_dev) n = min<int64_t>(n, *n_dev);
    // the sigma pass keeps only the sigma_net fragments and its 11 exchange tiles per group (57 KB:
    // two workgroups per CU); the others all 34 + 8 fragments and 30 tiles (158 KB)
    constexpr bool SIGONLY = PART == BWD_SIGMA;
    constexpr int NF32 = SIGONLY ? N_SIG32 : N_FRAG32, NF16 = SIGONLY ? N_SIG16 : N_FRAG16, NX = x_count<PART>();
    __shared__ v8 F32s[NF32 * 64];
    __shared__ v4 F16s[NF16 * 64];
    __shared__ __attribute__((aligned(16))) uint16_t X[BWD_WAVES * NX * 256];  // dW operand images
    {
        const v8* w32 = (const v8*)wpacked;
        const v4* w16 = (const v4*)(wpacked + N_FRAG32 * 512);
        for (int i = threadIdx.x; i < NF32 * 64; i += BWD_THREADS) {
            const int f = i >> 6;  // (sigma pass: B_L1 packed behind F_L2)
            F32s[i] = w32[(SIGONLY && f >= F_L3 ? f + (B_L1 - F_L3) : f) * 64 + (i & 63)];
        }
        for (int i = threadIdx.x; i < NF16 * 64; i += BWD_THREADS) F16s[i] = w16[(SIGONLY ? B_L2 * 64 : 0) + i];
    }
    if constexpr (PART == BWD_RGB) {  // the sigma pass max-reduces into the level_max rows: zero them
        if (blockIdx.x == 0 && level_max)
            for (int i = threadIdx.x; i < lm_rows * 16; i += BWD_THREADS) level_max[i] = 0.f;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float4_t acc[5];
#pragma unroll
    for (int t = 0; t < 5; t++) acc[t] = zero4();
    float lm[4] = {0.f, 0.f, 0.f, 0.f};
    const int64_t n_groups = (n + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * BWD_WAVES;
    int64_t base = (int64_t)blockIdx.x * BWD_WAVES;  // first group of this workgroup's step
    BwdIn<T> nxt;
    if (base + wid < n_groups)
        bwd_load<T, PART>(nxt, base + wid, n, lane, enc_cache, dirs, dL_dsig, dL_dsig2, dL_drgb, stq, sth0, order, S,
                          pos_src);
    for (; base < n_groups; base += stride) {
        const int64_t grp = base + wid;
        const int ng = (int)min<int64_t>(BWD_WAVES, n_groups - base);
        const BwdIn<T> cur = nxt;
        if (grp + stride < n_groups)
            bwd_load<T, PART>(nxt, grp + stride, n, lane, enc_cache, dirs, dL_dsig, dL_dsig2, dL_drgb, stq, sth0, order,
                              S, pos_src);
        if (grp < n_groups) {
            if ((PART & DE_POS_PART) != 0 && pos_out && (lane >> 4) < DE_POS_MLP_CLASSES && grp * 16 + (lane & 15) < n) {
                const int cls = lane >> 4;
                float* po = pos_out + cls * 3 * pos_stride + 3 * sc_perm(grp * 16 + (lane & 15), cls);
                po[0] = cur.px; po[1] = cur.py; po[2] = cur.pz;
            }
            typename std::conditional<SIGONLY, FragsSigma<T>, Frags<T>>::type F;
            const int z = opaque_zero();
            F.f32 = F32s + z;
            F.f16 = F16s + z;
            bwd_group<T, PART>(F, X + wid * NX * 256, cur, grp, n, n_stride, lane, dE_pairs, lm, inv_S, stq, sth0);
        }
        lds_barrier();  // (the dE stores and the next step's loads stay in flight)
        bwd_dw<T, PART>(X, ng, wid, lane, acc);
        lds_barrier();
    }
    bwd_store_dw<PART>(slab + (int64_t)blockIdx.x * NCN_FIELD_NW, wid, lane, acc, inv_S);
    if constexpr (PART == BWD_RGB) return;  // (no encoding gradient in the rgb pass)
    // level maxima: the 16 lanes of a row (same g) share their 4 levels; the row leaders of the 8
    // waves meet in LDS and the workgroup writes its row of level_max [blocks][16] (no atomics: the
    // scatter reduces the rows)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float m = lm[i];
        m = fmaxf(m, dppf<0x128>(m));  // row_ror 8
        m = fmaxf(m, dppf<0x124>(m));
        m = fmaxf(m, dppf<0x122>(m));
        m = fmaxf(m, dppf<0x121>(m));
        lm[i] = m;
    }
    __shared__ float lmw[BWD_WAVES][16];
    if ((lane & 15) == 0) {
        const int g = lane >> 4;
        lmw[wid][2 * g] = lm[0];
        lmw[wid][2 * g + 1] = lm[1];
        lmw[wid][8 + 2 * g] = lm[2];
        lmw[wid][9 + 2 * g] = lm[3];
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        float m = 0.f;
#pragma unroll
        for (int w = 0; w < BWD_WAVES; w++) m = fmaxf(m, lmw[w][threadIdx.x]);
        if constexpr (PART == BWD_SIGMA)  // (any grid size: rows zeroed by the rgb pass; m >= 0, so the
            // IEEE order is the unsigned order of the bits)
            atomicMax((unsigned*)&level_max[(blockIdx.x % lm_rows) * 16 + threadIdx.x], __float_as_uint(m));
        else
            level_max[blockIdx.x * 16 + threadIdx.x] = m;
    }
    // a capped grid (ncn_field_bwd_mlp_part's n_blocks) leaves the scatter's remaining rows neutral
    if (PART == BWD_ALL && blockIdx.x == 0)
        for (int i = (int)gridDim.x * 16 + threadIdx.x; i < lm_rows * 16; i += BWD_THREADS) level_max[i] = 0.f;
}

// Sum of the per-workgroup dW slabs: blockIdx.y takes a chunk of slabs (coalesced 1 KB rows),
// chunk partials are added with f32 atomics (gw accumulates, like every .grad).
constexpr int WRED_CHUNK = 16;
// (nb_sigma rows of the sigma_net weights W1, W2 and nb_rgb rows of the rgb_net's: the split
// backward's two passes run on grids of their own)
__global__ void reduce_wgrad_kernel(const float* __restrict__ slab, int nb_sigma, int nb_rgb, float* __restrict__ gw) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= NCN_FIELD_NW) return;
    const int nb = i < W3_OFF ? nb_sigma : nb_rgb;
    const int b0 = blockIdx.y * WRED_CHUNK, b1 = min(nb, b0 + WRED_CHUNK);
    if (b0 >= b1) return;
    float s = 0.f;
    for (int b = b0; b < b1; b++) s += slab[(int64_t)b * NCN_FIELD_NW + i];
    atomicAdd(gw + i, s);
}

// ---------------------------------------------------------------------------------------------
// Scatter of the encoding gradient into the fp32 table gradient (tcnn kernel_grid_backward).
// Hash-grid gradients are extremely local: the samples of one ray stay in the same cell of a
// coarse level for tens of steps, and the rays of a patch re-touch the same entries (per
// 2-8K-sample span the contributions per distinct entry are ~460 at level 0 and still ~6 at
// level 15).  So the work is organised around runs and a per-workgroup LDS table:
//  * a unit of work is (span of consecutive samples, level): 1024 lanes x C samples x rounds;
//  * a lane sums the eight corner contributions of its consecutive samples in the same cell in
//    registers (a run) and hands a finished run to the table;
//  * the lanes' samples are read from a copy of the positions in the unit's load order (sc_perm,
//    written by the MLP pass): a wave's round reads one contiguous stretch (round 6: 192 -> 176 us,
//    the coarse units' strided loads had cost one cache line per lane per load);
//  * coarse levels [0, SC_CELL_HI) are CELL-keyed: finished runs are queued per wave and added by
//    full-wave passes (sc_drain_cells): one lookup of the run's cell in a 4-way set-associative LDS
//    table and 16 ds_add_u64 into the cell's corner-major sums; fine
//    levels are ENTRY-keyed (sc_add): each of the 8 corners looked up in its own 4-way set (one
//    ds_read_b128 per set, ds_cmpst to claim a way) and its (x, y) added with two ds_add_u64;
//  * sums are 64-bit FIXED-POINT (exact integer arithmetic: order-independent and reproducible; an
//    LDS f32 atomic costs ~3 cycles per active lane on gfx950 against ~13 per wave-instruction for a
//    u64 add, and f32 slot sums measured 2-3x slower under the same-slot conflicts).  The
//    scale of a level is 2^k, k = 60 - log2(unit samples) - e (fine units 46 - e), max|dE| < 2^e (the
//    MLP pass records max|dE| per level), so an entry's unit sum stays below 2^62 and every addend
//    below 2^51 (sc_fix).  A corner whose set is full goes
//    straight to a global f32 atomic;
//  * at the end of the unit the claimed slots (the `used` list) are flushed with one f32 global
//    atomic per non-zero sum and reset.  A unit whose gradient is not finite adds every run straight
//    to global memory (NaN/Inf propagate as in the f32 path).
constexpr int SC_THREADS = 1024;  // one workgroup per CU (the LDS table takes the CU's LDS)
constexpr int SC_WAVES = SC_THREADS / 64;
constexpr int SC_WAYS = 4;        // 4-way set associative: one ds_read_b128 per lookup
constexpr int SC_SLOT_BYTES = 4 + 8 + 8 + 2;  // key, x and y sums, `used` entry
constexpr int SC_SETS_DIR = 1536;  // entry-keyed layout: 6 144 slots (132 KB)
// Cell-keyed layout (the coarse levels [0, SC_CELL_HI)): a slot is one grid CELL of the level and
// holds the 64-bit sums of its 8 corners' x and y (corner-major: vals[(2c + xy) * slots + slot]).
constexpr int SC_CELL_HI = 10;
constexpr int SC_CELL_VALS = 16;
// Finished coarse runs are queued per wave (key + 16 f32 sums, 68 B) and added to the table by a
// full-wave pass once the queue would overflow (sc_push_run / sc_drain_cells): a coarse sample step
// ends a run in only ~6-30 of 64 lanes, and adding them at once cost a set read and 16 ds_add_u64
// wave-instructions (plus 16 fixed-point conversions) per step for those few lanes.
// (Round 6: queued 180 vs 189 us for the whole scatter, levels 0-5 alone 43 vs 62 us per unit,
// profiles/round6/scatter_probe_queue.log; the table shrank from 1 024 cell slots for the queues.)
constexpr int SC_SETS_CELL = 160;  // 640 cell slots (86 KB) beside the run queues (70 KB)
constexpr int SC_QUEUE = 64;       // runs per wave queue
constexpr int SC_CELL_TABLE_BYTES = SC_SETS_CELL * SC_WAYS * (4 + SC_CELL_VALS * 8 + 2);
constexpr int SC_QUEUE_BYTES = SC_WAVES * SC_QUEUE * (4 + SC_CELL_VALS * 4);
constexpr int sc_max(int a, int b) { return a > b ? a : b; }
constexpr int SC_ARENA = sc_max(SC_CELL_TABLE_BYTES + SC_QUEUE_BYTES, SC_SETS_DIR * SC_WAYS * SC_SLOT_BYTES);
static_assert(SC_CELL_TABLE_BYTES % 16 == 0, "run queues 16-B aligned");
constexpr uint32_t SC_EMPTY = 0xFFFFFFFFu;
constexpr int SC_BATCH = 2;  // corners per batch of set reads in sc_add (2: 232 us, 4: 238 us (spills), 8: 298 us;
                             // round 5: 4 at 124 VGPRs 196 us (4 spills); at 120, no spills: 194-195 vs 190)
// Samples per lane of a fine-level unit (unit = 1024 x C samples): 4 (4096-sample units, in grabs of
// 64 x 2) up to level 14; level 15 takes 2 (its ~1 distinct entry per sample would overfill the
// 4-way sets of a 4096-sample unit; units of 2048 from level 13: 198, 14: 202, 15: 190, none: 202 us).
// (Measured round 5: 8192-sample units on levels 10-11 / 10-12: 288 / 281 us against 202; two
// 512-thread workgroups per CU with half the table each: slower.)
__host__ __device__ constexpr int sc_fine_c(int l) { return l < 15 ? 4 : 2; }
#ifndef NCN_SC_C_CELL
#define NCN_SC_C_CELL 4
#endif
constexpr int SC_C_CELL = NCN_SC_C_CELL;     // samples per lane per round on the cell levels

__device__ __forceinline__ uint32_t sc_set(uint32_t e, uint32_t sets) { return __umulhi(e * 0x9E3779B1u, sets); }

// round(v * 2^k) as int64 (|v * 2^k| < 2^51): v * 2^k is exact in f64, adding 1.5 * 2^52 rounds it
// to an integer in the low mantissa bits (round-to-nearest-even), and the bit pattern minus that of
// 1.5 * 2^52 is the two's-complement integer.  Three f64/int ops instead of an f32 hi/lo split.
__device__ __forceinline__ long long sc_fix(float v, int k) {
    const double magic = 6755399441055744.0;  // 1.5 * 2^52
    const double y = fma((double)v, __longlong_as_double((long long)(1023 + k) << 52), magic);
    return __double_as_longlong(y) - __double_as_longlong(magic);
}

// The current layout's arrays inside the arena (uniform pointers) and the per-workgroup counters.
struct ScShared {
    uint32_t* keys;
    long long *valx, *valy;  // (cell layout: valx = the 16 corner-major arrays)
    uint16_t* used;          // slots claimed since the last flush, in claim order
    float4* qval;            // (cell layout) the waves' run queues: [wave][SC_QUEUE][4] float4 (16 sums)
    uint32_t* qkey;          //               and their cell keys [wave][SC_QUEUE]
    uint32_t sets;
    int slots;
    int* fill;
    int* grab;  // the unit's grab counter (fine levels)
};
enum { SC_MODE_DIR = 0, SC_MODE_CELL = 1 };
__device__ __forceinline__ ScShared sc_layout(char* arena, int* fill, int mode) {
    ScShared sh;
    sh.sets = mode == SC_MODE_CELL ? SC_SETS_CELL : SC_SETS_DIR;
    sh.slots = (int)sh.sets * SC_WAYS;
    sh.valx = (long long*)arena;  // 8-B arrays first, then keys, used
    sh.valy = mode == SC_MODE_CELL ? sh.valx + (SC_CELL_VALS - 1) * sh.slots : sh.valx + sh.slots;
    sh.keys = (uint32_t*)(sh.valy + sh.slots);
    sh.used = (uint16_t*)(sh.keys + sh.slots);
    sh.qval = (float4*)(arena + SC_CELL_TABLE_BYTES);
    sh.qkey = (uint32_t*)(sh.qval + SC_WAVES * SC_QUEUE * 4);
    sh.fill = fill;
    return sh;
}

// Level geometry of the unit, uniform.
struct ScLevel {
    float scale;
    uint32_t res, params, off;
    bool dense, direct;
    int k;
};

__device__ __forceinline__ void sc_corner_entries(const ScLevel& L, uint32_t px, uint32_t py, uint32_t pz,
                                                  uint32_t (&e)[8]) {
    if (L.dense) {
        const uint32_t b0 = px + L.res * py + L.res * L.res * pz;
#pragma unroll
        for (int c = 0; c < 8; c++) {
            e[c] = b0 + (c & 1) + ((c >> 1) & 1) * L.res + ((c >> 2) & 1) * L.res * L.res;
            e[c] = e[c] < L.params ? e[c] : e[c] % L.params;  // as grid_index (boundary corner)
        }
    } else {  // params is 2^19 on every hashed level
        const uint32_t hy0 = py * 2654435761u, hy1 = (py + 1) * 2654435761u;
        const uint32_t hz0 = pz * 805459861u, hz1 = (pz + 1) * 805459861u;
#pragma unroll
        for (int c = 0; c < 8; c++)
            e[c] = ((px + (c & 1)) ^ ((c & 2) ? hy1 : hy0) ^ ((c & 4) ? hz1 : hz0)) & (L.params - 1);
    }
}

// Entry-keyed table: one contribution set per lane (cell px,py,pz; v = the 8 corners' (x, y) sums).
// Called by the whole wave; lanes with all-zero v add nothing.
__device__ __forceinline__ void sc_add(ScShared& sh, int lane, uint32_t px, uint32_t py, uint32_t pz,
                                       const float (&v)[16], const ScLevel& L, float* __restrict__ grad) {
    uint32_t e[8];
    sc_corner_entries(L, px, py, pz, e);
    if (L.direct) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (v[2 * c] != 0.f || v[2 * c + 1] != 0.f) {
                atomicAdd(grad + 2 * (size_t)(L.off + e[c]), v[2 * c]);
                atomicAdd(grad + 2 * (size_t)(L.off + e[c]) + 1, v[2 * c + 1]);
            }
        }
        return;
    }
    // Corners in batches of SC_BATCH: the batch's set reads (ds_read_b128) are issued together and
    // waited for once, then the hits and claims are resolved, then the batch's fixed-point adds
    // (ds_add_u64, no return) are issued back to back — a few LDS round trips per record instead of
    // two per corner.  A miss claims the first empty way of its set with ds_cmpst (a uniform branch
    // skips the claim step when no lane of the wave misses); a lost claim re-reads the set once;
    // a full set falls back to a global atomic.  Zero corners (beyond the span / zero dE / a lane
    // with no finished run) take part with nothing to add.
    uint32_t newmask = 0;
    int slot[8];
#pragma unroll
    for (int c0 = 0; c0 < 8; c0 += SC_BATCH) {
        uint4 kk[SC_BATCH];
        int p0[SC_BATCH];
#pragma unroll
        for (int b = 0; b < SC_BATCH; b++) {
            p0[b] = SC_WAYS * sc_set(e[c0 + b], sh.sets);
            kk[b] = *(const uint4*)&sh.keys[p0[b]];
        }
        int sl[SC_BATCH];
        bool vc[SC_BATCH], miss = false;
#pragma unroll
        for (int b = 0; b < SC_BATCH; b++) {
            const uint32_t k = e[c0 + b];
            vc[b] = (v[2 * (c0 + b)] != 0.f) | (v[2 * (c0 + b) + 1] != 0.f);
            sl[b] = kk[b].x == k ? p0[b] : kk[b].y == k ? p0[b] + 1 : kk[b].z == k ? p0[b] + 2
                  : kk[b].w == k ? p0[b] + 3 : -1;
            miss |= vc[b] && sl[b] < 0;
        }
        if (__ballot(miss)) {  // uniform
#pragma unroll
            for (int b = 0; b < SC_BATCH; b++) {
                if (vc[b] && sl[b] < 0) {
                    const uint32_t k = e[c0 + b];
#pragma unroll
                    for (int attempt = 0; attempt < 2 && sl[b] < 0; attempt++) {
                        if (attempt) {  // lost a claim: look again
                            asm volatile("" ::: "memory");
                            kk[b] = *(const uint4*)&sh.keys[p0[b]];
                        }
                        sl[b] = kk[b].x == k ? p0[b] : kk[b].y == k ? p0[b] + 1 : kk[b].z == k ? p0[b] + 2
                              : kk[b].w == k ? p0[b] + 3 : -1;
                        if (sl[b] >= 0) break;
                        const int cl = kk[b].x == SC_EMPTY ? p0[b] : kk[b].y == SC_EMPTY ? p0[b] + 1
                                     : kk[b].z == SC_EMPTY ? p0[b] + 2 : kk[b].w == SC_EMPTY ? p0[b] + 3 : -1;
                        if (cl < 0) break;  // set full
                        const uint32_t got = atomicCAS(&sh.keys[cl], SC_EMPTY, k);
                        if (got == SC_EMPTY) { sl[b] = cl; newmask |= 1u << (c0 + b); }
                        else if (got == k) sl[b] = cl;
                    }
                }
            }
        }
#pragma unroll
        for (int b = 0; b < SC_BATCH; b++) {
            const int c = c0 + b;
            slot[c] = sl[b];
            if (vc[b] && sl[b] >= 0) {
                atomicAdd((unsigned long long*)&sh.valx[sl[b]], (unsigned long long)sc_fix(v[2 * c], L.k));
                atomicAdd((unsigned long long*)&sh.valy[sl[b]], (unsigned long long)sc_fix(v[2 * c + 1], L.k));
            }
        }
        bool full = false;
#pragma unroll
        for (int b = 0; b < SC_BATCH; b++) full |= vc[b] && sl[b] < 0;
        if (__ballot(full)) {  // uniform: some lane's set is full of other entries
#pragma unroll
            for (int b = 0; b < SC_BATCH; b++) {
                const int c = c0 + b;
                if (vc[b] && sl[b] < 0) {
                    if (v[2 * c] != 0.f) atomicAdd(grad + 2 * (size_t)(L.off + e[c]), v[2 * c]);
                    if (v[2 * c + 1] != 0.f) atomicAdd(grad + 2 * (size_t)(L.off + e[c]) + 1, v[2 * c + 1]);
                }
            }
        }
    }
    // append the claimed slots to `used`: one LDS atomic per wave
    const int mine = __builtin_popcount(newmask);
    const float incl = wave_incl_sum_dpp((float)mine);
    const int wtot = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
    if (wtot) {
        int base = 0;
        if (lane == 0) base = atomicAdd(sh.fill, wtot);
        base = __builtin_amdgcn_readfirstlane(base);
        int pos = base + (int)incl - mine;
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (newmask & (1u << c)) sh.used[pos++] = (uint16_t)slot[c];
    }
}

// Sample position in [0,1]^3 as the forward computes it ((x - min) / extent; a power-of-two
// extent — 1.0 at the configs' scale 0.5 — multiplies by its exact reciprocal instead).
struct ScNorm {
    float mn, ext, inv;
    bool pow2;
    __device__ __forceinline__ float operator()(float v) const { return pow2 ? (v - mn) * inv : (v - mn) / ext; }
};

// The encoding gradient as the MLP pass stored it (field_bwd_kernel): pairs of the operand type, fp16
// at the chain's loss scale or bf16 unscaled; decoded to f32 and unscaled (1/S: a power of two, exact).
struct ScDE {
    float inv;
    bool bf16;
    __device__ __forceinline__ float2 operator()(uint32_t w) const {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 h = __builtin_bit_cast(h2, w);
        const float x = bf16 ? __uint_as_float(w << 16) : (float)h[0];
        const float y = bf16 ? __uint_as_float(w & 0xFFFF0000u) : (float)h[1];
        return make_float2(x * inv, y * inv);
    }
};

__device__ __forceinline__ void sc_corner_sums(const LevelPos& p, float2 g, float (&v)[16]) {
    // corner weights in the forward's association ((wx * wy) * wz)
    const float wx[2] = {1.0f - p.fx, p.fx}, wy[2] = {1.0f - p.fy, p.fy}, wz[2] = {1.0f - p.fz, p.fz};
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
        v[2 * c] = fmaf(w, g.x, v[2 * c]);
        v[2 * c + 1] = fmaf(w, g.y, v[2 * c + 1]);
    }
}

// A lane's C consecutive samples (normalised positions and dE of the unit's level), loaded at the
// start of the unit in one batch; samples past the end carry dE = 0.
template <int C>
struct ScChunk {
    float x[C], y[C], z[C];
    float2 g[C];
};
// C is 2 or 4 and the lane's first sample sb a multiple of C: the chunk's xyz (12C bytes) and dE
// (4C bytes) are 16-B (C = 4) / 8-B (C = 2) aligned pieces, loaded with dwordx4 / dwordx2 — a lane
// reads contiguous bytes, so fewer, wider load instructions (the lane-strided pattern costs TA
// cycles per touched cache line).  A partial last chunk falls back to per-sample loads.
template <int C>
__device__ __forceinline__ void sc_load_de(ScChunk<C>& ch, const uint32_t* __restrict__ p, const ScDE& de) {
    if constexpr (C == 4) {
        const uint4 v = *(const uint4*)p;
        ch.g[0] = de(v.x); ch.g[1] = de(v.y); ch.g[2] = de(v.z); ch.g[3] = de(v.w);
    } else {
        const uint2 v = *(const uint2*)p;
        ch.g[0] = de(v.x); ch.g[1] = de(v.y);
    }
}
// xyzs: the unit class's permuted positions (sc_perm) with pb = the chunk's place in them, or (with
// `order`, pb unused) the sample-ordered positions gathered through order.
template <int C>
__device__ __forceinline__ void sc_load_chunk(ScChunk<C>& ch, int64_t sb, int64_t pb, int64_t s1,
                                               const float* __restrict__ xyzs, const uint32_t* __restrict__ dEl,
                                               const ScDE& de, const ScNorm& nrm, const int32_t* __restrict__ order) {
    static_assert(C == 2 || C == 4, "chunk of 2 or 4 samples");
    float xs[3 * C];
    if (order) {  // positions sb.. in processing order: dE contiguous, positions gathered
        int64_t src[C];
#pragma unroll
        for (int i = 0; i < C; i++) src[i] = sb + i < s1 ? (int64_t)order[sb + i] : -1;
        if (sb + C <= s1) {
            sc_load_de<C>(ch, dEl + sb, de);
        } else {
#pragma unroll
            for (int i = 0; i < C; i++) ch.g[i] = src[i] >= 0 ? de(dEl[sb + i]) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < C; i++) {
            const int64_t sc = src[i] >= 0 ? src[i] : 0;
            xs[3 * i] = xyzs[3 * sc];
            xs[3 * i + 1] = xyzs[3 * sc + 1];
            xs[3 * i + 2] = xyzs[3 * sc + 2];
        }
    } else if (sb + C <= s1) {
        if constexpr (C == 4) {
            const float4* px = (const float4*)(xyzs + 3 * pb);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const float4 v = px[q];
                xs[4 * q] = v.x; xs[4 * q + 1] = v.y; xs[4 * q + 2] = v.z; xs[4 * q + 3] = v.w;
            }
        } else {
            const float2* px = (const float2*)(xyzs + 3 * pb);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const float2 v = px[q];
                xs[2 * q] = v.x; xs[2 * q + 1] = v.y;
            }
        }
        sc_load_de<C>(ch, dEl + sb, de);
    } else {
#pragma unroll
        for (int i = 0; i < C; i++) {
            const bool in = sb + i < s1;
            const int64_t sc = in ? sb + i : 0, pc = in ? pb + i : 0;
            ch.g[i] = in ? de(dEl[sc]) : make_float2(0.f, 0.f);
            xs[3 * i] = in ? xyzs[3 * pc] : 0.f;
            xs[3 * i + 1] = in ? xyzs[3 * pc + 1] : 0.f;
            xs[3 * i + 2] = in ? xyzs[3 * pc + 2] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < C; i++) {
        ch.x[i] = nrm(xs[3 * i]);
        ch.y[i] = nrm(xs[3 * i + 1]);
        ch.z[i] = nrm(xs[3 * i + 2]);
    }
}

// Fine levels: the lane's consecutive samples in the same cell are summed in registers (a run), and
// a run's 8 corners go to the table when the cell changes (sc_add is called by the whole wave;
// lanes without a finished run take part with zeros).
template <int C>
__device__ __forceinline__ void sc_direct(ScShared& sh, int lane, const ScChunk<C>& ch, const ScLevel& L,
                                          float* __restrict__ grad) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = 0.f;
    LevelPos p = level_pos(L.scale, ch.x[0], ch.y[0], ch.z[0]);
    sc_corner_sums(p, ch.g[0], v);
#pragma unroll
    for (int i = 1; i <= C; i++) {
        LevelPos q = p;
        bool emit = true;
        if (i < C) {
            q = level_pos(L.scale, ch.x[i], ch.y[i], ch.z[i]);
            emit = q.px != p.px || q.py != p.py || q.pz != p.pz;
        }
        if (__ballot(emit)) {  // uniform
            float ve[16];
#pragma unroll
            for (int j = 0; j < 16; j++) ve[j] = emit ? v[j] : 0.f;
            sc_add(sh, lane, p.px, p.py, p.pz, ve, L, grad);
        }
        if (i < C) {
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = emit ? 0.f : v[j];
            sc_corner_sums(q, ch.g[i], v);
        }
        p = q;
    }
}

// ---- cell-keyed form (coarse levels) ----
// One LDS lookup per run instead of one per corner: the run's cell (px, py, pz) is the key
// (px | py << 11 | pz << 22; cells outside that range go straight to global memory) and its 8
// corners' sums are 16 ds_add_u64 into the slot's corner arrays.  The flush forms each claimed
// cell's corner entries and adds them to the table gradient (a corner shared by several cells of
// the unit gets one global add per cell: coarse levels have few cells per unit).
__device__ __forceinline__ uint32_t sc_corner_entry(const ScLevel& L, uint32_t px, uint32_t py, uint32_t pz, int c) {
    const uint32_t x = px + (c & 1), y = py + ((c >> 1) & 1), z = pz + ((c >> 2) & 1);
    if (L.dense) {
        const uint32_t e = x + L.res * y + L.res * L.res * z;
        return e < L.params ? e : e % L.params;
    }
    return (x ^ (y * 2654435761u) ^ (z * 805459861u)) & (L.params - 1);
}

// A lane's run of consecutive samples in one cell of a coarse level: the 8 corners' weighted sums
// in registers, carried over the lane's chunks of a unit; a finished run goes to the wave's queue
// (sc_push_run), whose full-wave passes add the runs to the cell table (sc_drain_cells).
struct ScRun {
    uint32_t px, py, pz;
    bool any, init;
    float v[16];
};

// Diagnostic builds (tools/scatter_probe.py): NCN_DIAG_SC_TIMES records wave 0's cycles per phase of
// the fine-level units; NCN_DIAG_SC_LEVELS_MASK skips the levels whose bit is clear.
#ifdef NCN_DIAG_SC_SPAN
__device__ unsigned long long ncn_sc_span[256][20];  // per workgroup: realtime (100 MHz) start/end, cycles start/end,
                                                     // then (unit, realtime at its end) for the first 8 units
#endif
#ifdef NCN_DIAG_SC_TIMES
__device__ unsigned long long ncn_sc_times[256][10];  // per workgroup, wave 0: cycles per phase
#define SC_TNOW(v) const unsigned long long v = __builtin_readcyclecounter()
#define SC_TADD(i, a, b) if (threadIdx.x == 0 && blockIdx.x < 256) ncn_sc_times[blockIdx.x][(i) * 2 + 1] += (b) - (a)
#define SC_TADDC(i, a, b) if (threadIdx.x == 0 && blockIdx.x < 256) ncn_sc_times[blockIdx.x][(i) * 2] += (b) - (a)
#define SC_TWAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define SC_TNOW(v)
#define SC_TADD(i, a, b)
#define SC_TADDC(i, a, b)
#define SC_TWAIT()
#endif

// The wave's queued runs [0, qn) into the cell table, one run per lane: one set read and claim per
// run, the 16 sums as fixed-point ds_add_u64 in four float4 groups; a run whose set is full goes to
// global f32 atomics.
__device__ __forceinline__ void sc_drain_cells(ScShared& sh, int lane, const uint32_t* qk, const float4* qv, int qn,
                                               const ScLevel& L, float* __restrict__ grad) {
    asm volatile("" ::: "memory");  // (the wave's queue writes come first: a wave's LDS operations execute in order)
    SC_TNOW(td0);
    const bool act = lane < qn;
    const uint32_t key = act ? qk[lane] : 0u;
    const int p0 = SC_WAYS * (int)sc_set(key, sh.sets);
    int sl = -1;
    bool isnew = false;
    uint4 kk = make_uint4(0u, 0u, 0u, 0u);
    if (act) {
        kk = *(const uint4*)&sh.keys[p0];
        sl = kk.x == key ? p0 : kk.y == key ? p0 + 1 : kk.z == key ? p0 + 2 : kk.w == key ? p0 + 3 : -1;
    }
    if (__ballot(act && sl < 0)) {  // uniform: some lane claims
        if (act && sl < 0) {
#pragma unroll
            for (int attempt = 0; attempt < 2 && sl < 0; attempt++) {
                if (attempt) {  // lost a claim: look again
                    asm volatile("" ::: "memory");
                    kk = *(const uint4*)&sh.keys[p0];
                    sl = kk.x == key ? p0 : kk.y == key ? p0 + 1 : kk.z == key ? p0 + 2 : kk.w == key ? p0 + 3 : -1;
                    if (sl >= 0) break;
                }
                const int cl = kk.x == SC_EMPTY ? p0 : kk.y == SC_EMPTY ? p0 + 1 : kk.z == SC_EMPTY ? p0 + 2
                             : kk.w == SC_EMPTY ? p0 + 3 : -1;
                if (cl < 0) break;  // set full
                const uint32_t got = atomicCAS(&sh.keys[cl], SC_EMPTY, key);
                if (got == SC_EMPTY) { sl = cl; isnew = true; }
                else if (got == key) sl = cl;
            }
        }
    }
    const bool fb = act && sl < 0;
    const bool anyfb = __ballot(fb) != 0;  // uniform: a set full of other cells
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const float4 v = act ? qv[4 * lane + g] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int j = 4 * g + h;  // corner j / 2, component j % 2
            if (act && sl >= 0)
                atomicAdd((unsigned long long*)&sh.valx[j * sh.slots + sl], (unsigned long long)sc_fix(vv[h], L.k));
        }
        if (anyfb && fb) {
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const int j = 4 * g + h;
                const uint32_t e = L.off + sc_corner_entry(L, key & 2047u, (key >> 11) & 2047u, key >> 22, j >> 1);
                if (vv[h] != 0.f) atomicAdd(grad + 2 * (size_t)e + (j & 1), vv[h]);
            }
        }
    }
    // append the claimed slots to `used`: one LDS atomic per wave
    const uint64_t nm = __ballot(isnew);
    if (nm) {
        int base = 0;
        if (lane == 0) base = atomicAdd(sh.fill, (int)__popcll(nm));
        base = __builtin_amdgcn_readfirstlane(base);
        if (isnew)
            sh.used[base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0))] =
                (uint16_t)sl;
    }
    asm volatile("" ::: "memory");  // (the queue is rewritten after these reads)
    SC_TWAIT();
    SC_TNOW(td1);
    SC_TADDC(2, td0, td1);
}

// Queue the finished runs of the lanes with `fin` (whole wave calls; qn wave-uniform): a full queue
// is drained first.  Cells outside the key range go straight to global memory.
__device__ __forceinline__ void sc_push_run(ScShared& sh, int lane, bool fin, const ScRun& st, uint32_t* qk, float4* qv,
                                            int& qn, const ScLevel& L, float* __restrict__ grad) {
    const bool inkey = st.px < 2048u && st.py < 2048u && st.pz < 1024u;
    const uint64_t bm = __ballot(fin && inkey);
    if (bm) {
        const int n = (int)__popcll(bm);
        if (qn + n > SC_QUEUE) {
            sc_drain_cells(sh, lane, qk, qv, qn, L, grad);
            qn = 0;
        }
        if (fin && inkey) {
            const int p = qn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0));
            qk[p] = st.px | (st.py << 11) | (st.pz << 22);
#pragma unroll
            for (int g = 0; g < 4; g++)
                qv[4 * p + g] = make_float4(st.v[4 * g], st.v[4 * g + 1], st.v[4 * g + 2], st.v[4 * g + 3]);
        }
        qn += n;
    }
    if (__ballot(fin && !inkey)) {  // uniform: (not on the configs' levels) straight to global memory
        if (fin && !inkey) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const uint32_t e = L.off + sc_corner_entry(L, st.px, st.py, st.pz, c);
                if (st.v[2 * c] != 0.f) atomicAdd(grad + 2 * (size_t)e, st.v[2 * c]);
                if (st.v[2 * c + 1] != 0.f) atomicAdd(grad + 2 * (size_t)e + 1, st.v[2 * c + 1]);
            }
        }
    }
}
template <int C>
__device__ __forceinline__ void sc_cells_run(ScShared& sh, int lane, const ScChunk<C>& ch, const ScLevel& L,
                                             float* __restrict__ grad, ScRun& st, bool last, uint32_t* qk, float4* qv,
                                             int& qn) {
#pragma unroll
    for (int i = 0; i < C; i++) {
        const LevelPos q = level_pos(L.scale, ch.x[i], ch.y[i], ch.z[i]);
        const bool change = st.init && (q.px != st.px || q.py != st.py || q.pz != st.pz);
        sc_push_run(sh, lane, change && st.any, st, qk, qv, qn, L, grad);
        if (change || !st.init) {
#pragma unroll
            for (int j = 0; j < 16; j++) st.v[j] = 0.f;
            st.any = false;
            st.px = q.px; st.py = q.py; st.pz = q.pz;
            st.init = true;
        }
        st.any = st.any || ch.g[i].x != 0.f || ch.g[i].y != 0.f;
        sc_corner_sums(q, ch.g[i], st.v);
    }
    if (last) {  // the unit's last runs, then the rest of the queue
        sc_push_run(sh, lane, st.any, st, qk, qv, qn, L, grad);
        if (qn) sc_drain_cells(sh, lane, qk, qv, qn, L, grad);
        qn = 0;
    }
}

// Flush of a cell unit: 16 lanes per claimed cell (one corner component each), form the corner's
// entry, f32 global adds; lane 0 of the cell resets the key, each lane its value.
__device__ __forceinline__ void sc_flush_cells(ScShared& sh, const ScLevel& L, float* __restrict__ grad) {
    const int nf = *sh.fill;
    constexpr int V = SC_CELL_VALS;
    for (int i = threadIdx.x; i < V * nf; i += SC_THREADS) {
        const int slot = sh.used[i / V], j = i % V;
        const uint32_t key = sh.keys[slot];
        long long* pv = &sh.valx[j * sh.slots + slot];
        const long long q = *pv;
        *pv = 0;
        if (q != 0) {
            const uint32_t e = L.off + sc_corner_entry(L, key & 2047u, (key >> 11) & 2047u, key >> 22, j >> 1);
            atomicAdd(grad + 2 * (size_t)e + (j & 1), (float)ldexp((double)q, -L.k));
        }
        if (j == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the cell's other lanes have read the key: same wave)
            sh.keys[slot] = SC_EMPTY;
        }
    }
}


__device__ __forceinline__ ScLevel sc_level(const LevelTable& Lt, int l, float m, int kbase) {
    ScLevel L;
    L.scale = Lt.scale[l];
    L.res = Lt.res[l];
    L.params = Lt.params[l];
    L.off = Lt.offset[l];
    L.dense = (uint64_t)L.res * L.res * L.res <= L.params;  // tcnn: stride stays <= params
    L.direct = !isfinite(m);  // (uniform) non-finite gradient: every corner straight to global memory
    int e2 = 0;
    (void)frexpf(L.direct ? 1.f : m, &e2);  // m < 2^e2
    // |sum| <= (unit samples) * m * 2^k + rounding (a sample's 8 corner weights sum to 1): < 2^62,
    // and every addend (a run's corner sum) < 2^51, sc_fix's range (the callers' kbase)
    L.k = kbase - e2;
    return L;
}

// The next unit of the workgroup (field_scatter_kernel's queue): thread 0 draws it when its samples
// are done (few live registers there; the atomic's return is hidden behind the unit's barrier wait
// and flush) and publishes it in LDS before the unit's closing barrier.
struct ScDraw {
    unsigned* queue;
    int* slot;
};

// One fine-level unit of 1024 x C samples: the samples in grabs, then the flush of the claimed slots.
// (C is a run-time value: one inlined copy of the grab loop serves every fine level.)
__device__ __forceinline__ void sc_unit(ScShared& sh, int wid, int lane, int l, int C, int64_t s0, int64_t s1,
                                        const float* __restrict__ xyzs, const uint32_t* __restrict__ dEl,
                                        const ScDE& de, const ScNorm& nrm, const LevelTable& Lt, float m, float* __restrict__ grad,
                                        const int32_t* __restrict__ order, bool perm, const ScDraw& draw) {
    SC_TNOW(t0);
    // (a fine unit holds at most 4096 samples: 2^46 leaves the sums four bits of headroom below 2^62)
    const ScLevel L = sc_level(Lt, l, m, 46);
    SC_TNOW(t1);
    // The unit's 1024 x C samples in grabs of 64 lanes x 2: grab k gives lane t the samples
    // s0 + (t * NG + k) * 2 — the 64 lanes of one wave-instruction hold samples 2 * NG positions
    // apart, so they rarely address the same LDS slot at once (same-address LDS atomics
    // serialise).  Wave w takes grab w first, then draws grabs from the unit's LDS counter after
    // each grab's adds, so a wave slowed by claims / set-full fallbacks takes fewer grabs and the
    // waves reach the unit's barrier together (191 vs 195 us static; drawing one grab ahead so
    // that its loads overlap spills 9 VGPRs: 194).  Round 5: level 15's 2048-sample units go through
    // the same loop (16 grabs for 16 waves: the assignment of the former static 2-sample chunks; one
    // code path, 186-188 vs 189-190 us in the probe); 1-sample grabs (finer balance, shorter runs) on
    // levels 13-15 were no better.
    const int NG = SC_THREADS * C / 128;
    int k = wid;
    ScChunk<2> cg;
    // (positions: the class array holds grab k's 64 chunks of 2 side by side, sc_perm)
#define SC_GRAB_S(k) (s0 + ((int64_t)lane * NG + (k)) * 2)
#define SC_GRAB_P(k) (perm ? s0 + ((int64_t)(k) * 64 + lane) * 2 : SC_GRAB_S(k))
    sc_load_chunk<2>(cg, SC_GRAB_S(k), SC_GRAB_P(k), s1, xyzs, dEl, de, nrm, order);
    while (k < NG) {  // (wave-uniform)
        sc_direct<2>(sh, lane, cg, L, grad);
        int kn = 0;
        if (lane == 0) kn = atomicAdd(sh.grab, 1);
        kn = __builtin_amdgcn_readfirstlane(kn) + SC_WAVES;
        if (kn < NG) sc_load_chunk<2>(cg, SC_GRAB_S(kn), SC_GRAB_P(kn), s1, xyzs, dEl, de, nrm, order);
        k = kn;
    }
    SC_TNOW(t2);
#ifdef NCN_DIAG_SC_TIMES
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (diagnostic: the wave's own LDS ops drain)
#endif
    SC_TNOW(t2b);
    unsigned next = 0;
    if (threadIdx.x == 0) next = atomicAdd(draw.queue, 1u);  // (its return waits behind the barrier and the flush)
    lds_barrier();
    SC_TNOW(t3);
    // flush: the claimed slots, two lanes per slot (x and y of one entry are adjacent floats, one
    // 8-B piece of one 64-B granule per lane pair); each lane resets the half it read (the even
    // lane the key and x, the odd one y), so one barrier closes the unit
    const int nf = *sh.fill;
    for (int i = threadIdx.x; i < 2 * nf; i += SC_THREADS) {
        const int slot = sh.used[i >> 1];
        const uint32_t key = sh.keys[slot];
        long long* pv = (i & 1) ? &sh.valy[slot] : &sh.valx[slot];
        const float gv = (float)ldexp((double)*pv, -L.k);
        *pv = 0;
        if (gv != 0.f) atomicAdd(grad + 2 * (size_t)(L.off + key) + (i & 1), gv);
        if (!(i & 1)) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the odd lane has read the key: same wave)
            sh.keys[slot] = SC_EMPTY;
        }
    }
    if (threadIdx.x == 0) *draw.slot = (int)next;
    lds_barrier();
    SC_TNOW(t4);
    SC_TADD(0, t0, t1);
    SC_TADD(1, t1, t2);
    SC_TADD(2, t2, t2b);
    SC_TADD(3, t2b, t3);
    SC_TADD(4, t3, t4);
}

// Cell units: 1024 x C x `rounds` consecutive samples, then one flush.  Lane t of wave w takes the
// unit's (t * SC_WAVES + w)-th slice of C x rounds consecutive samples (neighbouring slices in
// different waves), a chunk of C per round, and carries its current run over the rounds, so a run
// ends only where the samples leave the cell.  Rounds per level: coarse levels have few cells, so
// longer units mean fewer flushes and barriers.  (Round 5: carried runs with the next chunk loaded
// at the top of the round, no prefetch: levels 0-9 95 -> 75 us, all levels 201 -> 192 us; with the
// prefetch the carried state spilled 18 VGPRs: 199 us.)
#ifndef NCN_SC_R_LO
#define NCN_SC_R_LO 8
#endif
#ifndef NCN_SC_R_MID
#define NCN_SC_R_MID 4
#endif
__host__ __device__ constexpr int sc_cell_rounds(int l) { return l < 6 ? NCN_SC_R_LO : l < 10 ? NCN_SC_R_MID : 1; }
// samples of one unit of level l
__host__ __device__ constexpr int64_t sc_unit_span(int l) {
    return (int64_t)SC_THREADS * (l < SC_CELL_HI ? SC_C_CELL * sc_cell_rounds(l) : sc_fine_c(l));
}

template <int C>
__device__ __forceinline__ void sc_cell_unit(ScShared& sh, int wid, int lane, int l, int64_t s0, int64_t s1, int rounds,
                                             const float* __restrict__ xyzs, const uint32_t* __restrict__ dEl,
                                             const ScDE& de, const ScNorm& nrm, const LevelTable& Lt, float m, float* __restrict__ grad,
                                             const int32_t* __restrict__ order, bool perm, const ScDraw& draw) {
    const int lg_unit = (31 - __builtin_clz(SC_THREADS * C)) + (31 - __builtin_clz((unsigned)rounds));
    // scale 2^k, k = 60 - lg_unit - e: the unit's sum of every corner stays below 2^61, and one run
    // (at most rounds x C <= 2^(lg_unit - 10) samples) below 2^(50) — sc_fix needs |addend| < 2^51
    const ScLevel L = sc_level(Lt, l, m, 60 - lg_unit);
    const int64_t lane_off = ((int64_t)lane * SC_WAVES + wid) * rounds * C;
    ScRun st;
    st.init = st.any = false;
    st.px = st.py = st.pz = 0;
    uint32_t* qk = sh.qkey + wid * SC_QUEUE;  // (this wave's run queue)
    float4* qv = sh.qval + wid * SC_QUEUE * 4;
    int qn = 0;
    for (int r = 0; r < rounds; r++) {
        ScChunk<C> ch;
        // (positions: the class array holds a round's 64 chunks of a wave side by side, sc_perm)
        const int64_t sb = s0 + lane_off + (int64_t)r * C;
        SC_TNOW(tc0);
        sc_load_chunk<C>(ch, sb, perm ? s0 + (((int64_t)r * SC_WAVES + wid) * 64 + lane) * C : sb, s1, xyzs, dEl, de, nrm,
                         order);
        SC_TWAIT();
        SC_TNOW(tc1);
        SC_TADDC(0, tc0, tc1);
        if (L.direct)
            sc_direct<C>(sh, lane, ch, L, grad);  // (sc_add's direct form: f32 global adds, NaN/Inf propagate)
        else
            sc_cells_run<C>(sh, lane, ch, L, grad, st, r + 1 == rounds, qk, qv, qn);
        SC_TWAIT();
        SC_TNOW(tc2);
        SC_TADDC(1, tc1, tc2);  // (run work including the drains, which add to slot 2 as well)
    }
    SC_TNOW(tc3);
    unsigned next = 0;
    if (threadIdx.x == 0) next = atomicAdd(draw.queue, 1u);  // (its return waits behind the barrier and the flush)
    lds_barrier();
    SC_TNOW(tc4);
    sc_flush_cells(sh, L, grad);
    if (threadIdx.x == 0) *draw.slot = (int)next;
    lds_barrier();
    SC_TNOW(tc5);
    SC_TADDC(3, tc3, tc4);
    SC_TADDC(4, tc4, tc5);
}

// Unit classes by the sample layout their loads use: coarse levels 0-5 (rounds NCN_SC_R_LO) and 6-9
// (NCN_SC_R_MID), fine levels 10-14 (C = 4) and 15 (C = 2).
constexpr int SC_N_CLASSES = 4;
__host__ __device__ constexpr int sc_class(int l) { return l < 6 ? 0 : l < SC_CELL_HI ? 1 : l < 15 ? 2 : 3; }
constexpr int64_t SC_MAX_SPAN = (int64_t)SC_THREADS * SC_C_CELL * NCN_SC_R_LO;
static_assert(sc_cell_rounds(0) == NCN_SC_R_LO && NCN_SC_R_LO >= NCN_SC_R_MID && sc_fine_c(10) <= SC_C_CELL, "spans");
// the permuted positions' row length (every class array holds whole units)
__host__ __device__ constexpr int64_t sc_perm_stride(int64_t n_stride) {
    return (n_stride + SC_MAX_SPAN - 1) / SC_MAX_SPAN * SC_MAX_SPAN;
}
__host__ __device__ int64_t de_queue_offset(int64_t e_stride) {
    return DE_HEADER_FLOATS + 16 * e_stride + SC_N_CLASSES * 3 * sc_perm_stride(e_stride);
}
// Where sample s sits in its class's permuted position array: the samples a wave loads in one
// instruction lie side by side, so a coarse round or a fine grab reads one contiguous stretch
// (coalesced) while each lane keeps its own consecutive samples (the runs).  Coarse: lane t of wave
// w owns the unit's slice t * 16 + w of 4R samples and reads chunk r in round r; fine: lane t reads
// the pair t * NG + k in grab k.  A chunk (4 coarse / 2 fine samples) stays contiguous.
__device__ __forceinline__ int64_t sc_perm(int64_t s, int cls) {
    if (cls < 2) {
        const int R = sc_cell_rounds(cls == 0 ? 0 : 6), CR = SC_C_CELL * R;
        const int64_t U = (int64_t)SC_THREADS * CR, o = s % U;
        const int64_t slice = o / CR, within = o % CR;
        const int64_t t = slice / SC_WAVES, w = slice % SC_WAVES, r = within / SC_C_CELL, i = within % SC_C_CELL;
        return (s - o) + ((r * SC_WAVES + w) * 64 + t) * SC_C_CELL + i;
    }
    const int C = sc_fine_c(cls == 2 ? 10 : 15), NG = SC_THREADS * C / 128;
    const int64_t U = (int64_t)SC_THREADS * C, o = s % U;
    const int64_t pair = o >> 1, t = pair / NG, k = pair % NG;
    return (s - o) + (k * 64 + t) * 2 + (o & 1);
}

// The sample positions in the permuted order of each class the scatter needs (class_mask), into
// the dE workspace behind the encoding gradient: a thread takes 4 consecutive samples (one 48-B
// piece in, one 48-B coarse chunk / two 24-B fine pairs out per class).
__global__ __launch_bounds__(256) void sc_perm_positions_kernel(const float* __restrict__ xyzs, int64_t n_stride,
                                                                const int32_t* __restrict__ n_dev, int class_mask,
                                                                float* __restrict__ xyz_perm, float* __restrict__ flag,
                                                                float flag_value) {
    const int64_t n = n_dev ? min<int64_t>(n_stride, *n_dev) : n_stride;
    if (blockIdx.x == 0 && threadIdx.x == 0) *flag = flag_value;
    const int64_t ps = sc_perm_stride(n_stride);
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; 4 * j < n; j += (int64_t)gridDim.x * 256) {
        const int64_t sb = 4 * j;
        float v[12];
        if (sb + 4 <= n) {
            const float4* px = (const float4*)(xyzs + 3 * sb);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const float4 f = px[q];
                v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 12; i++) v[i] = sb + i / 3 < n ? xyzs[3 * sb + i] : 0.f;
        }
#pragma unroll
        for (int cls = 0; cls < SC_N_CLASSES; cls++) {
            if (!((class_mask >> cls) & 1)) continue;
            float* out = xyz_perm + cls * 3 * ps;
            if (cls < 2) {  // the 4 samples are one chunk
                float4* po = (float4*)(out + 3 * sc_perm(sb, cls));
                po[0] = make_float4(v[0], v[1], v[2], v[3]);
                po[1] = make_float4(v[4], v[5], v[6], v[7]);
                po[2] = make_float4(v[8], v[9], v[10], v[11]);
            } else {  // two pairs
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    float2* po = (float2*)(out + 3 * sc_perm(sb + 2 * h, cls));
                    po[0] = make_float2(v[6 * h], v[6 * h + 1]);
                    po[1] = make_float2(v[6 * h + 2], v[6 * h + 3]);
                    po[2] = make_float2(v[6 * h + 4], v[6 * h + 5]);
                }
            }
        }
    }
}

// One unit u of the scatter (see field_scatter_kernel): its level, span and layout.
__device__ __forceinline__ bool sc_one_unit(int64_t u, int64_t n, const int* unit_start, const int* unit_level, int& layout,
                                            int& par, const ScDraw& draw, ScShared& sh,
                                            char* arena, int* fill, const float* lmax_s, int wid, int lane,
                                            const float* __restrict__ xyzs, const float* __restrict__ pos, int perm_mask,
                                            const uint32_t* __restrict__ dE,
                                            int64_t e_stride, const ScDE& de, const ScNorm& nrm, const LevelTable& Lt,
                                            float* __restrict__ grad, const int32_t* __restrict__ order) {
    int i = 0;  // (uniform) unit u is unit v of level l
    while (i < 15 && u >= unit_start[i + 1]) i++;
    const int l = unit_level[i];
    const int64_t v = u - unit_start[i], span = sc_unit_span(l);
    const int64_t s0 = v * span, s1 = min(n, s0 + span);
    const int mode = l < SC_CELL_HI ? SC_MODE_CELL : SC_MODE_DIR;
    if (mode != layout) {  // (re)initialise the table of the new layout
        lds_barrier();
        sh = sc_layout(arena, fill, mode);
        const int nv = mode == SC_MODE_CELL ? SC_CELL_VALS * sh.slots : 2 * sh.slots;
        for (int i = threadIdx.x; i < sh.slots; i += SC_THREADS) sh.keys[i] = SC_EMPTY;
        for (int i = threadIdx.x; i < nv; i += SC_THREADS) sh.valx[i] = 0;
        if (threadIdx.x == 0) fill[0] = fill[1] = fill[2] = fill[3] = 0;
        lds_barrier();
        layout = mode;
        par = 0;
    }
    float m = lmax_s[l];
#ifdef NCN_DIAG_SC_LEVELS_MASK
    if (!((NCN_DIAG_SC_LEVELS_MASK >> l) & 1)) m = 0.f;  // diagnostic: skip this level
#endif
    if (m == 0.f) return false;  // uniform: nothing to add on this level (no barrier, parity kept; no draw)
    // the unit claims into fill[par]; fill[par ^ 1] (read by every lane before the previous
    // unit's closing barrier) is reset here for the next unit
    sh.fill = fill + par;
    sh.grab = fill + 2 + par;  // (the grab counters behind the claim counts, alternating alike)
    if (threadIdx.x == 0) { fill[par ^ 1] = 0; fill[2 + (par ^ 1)] = 0; }
    par ^= 1;
    const uint32_t* dEl = dE + (int64_t)l * e_stride;
    // (positions: the level's class array, or the sample-ordered ones)
    const bool perm = (perm_mask >> sc_class(l)) & 1;
    if (perm) xyzs = pos + sc_class(l) * 3 * sc_perm_stride(e_stride);
    if (mode == SC_MODE_CELL)
        sc_cell_unit<SC_C_CELL>(sh, wid, lane, l, s0, s1, sc_cell_rounds(l), xyzs, dEl, de, nrm, Lt, m, grad, order, perm,
                                draw);
    else
        sc_unit(sh, wid, lane, l, sc_fine_c(l), s0, s1, xyzs, dEl, de, nrm, Lt, m, grad, order, perm, draw);
    return true;
}

// (ncn_field_scatter_wgrad) the MLP weight-gradient slab rows summed into gw, in SC_WGRAD_SLICES
// contiguous slices of the weights, one per queue entry behind the table units (so the workgroups that
// finish their table units first take them; round 6: the reduction at the start of every workgroup
// delayed all units by its duration): the threads of a slice take (weight, 16-row chunk) pairs with
// the weight varying fastest (coalesced rows); one f32 atomic per pair, as reduce_wgrad_kernel.
constexpr int SC_WGRAD_SLICES = 256;
__device__ __forceinline__ void sc_wgrad_slice(int slice, const float* __restrict__ wslab, int nb_sigma, int nb_rgb,
                                               float* __restrict__ gw) {
    const int per = (NCN_FIELD_NW + SC_WGRAD_SLICES - 1) / SC_WGRAD_SLICES;
    const int w0 = slice * per, nw = min(NCN_FIELD_NW, w0 + per) - w0;
    const int chunks = (max(nb_sigma, nb_rgb) + WRED_CHUNK - 1) / WRED_CHUNK;
    for (int idx = threadIdx.x; idx < nw * chunks; idx += SC_THREADS) {
        const int w = w0 + idx % nw, c = idx / nw;
        const int nb = w < W3_OFF ? nb_sigma : nb_rgb;
        const int b1 = min(nb, (c + 1) * WRED_CHUNK);
        float acc = 0.f;
        for (int b = c * WRED_CHUNK; b < b1; b++) acc += wslab[(int64_t)b * NCN_FIELD_NW + w];
        if (c * WRED_CHUNK < nb) atomicAdd(gw + w, acc);
    }
}

__global__ __launch_bounds__(SC_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void field_scatter_kernel(const float* __restrict__ xyzs, int64_t n_stride,
                                                                   const int32_t* __restrict__ n_dev, LevelTable Lt,
                                                                   float xyz_min, float xyz_extent,
                                                                   const float* __restrict__ dE_ws,
                                                                   float* __restrict__ grad,
                                                                   const float* __restrict__ level_max, int lm_rows,
                                                                   int level_lo, int level_hi,
                                                                   const int32_t* __restrict__ order,
                                                                   const float* __restrict__ wslab = nullptr,
                                                                   int nb_sigma = 0, int nb_rgb = 0,
                                                                   float* __restrict__ gw = nullptr,
                                                                   unsigned* __restrict__ queue = nullptr) {
    __shared__ __attribute__((aligned(16))) char arena[SC_ARENA];
    __shared__ int fill[4];  // claimed-slot counts [0, 2) and grab counters [2, 4), alternating per unit (reset one unit ahead)
    // per-level max |dE| over the MLP pass's workgroup rows (the fixed-point scale of each level);
    // visible to every thread at the first layout barrier
    __shared__ float lmax_s[16];
    // the launch's levels in order: unit_start[i] = the first unit of the i-th of them (padded with
    // the unit count to 16), unit_level[i] its level
    __shared__ int unit_start[17], unit_level[16];
    const int64_t n = n_dev ? min<int64_t>(n_stride, *n_dev) : n_stride;
    if (threadIdx.x < 16) lmax_s[threadIdx.x] = 0.f;
    if (threadIdx.x == 0) {
        int acc = 0, k = 0;
        for (int l = level_lo; l < level_hi; l++) {
            unit_start[k] = acc;
            unit_level[k++] = l;
            acc += (int)((n + sc_unit_span(l) - 1) / sc_unit_span(l));
        }
        for (; k < 17; k++) unit_start[k] = acc;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < lm_rows * 16; i += SC_THREADS)  // one load per thread, LDS max
        atomicMax((unsigned*)&lmax_s[i & 15], __float_as_uint(level_max[i]));  // (non-negative floats)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#ifdef NCN_DIAG_SC_SPAN
    if (threadIdx.x == 0 && blockIdx.x < 256) {
        ncn_sc_span[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
        ncn_sc_span[blockIdx.x][2] = __builtin_readcyclecounter();
    }
#endif
    const int64_t e_stride = (n_stride + 3) & ~(int64_t)3;  // dE row stride (as written by field_bwd)
    ScNorm nrm;
    nrm.mn = xyz_min;
    nrm.ext = xyz_extent;
    nrm.inv = 1.0f / xyz_extent;
    nrm.pow2 = (__float_as_uint(xyz_extent) & 0x807FFFFFu) == 0u && xyz_extent > 0.f;
    // the MLP pass's dE workspace: header {1 / S, operand type}, then [16][e_stride] pairs
    ScDE de;
    de.inv = dE_ws[0];
    de.bf16 = dE_ws[1] != 0.f;
    const uint32_t* dE = (const uint32_t*)(dE_ws + DE_HEADER_FLOATS);
    // positions: a unit class's permuted copy behind dE when the MLP pass (or
    // ncn_field_scatter_positions) wrote it (header mask), else the sample-ordered xyzs (strided loads)
    const int perm_mask = order ? 0 : (int)dE_ws[DE_POS_FLAG];
    const float* pos = dE_ws + DE_HEADER_FLOATS + 16 * e_stride;
    // units of the levels [level_lo, level_hi), sc_unit_span(l) samples each: cell levels
    // [0, SC_CELL_HI) in spans of 1024 * C_CELL * rounds(l), fine levels 1024 * sc_fine_c(l)
    const int64_t n_units = unit_start[16], n_all = n_units + (wslab ? SC_WGRAD_SLICES : 0);
    // Units level-major (the cell levels' long units first): workgroup b takes unit b first, then draws
    // the next from the launch's queue — at the end of each unit's samples (ScDraw), so the draw's
    // return is hidden behind the unit's barrier wait and flush.  A workgroup's units go cell -> fine:
    // at most one layout switch.  (Round 6: the static stride b, b + gridDim.x, ... left the
    // workgroups' ends spread over 94-169 us for a mean of 142 us of work — about five units of 20-55
    // us each, profiles/round6/scatter_probe_span.log; with the queue 130-159 us and the scatter 175.8
    // -> 164-165 us, scatter_probe_queue_dynamic.log.  Fine levels drawn in cost order instead of
    // level-major, or coarse units of half the samples, measured no better: scatter_probe_order.log.)
    int layout = -1, par = 0;
    ScShared sh;
    __shared__ int next_unit[2];  // (alternating: a slot is rewritten only after a barrier every reader passed)
#ifdef NCN_DIAG_SC_SPAN
    int diag_k = 0;
#endif
    int64_t u = blockIdx.x;
    for (int qpar = 0; u < n_all; qpar ^= 1) {  // (uniform)
        ScDraw draw;
        draw.queue = queue;
        draw.slot = next_unit + qpar;
        bool drew = false;
        if (u < n_units)
            drew = sc_one_unit(u, n, unit_start, unit_level, layout, par, draw, sh, arena, fill, lmax_s, wid, lane, xyzs, pos,
                               perm_mask, dE, e_stride, de, nrm, Lt, grad, order);
        else
            sc_wgrad_slice((int)(u - n_units), wslab, nb_sigma, nb_rgb, gw);
#ifdef NCN_DIAG_SC_SPAN
        if (threadIdx.x == 0 && blockIdx.x < 256 && diag_k < 8) {
            ncn_sc_span[blockIdx.x][4 + 2 * diag_k] = (unsigned long long)u;
            ncn_sc_span[blockIdx.x][5 + 2 * diag_k] = __builtin_amdgcn_s_memrealtime();
        }
        diag_k++;
#endif
        if (!drew) {  // (uniform) a skipped unit: draw here
            if (threadIdx.x == 0) next_unit[qpar] = (int)atomicAdd(queue, 1u);
            __syncthreads();
        }
        u = (int64_t)next_unit[qpar] + gridDim.x;
    }
    // the last workgroup out leaves the queue zero for the next launch on this workspace (every
    // workgroup has made its last draw before it departs)
    if (threadIdx.x == 0 && atomicAdd(queue + 1, 1u) == gridDim.x - 1) {
        __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#ifdef NCN_DIAG_SC_SPAN
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 256) {
        ncn_sc_span[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
        ncn_sc_span[blockIdx.x][3] = __builtin_readcyclecounter();
    }
#endif
}

static int scatter_grid(int64_t n_cap) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(256 * 1024 / SC_THREADS, (n_cap + 255) / 256));  // 1024 threads per CU
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


constexpr int64_t NCN_FWD_MAX_BLOCKS = 4096;  // (round 5: 1792 / 2048 / 8192 blocks measured the same, 84-85 us)
static int fwd_grid(int64_t n) {
    const int64_t groups = (n + 15) / 16;
    const int64_t g = std::min<int64_t>(std::max<int64_t>((groups + 3) / 4, 1), NCN_FWD_MAX_BLOCKS);
    return (int)((g + 7) & ~(int64_t)7);  // a multiple of 8 (xcd_block)
}

}  // namespace ncn

using namespace ncn;

template <int PART>
static void launch_bwd_part(int precision, int nb, hipStream_t st, const float* xyzs, const float* dirs, int64_t n,
                            const int32_t* n_dev, const uint16_t* wp, const uint16_t* enc, const float* dsig,
                            const float* drgb, const float* loss_scale, float* dE_ws, float* slab, float* level_max,
                            const int32_t* order, const float* dsig2, float* stash) {
    if (precision == NCN_PREC_F16)
        hipLaunchKernelGGL((field_bwd_kernel<_Float16, PART>), dim3(nb), dim3(BWD_THREADS), 0, st, dirs, n, n_dev, wp,
                           (const Mfma<_Float16>::v8*)enc, dsig, drgb, loss_scale, dE_ws, slab, level_max, order, dsig2,
                           stash, xyzs);
    else
        hipLaunchKernelGGL((field_bwd_kernel<__bf16, PART>), dim3(nb), dim3(BWD_THREADS), 0, st, dirs, n, n_dev, wp,
                           (const Mfma<__bf16>::v8*)enc, dsig, drgb, loss_scale, dE_ws, slab, level_max, order, dsig2,
                           stash, xyzs);
}

extern "C" {

int ncn_field_pack_map(int32_t* src_index, void* stream) {
    hipLaunchKernelGGL(pack_map_kernel, dim3(N_FRAG32 + N_FRAG16), dim3(64), 0, (hipStream_t)stream, src_index);
    NCN_LAUNCH_CHECK("ncn_field_pack_map");
    return 0;
}

int ncn_field_pack_weights(const float* w_master, uint16_t* weights_packed, int precision, void* stream) {
    NCN_REQUIRE(precision == NCN_PREC_F16 || precision == NCN_PREC_BF16, hipErrorInvalidValue,
                "ncn_field_pack_weights: precision must be NCN_PREC_F16 or NCN_PREC_BF16");
    if (precision == NCN_PREC_F16)
        hipLaunchKernelGGL(pack_weights_kernel<_Float16>, dim3(N_FRAG32 + N_FRAG16), dim3(64), 0, (hipStream_t)stream,
                           w_master, (_Float16*)weights_packed);
    else
        hipLaunchKernelGGL(pack_weights_kernel<__bf16>, dim3(N_FRAG32 + N_FRAG16), dim3(64), 0, (hipStream_t)stream,
                           w_master, (__bf16*)weights_packed);
    NCN_LAUNCH_CHECK("ncn_field_pack_weights");
    return 0;
}

// `levels` is a HOST array of 16 x {scale f32 bits, resolution, params, offset}.
int ncn_field_sort_windows(const float* xyzs, int64_t n, const int32_t* n_dev, float xyz_min, float xyz_extent,
                           int32_t* order, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(xyz_extent > 0.f, hipErrorInvalidValue, "ncn_field_sort_windows: xyz_extent must be positive");
    hipLaunchKernelGGL(sort_windows_kernel, dim3((unsigned)cdiv(n, SORT_W)), dim3(SORT_THREADS), 0, (hipStream_t)stream,
                       xyzs, n, n_dev, xyz_min, 1.0f / xyz_extent, order);
    NCN_LAUNCH_CHECK("ncn_field_sort_windows");
    return 0;
}

int ncn_field_fwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                  const float* table,
                  const uint32_t* levels,
                  float xyz_min, float xyz_extent, const uint16_t* weights_packed, int precision, int mode,
                  float* sigmas, float* rgbs, uint16_t* enc_cache, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(mode >= 0 && mode <= 2, hipErrorInvalidValue, "ncn_field_fwd: mode must be 0, 1 or 2");
    NCN_REQUIRE(mode != 2 || (enc_cache && !order), hipErrorInvalidValue,
                "ncn_field_fwd: mode 2 needs enc_cache (scratch) and no processing order");
    NCN_REQUIRE(precision == NCN_PREC_F16 || precision == NCN_PREC_BF16, hipErrorInvalidValue,
                "ncn_field_fwd: precision must be NCN_PREC_F16 or NCN_PREC_BF16");
    NCN_REQUIRE(((uintptr_t)table & 7) == 0 && ((uintptr_t)enc_cache & 15) == 0 && ((uintptr_t)weights_packed & 15) == 0,
                hipErrorInvalidValue, "ncn_field_fwd: table 8-byte, enc_cache / weights_packed 16-byte aligned");
    const LevelTable Lt = make_table(levels);
    if (mode == 2) {  // level-split encoding over the XCDs first (n = capacity; n_dev = the count)
        NCN_REQUIRE(n <= (int64_t)INT32_MAX * 256 / 16, hipErrorInvalidValue, "ncn_field_fwd: n too large");
        const int nb = (int)((n + 255) / 256);
        if (precision == NCN_PREC_F16)
            hipLaunchKernelGGL(encode_xcd_kernel<_Float16>, dim3(16 * nb), dim3(256), 0, (hipStream_t)stream, xyzs, n,
                               n_dev, (const float2*)table, Lt, xyz_min, xyz_extent, nb, (_Float16*)enc_cache);
        else
            hipLaunchKernelGGL(encode_xcd_kernel<__bf16>, dim3(16 * nb), dim3(256), 0, (hipStream_t)stream, xyzs, n,
                               n_dev, (const float2*)table, Lt, xyz_min, xyz_extent, nb, (__bf16*)enc_cache);
        NCN_LAUNCH_CHECK("ncn_field_fwd (encode)");
    }
    if (precision == NCN_PREC_F16)
        hipLaunchKernelGGL((mode == 2 ? field_fwd_kernel<_Float16, true> : field_fwd_kernel<_Float16, false>),
                           dim3(fwd_grid(n)), dim3(256), 0, (hipStream_t)stream, xyzs, dirs,
                           n, n_dev, (const float2*)table, Lt, xyz_min, xyz_extent,
                           (const Mfma<_Float16>::v8*)weights_packed, mode, sigmas, rgbs,
                           (Mfma<_Float16>::v8*)enc_cache, order);
    else
        hipLaunchKernelGGL((mode == 2 ? field_fwd_kernel<__bf16, true> : field_fwd_kernel<__bf16, false>),
                           dim3(fwd_grid(n)), dim3(256), 0, (hipStream_t)stream, xyzs, dirs,
                           n, n_dev, (const float2*)table, Lt, xyz_min, xyz_extent,
                           (const Mfma<__bf16>::v8*)weights_packed, mode, sigmas, rgbs, (Mfma<__bf16>::v8*)enc_cache,
                           order);
    NCN_LAUNCH_CHECK("ncn_field_fwd");
    return 0;
}

int ncn_field_bwd_blocks(int64_t n) { return bwd_blocks_of(n); }

int64_t ncn_field_bwd_dE_floats(int64_t n) {
    if (n <= 0) return 0;
    const int64_t e_stride = (n + 3) & ~(int64_t)3;
    // header, the level-major encoding gradient, the scatter's permuted positions per class, then
    // the scatter's unit-queue words
    return de_queue_offset(e_stride) + SC_QUEUE_WORDS;
}

int ncn_field_bwd_mlp(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                      const uint16_t* weights_packed,
                      int precision, const uint16_t* enc_cache, const float* dL_dsigmas, const float* dL_drgbs,
                      const float* loss_scale, float* slab, float* dE_ws, float* level_max, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(precision == NCN_PREC_F16 || precision == NCN_PREC_BF16, hipErrorInvalidValue,
                "ncn_field_bwd_mlp: precision must be NCN_PREC_F16 or NCN_PREC_BF16");
    NCN_REQUIRE(((uintptr_t)dE_ws & 15) == 0 && ((uintptr_t)enc_cache & 15) == 0 && ((uintptr_t)weights_packed & 15) == 0,
                hipErrorInvalidValue, "ncn_field_bwd_mlp: dE_ws / enc_cache / weights_packed must be 16-byte aligned");
    NCN_REQUIRE(level_max != nullptr, hipErrorInvalidValue, "ncn_field_bwd_mlp: level_max workspace required");
    NCN_REQUIRE(((uintptr_t)xyzs & 15) == 0, hipErrorInvalidValue, "ncn_field_bwd_mlp: xyzs must be 16-byte aligned");
    launch_bwd_part<BWD_ALL>(precision, ncn_field_bwd_blocks(n), (hipStream_t)stream, xyzs, dirs, n, n_dev,
                             weights_packed, enc_cache, dL_dsigmas, dL_drgbs, loss_scale, dE_ws, slab, level_max, order,
                             nullptr, nullptr);
    NCN_LAUNCH_CHECK("ncn_field_bwd_mlp");
    return 0;
}

// per 16-sample group: 64 lanes x 4 operand values (2 B) + 16 fp32 row-0 elements = 144 floats
int64_t ncn_field_bwd_stash_floats(int64_t n) { return n > 0 ? 144 * ((n + 15) / 16) : 0; }

// the sigma pass fits two workgroups per CU (compact LDS): twice the one-pass grid, at most 512
int ncn_field_bwd_part_blocks(int64_t n, int part) {
    const int nb = ncn_field_bwd_blocks(n);
    return part == 2 ? std::min(512, 2 * nb) : nb;
}

int ncn_field_bwd_mlp_part(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                           const uint16_t* weights_packed, int precision, const uint16_t* enc_cache,
                           const float* dL_dsigmas, const float* dL_dsigmas2, const float* dL_drgbs,
                           const float* loss_scale, int part, int n_blocks, float* slab, float* dE_ws,
                           float* level_max, float* dh_stash, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(precision == NCN_PREC_F16 || precision == NCN_PREC_BF16, hipErrorInvalidValue,
                "ncn_field_bwd_mlp_part: precision must be NCN_PREC_F16 or NCN_PREC_BF16");
    NCN_REQUIRE(part == 1 || part == 2 || part == 3, hipErrorInvalidValue,
                "ncn_field_bwd_mlp_part: part must be 1 (rgb), 2 (sigma) or 3 (both)");
    NCN_REQUIRE(((uintptr_t)dE_ws & 15) == 0 && ((uintptr_t)enc_cache & 15) == 0 &&
                    ((uintptr_t)weights_packed & 15) == 0 && ((uintptr_t)dh_stash & 15) == 0,
                hipErrorInvalidValue, "ncn_field_bwd_mlp_part: dE_ws / enc_cache / weights_packed / dh_stash must be 16-byte aligned");
    NCN_REQUIRE(level_max != nullptr, hipErrorInvalidValue, "ncn_field_bwd_mlp_part: level_max workspace required");
    NCN_REQUIRE(part == 3 || dh_stash != nullptr, hipErrorInvalidValue, "ncn_field_bwd_mlp_part: dh_stash required for a split pass");
    const int nb = n_blocks > 0 ? std::min(n_blocks, ncn_field_bwd_part_blocks(n, part))
                                : ncn_field_bwd_part_blocks(n, part);
    const hipStream_t st = (hipStream_t)stream;
    if (part == 1)
        launch_bwd_part<1>(precision, nb, st, xyzs, dirs, n, n_dev, weights_packed, enc_cache, dL_dsigmas, dL_drgbs,
                           loss_scale, dE_ws, slab, level_max, order, dL_dsigmas2, dh_stash);
    else if (part == 2)
        launch_bwd_part<2>(precision, nb, st, xyzs, dirs, n, n_dev, weights_packed, enc_cache, dL_dsigmas, dL_drgbs,
                           loss_scale, dE_ws, slab, level_max, order, dL_dsigmas2, dh_stash);
    else
        launch_bwd_part<3>(precision, nb, st, xyzs, dirs, n, n_dev, weights_packed, enc_cache, dL_dsigmas, dL_drgbs,
                           loss_scale, dE_ws, slab, level_max, order, dL_dsigmas2, dh_stash);
    NCN_LAUNCH_CHECK("ncn_field_bwd_mlp_part");
    return 0;
}

int ncn_field_scatter_wgrad(const float* xyzs, int64_t n, const int32_t* n_dev, const int32_t* order,
                            const uint32_t* levels, float xyz_min, float xyz_extent, const float* dE_ws,
                            const float* level_max, int level_lo, int level_hi, int max_blocks, float* grad_table,
                            const float* slab, int n_blocks_sigma, int n_blocks_rgb, float* grad_w, void* stream) {
    if (n <= 0 || level_hi <= level_lo) return slab ? ncn_field_reduce_wgrad_parts(slab, n_blocks_sigma, n_blocks_rgb,
                                                                                   grad_w, stream) : 0;
    NCN_REQUIRE(0 <= level_lo && level_hi <= 16, hipErrorInvalidValue, "ncn_field_scatter: levels must lie in [0, 16)");
    NCN_REQUIRE(((uintptr_t)dE_ws & 15) == 0 && ((uintptr_t)xyzs & 15) == 0, hipErrorInvalidValue,
                "ncn_field_scatter: dE_ws and xyzs must be 16-byte aligned");
    NCN_REQUIRE(!slab || grad_w, hipErrorInvalidValue, "ncn_field_scatter_wgrad: grad_w required with a slab");
    const LevelTable Lt = make_table(levels);
    int grid = scatter_grid(n);
    if (max_blocks > 0) grid = std::min(grid, max_blocks * (1024 / SC_THREADS));  // (max_blocks: CUs)
    hipLaunchKernelGGL(field_scatter_kernel, dim3(grid), dim3(SC_THREADS), 0, (hipStream_t)stream, xyzs, n, n_dev, Lt,
                       xyz_min, xyz_extent, dE_ws, grad_table, level_max, ncn_field_bwd_blocks(n),
                       level_lo, level_hi, order, slab, n_blocks_sigma, n_blocks_rgb, grad_w,
                       (unsigned*)const_cast<float*>(dE_ws + de_queue_offset((n + 3) & ~(int64_t)3)) + 2 * level_lo);
    NCN_LAUNCH_CHECK("ncn_field_scatter");
    return 0;
}

int ncn_field_scatter_positions(const float* xyzs, int64_t n, const int32_t* n_dev, float* dE_ws, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(((uintptr_t)dE_ws & 15) == 0 && ((uintptr_t)xyzs & 15) == 0, hipErrorInvalidValue,
                "ncn_field_scatter_positions: dE_ws and xyzs must be 16-byte aligned");
    const int64_t e_stride = (n + 3) & ~(int64_t)3;
    const int pgrid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, cdiv(cdiv(n, 4), 256)));
    hipLaunchKernelGGL(sc_perm_positions_kernel, dim3(pgrid), dim3(256), 0, (hipStream_t)stream, xyzs, n, n_dev,
                       (1 << SC_N_CLASSES) - 1, dE_ws + DE_HEADER_FLOATS + 16 * e_stride, dE_ws + DE_POS_FLAG,
                       (float)((1 << SC_N_CLASSES) - 1));
    NCN_LAUNCH_CHECK("ncn_field_scatter_positions");
    return 0;
}

int ncn_field_scatter(const float* xyzs, int64_t n, const int32_t* n_dev, const int32_t* order,
                      const uint32_t* levels, float xyz_min,
                      float xyz_extent, const float* dE_ws, const float* level_max, int level_lo, int level_hi,
                      int max_blocks, float* grad_table, void* stream) {
    return ncn_field_scatter_wgrad(xyzs, n, n_dev, order, levels, xyz_min, xyz_extent, dE_ws, level_max, level_lo,
                                   level_hi, max_blocks, grad_table, nullptr, 0, 0, nullptr, stream);
}

int ncn_field_bwd(const float* xyzs, const float* dirs, int64_t n, const int32_t* n_dev, const int32_t* order,
                  const uint32_t* levels,
                  float xyz_min, float xyz_extent, const uint16_t* weights_packed, int precision,
                  const uint16_t* enc_cache, const float* dL_dsigmas, const float* dL_drgbs, const float* loss_scale,
                  float* grad_table, float* slab, float* dE_ws, float* level_max, void* stream) {
    if (n <= 0) return 0;
    const int e = ncn_field_bwd_mlp(xyzs, dirs, n, n_dev, order, weights_packed, precision, enc_cache, dL_dsigmas, dL_drgbs,
                                    loss_scale, slab, dE_ws, level_max, stream);
    if (e) return e;
    return ncn_field_scatter(xyzs, n, n_dev, order, levels, xyz_min, xyz_extent, dE_ws, level_max, 0, 16, 0,
                             grad_table, stream);
}


#ifdef NCN_DIAG_SC_TIMES
int ncn_diag_sc_times(unsigned long long* host, int reset) {
    if (reset) {
        static unsigned long long zero[256][10];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(ncn_sc_times), zero, sizeof(zero));
    }
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ncn_sc_times), 256 * 10 * sizeof(unsigned long long));
}
#endif

#ifdef NCN_DIAG_SC_SPAN
int ncn_diag_sc_span(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ncn_sc_span), 256 * 20 * sizeof(unsigned long long));
}
#endif

int ncn_field_reduce_wgrad(const float* slab, int n_blocks, float* grad_w, void* stream) {
    if (n_blocks <= 0) return 0;
    hipLaunchKernelGGL(reduce_wgrad_kernel, dim3(cdiv(NCN_FIELD_NW, 256), cdiv(n_blocks, WRED_CHUNK)), dim3(256), 0,
                       (hipStream_t)stream, slab, n_blocks, n_blocks, grad_w);
    NCN_LAUNCH_CHECK("ncn_field_reduce_wgrad");
    return 0;
}

int ncn_field_reduce_wgrad_parts(const float* slab, int n_blocks_sigma, int n_blocks_rgb, float* grad_w,
                                 void* stream) {
    const int nb = std::max(n_blocks_sigma, n_blocks_rgb);
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(reduce_wgrad_kernel, dim3(cdiv(NCN_FIELD_NW, 256), cdiv(nb, WRED_CHUNK)), dim3(256), 0,
                       (hipStream_t)stream, slab, n_blocks_sigma, n_blocks_rgb, grad_w);
    NCN_LAUNCH_CHECK("ncn_field_reduce_wgrad_parts");
    return 0;
}

}  // extern "C"
