// Diagnostic lab (not product code): the product composite forward (csrc/vren.hip) with switches
// that remove one piece of its dependency chain at a time, to attribute the kernel's time.
// F_NOWS: no ws stores; F_ONEROUND: stop after the first round of ROWS rows (wrong for long rays);
// F_FAKESEG: segment = (n * 70, 70) without waiting for rays_a (wrong, timing only).
#include "../normal-clustering-nerf_amd/csrc/common.h"

using namespace ncn;

namespace lab2 {
constexpr int C = 3;
// ---- multi-row DPP inclusive product scans (interleaved: no s_nop inside for K >= 4) ----
#define NCN_DPPM(R, CTRL) "v_mul_f32_dpp %" #R ", %" #R ", %" #R " " CTRL "\n\t"
#define NCN_S1 "row_shr:1 row_mask:0xf bank_mask:0xf"
#define NCN_S2 "row_shr:2 row_mask:0xf bank_mask:0xf"
#define NCN_S4 "row_shr:4 row_mask:0xf bank_mask:0xf"
#define NCN_S8 "row_shr:8 row_mask:0xf bank_mask:0xf"
#define NCN_S15 "row_bcast:15 row_mask:0xa bank_mask:0xf"
#define NCN_S31 "row_bcast:31 row_mask:0xc bank_mask:0xf"
#define NCN_STEP2(C) NCN_DPPM(0, C) NCN_DPPM(1, C) "s_nop 0\n\t"
#define NCN_STEP4(C) NCN_DPPM(0, C) NCN_DPPM(1, C) NCN_DPPM(2, C) NCN_DPPM(3, C)
#define NCN_STEP8(C) NCN_STEP4(C) NCN_DPPM(4, C) NCN_DPPM(5, C) NCN_DPPM(6, C) NCN_DPPM(7, C)
template <int K>
__device__ __forceinline__ void wave_incl_prod_multi(float (&v)[K]) {
    if constexpr (K == 1) {
        v[0] = wave_incl_prod_dpp_fused(v[0]);
    } else if constexpr (K == 2) {
        asm volatile("s_nop 1\n\t" NCN_STEP2(NCN_S1) NCN_STEP2(NCN_S2) NCN_STEP2(NCN_S4) NCN_STEP2(NCN_S8)
                         NCN_STEP2(NCN_S15) NCN_STEP2(NCN_S31) "s_nop 1"
                     : "+v"(v[0]), "+v"(v[1]));
    } else if constexpr (K == 4) {
        asm volatile("s_nop 1\n\t" NCN_STEP4(NCN_S1) NCN_STEP4(NCN_S2) NCN_STEP4(NCN_S4) NCN_STEP4(NCN_S8)
                         NCN_STEP4(NCN_S15) NCN_STEP4(NCN_S31) "s_nop 1"
                     : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
    } else {
        static_assert(K == 8, "K in {1,2,4,8}");
        asm volatile("s_nop 1\n\t" NCN_STEP8(NCN_S1) NCN_STEP8(NCN_S2) NCN_STEP8(NCN_S4) NCN_STEP8(NCN_S8)
                         NCN_STEP8(NCN_S15) NCN_STEP8(NCN_S31) "s_nop 1"
                     : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                       "+v"(v[7]));
    }
}
enum { F_NOWS = 1, F_ONEROUND = 2, F_FAKESEG = 4 };

template <int ROWS, int F>
__global__ __launch_bounds__(256) void cfw(const float* __restrict__ sigmas, const float* __restrict__ raws,
                                           const float* __restrict__ deltas, const float* __restrict__ ts,
                                           const int64_t* __restrict__ rays_a, int64_t R, float T_thr,
                                           int64_t* __restrict__ total_samples, float* __restrict__ opacity,
                                           float* __restrict__ depth, float* __restrict__ rend,
                                           float* __restrict__ ws, int64_t S) {
    const int lane = threadIdx.x & 63;
    const int64_t n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int64_t n = n0 < R ? n0 : R - 1;
    int64_t ray, start;
    int N;
    if (F & F_FAKESEG) {
        ray = n;
        start = n * 70 < S - 70 ? n * 70 : S - 70;
        N = 70;
    } else {
        ray = rays_a[3 * n];
        start = rays_a[3 * n + 1];
        N = (int)rays_a[3 * n + 2];
    }
    const uint32_t nb = (uint32_t)N * 4u;
    const auto r_s = buf_rsrc(sigmas + start, nb), r_d = buf_rsrc(deltas + start, nb);
    const auto r_t = buf_rsrc(ts + start, nb), r_r = buf_rsrc(raws + start * C, nb * C);
    const auto r_w = buf_rsrc(ws + start, nb);
    float Tc = 1.0f;
    float acc[2 + C];
#pragma unroll
    for (int i = 0; i < 2 + C; i++) acc[i] = 0.f;
    int total = N;
    for (int base = 0; base == 0 || base < N; base += 64 * ROWS) {
        float sg[ROWS], dl[ROWS], tt[ROWS], rr[ROWS][C];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint32_t k = (uint32_t)(base + r * 64 + lane);
            if (r == 0 || base + r * 64 < N) {
                sg[r] = buf_load(r_s, k * 4u);
                dl[r] = buf_load(r_d, k * 4u);
                tt[r] = buf_load(r_t, k * 4u);
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = buf_load(r_r, k * (4u * C) + 4u * i);
            } else {
                sg[r] = dl[r] = tt[r] = 0.f;
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = 0.f;
            }
        }
        bool stopped = false;
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int kb = base + r * 64;
            if (kb >= N) break;
            const float a = 1.0f - __expf(-sg[r] * dl[r]);
            const float om = 1.0f - a;
            const float Tb = Tc * wave_shr1_dpp(wave_incl_prod_dpp_fused(om), 1.0f);
            const float Ta = Tb * om;
            const uint64_t stopm = __ballot(Ta <= T_thr);
            const int stop_lane = stopm ? __builtin_ctzll(stopm) : 64;
            const float w = lane <= stop_lane ? a * Tb : 0.f;
            if (!(F & F_NOWS)) buf_store(r_w, (uint32_t)(kb + lane) * 4u, w);
            acc[0] += w;
            acc[1] = fmaf(w, tt[r], acc[1]);
#pragma unroll
            for (int i = 0; i < C; i++) acc[2 + i] = fmaf(w, rr[r][i], acc[2 + i]);
            if (stopm) {
                total = kb + stop_lane;
                if (!(F & F_NOWS))
                    for (int k = kb + 64 + lane; k < N; k += 64) buf_store(r_w, (uint32_t)k * 4u, 0.f);
                stopped = true;
                break;
            }
            Tc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Ta), 63));
        }
        if (stopped || (F & F_ONEROUND)) break;
    }
    wave_sum_multi<2 + C>(acc);
    if (n0 < R && lane == 0) {
        opacity[ray] = acc[0];
        depth[ray] = acc[1];
#pragma unroll
        for (int i = 0; i < C; i++) rend[ray * C + i] = acc[2 + i];
        total_samples[ray] = total;
    }
}

// Block structure: the ray's rows are taken in one block of 1/2/4 rows (by N) or in blocks of 8;
// sigma/delta of every row of the block are loaded up front (the transmittance needs only them),
// t/raw of rows 0-3 too; t/raw of rows 4-7 are loaded after rows 0-3 are accumulated.
// All rows' product scans are interleaved (one asm), then the carries chain through readlane.
template <int ROWS, bool GUARD>
__device__ __forceinline__ bool blk(const __amdgpu_buffer_rsrc_t& r_s, const __amdgpu_buffer_rsrc_t& r_d,
                                    const __amdgpu_buffer_rsrc_t& r_t, const __amdgpu_buffer_rsrc_t& r_r,
                                    const __amdgpu_buffer_rsrc_t& r_w, int base, int N, float T_thr, int lane,
                                    float& Tc, float (&acc)[5], int& total) {
    constexpr int RT = ROWS < 4 ? ROWS : 4;
    float sg[ROWS], dl[ROWS], tt[RT], rr[RT][C];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const uint32_t k = (uint32_t)(base + r * 64 + lane);
        if (!GUARD || r == 0 || base + r * 64 < N) {
            sg[r] = buf_load(r_s, k * 4u);
            dl[r] = buf_load(r_d, k * 4u);
            if (r < RT) {
                tt[r] = buf_load(r_t, k * 4u);
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = buf_load(r_r, k * (4u * C) + 4u * i);
            }
        } else {
            sg[r] = dl[r] = 0.f;
            if (r < RT) {
                tt[r] = 0.f;
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = 0.f;
            }
        }
    }
    float a[ROWS], p[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        a[r] = 1.0f - __expf(-sg[r] * dl[r]);
        p[r] = 1.0f - a[r];
    }
    float om[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) om[r] = p[r];
    wave_incl_prod_multi<ROWS>(p);
    float Tb[ROWS];
    uint64_t m[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        Tb[r] = Tc * wave_shr1_dpp(p[r], 1.0f);
        const float Ta = Tb[r] * om[r];
        m[r] = __ballot(Ta <= T_thr);
        Tc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Ta), 63));
    }
    int srow = ROWS, slane = 64;
#pragma unroll
    for (int r = ROWS - 1; r >= 0; r--)
        if (m[r]) { srow = r; slane = __builtin_ctzll(m[r]); }
    float w[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const bool inc = r < srow || (r == srow && lane <= slane);
        w[r] = inc ? a[r] * Tb[r] : 0.f;
        if (!GUARD || r == 0 || base + r * 64 < N) buf_store(r_w, (uint32_t)(base + r * 64 + lane) * 4u, w[r]);
    }
#pragma unroll
    for (int r = 0; r < RT; r++) {
        acc[0] += w[r];
        acc[1] = fmaf(w[r], tt[r], acc[1]);
#pragma unroll
        for (int i = 0; i < C; i++) acc[2 + i] = fmaf(w[r], rr[r][i], acc[2 + i]);
    }
    if constexpr (ROWS > 4) {
        if (base + 4 * 64 < N && srow > 4 - 1) {
            float t2[4], r2[4][C];
#pragma unroll
            for (int r = 4; r < ROWS; r++) {
                const uint32_t k = (uint32_t)(base + r * 64 + lane);
                if (base + r * 64 < N) {
                    t2[r - 4] = buf_load(r_t, k * 4u);
#pragma unroll
                    for (int i = 0; i < C; i++) r2[r - 4][i] = buf_load(r_r, k * (4u * C) + 4u * i);
                } else {
                    t2[r - 4] = 0.f;
#pragma unroll
                    for (int i = 0; i < C; i++) r2[r - 4][i] = 0.f;
                }
            }
#pragma unroll
            for (int r = 4; r < ROWS; r++) {
                acc[0] += w[r];
                acc[1] = fmaf(w[r], t2[r - 4], acc[1]);
#pragma unroll
                for (int i = 0; i < C; i++) acc[2 + i] = fmaf(w[r], r2[r - 4][i], acc[2 + i]);
            }
        }
    }
    if (srow < ROWS) {
        total = base + srow * 64 + slane;
        for (int k = base + ROWS * 64 + lane; k < N; k += 64) buf_store(r_w, (uint32_t)k * 4u, 0.f);
        return true;
    }
    return false;
}

__global__ __launch_bounds__(256) void cfw_blk(const float* __restrict__ sigmas, const float* __restrict__ raws,
                                               const float* __restrict__ deltas, const float* __restrict__ ts,
                                               const int64_t* __restrict__ rays_a, int64_t R, float T_thr,
                                               int64_t* __restrict__ total_samples, float* __restrict__ opacity,
                                               float* __restrict__ depth, float* __restrict__ rend,
                                               float* __restrict__ ws, int64_t S) {
    const int lane = threadIdx.x & 63;
    const int64_t n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int64_t n = n0 < R ? n0 : R - 1;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    const uint32_t nb = (uint32_t)N * 4u;
    const auto r_s = buf_rsrc(sigmas + start, nb), r_d = buf_rsrc(deltas + start, nb);
    const auto r_t = buf_rsrc(ts + start, nb), r_r = buf_rsrc(raws + start * C, nb * C);
    const auto r_w = buf_rsrc(ws + start, nb);
    float Tc = 1.0f;
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    int total = N;
    if (N <= 64) {
        blk<1, false>(r_s, r_d, r_t, r_r, r_w, 0, N, T_thr, lane, Tc, acc, total);
    } else if (N <= 128) {
        blk<2, false>(r_s, r_d, r_t, r_r, r_w, 0, N, T_thr, lane, Tc, acc, total);
    } else if (N <= 256) {
        blk<4, false>(r_s, r_d, r_t, r_r, r_w, 0, N, T_thr, lane, Tc, acc, total);
    } else {
        for (int base = 0; base < N; base += 512)
            if (blk<8, true>(r_s, r_d, r_t, r_r, r_w, base, N, T_thr, lane, Tc, acc, total)) break;
    }
    wave_sum_multi<5>(acc);
    if (n0 < R && lane == 0) {
        opacity[ray] = acc[0];
        depth[ray] = acc[1];
#pragma unroll
        for (int i = 0; i < C; i++) rend[ray * C + i] = acc[2 + i];
        total_samples[ray] = total;
    }
}
}  // namespace lab2

extern "C" int lab2_cfw(int variant, const float* sigmas, const float* raws, const float* deltas, const float* ts,
                        const int64_t* rays_a, int64_t R, int64_t S, float T_thr, int64_t* total, float* opacity,
                        float* depth, float* rend, float* ws, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((unsigned)cdiv(R, 4)), b(256);
#define ARGS sigmas, raws, deltas, ts, rays_a, R, T_thr, total, opacity, depth, rend, ws, S
    switch (variant) {
        case 0: hipLaunchKernelGGL((lab2::cfw<4, 0>), g, b, 0, s, ARGS); break;
        case 1: hipLaunchKernelGGL((lab2::cfw<4, lab2::F_NOWS>), g, b, 0, s, ARGS); break;
        case 2: hipLaunchKernelGGL((lab2::cfw<4, lab2::F_ONEROUND>), g, b, 0, s, ARGS); break;
        case 3: hipLaunchKernelGGL((lab2::cfw<4, lab2::F_FAKESEG>), g, b, 0, s, ARGS); break;
        case 4: hipLaunchKernelGGL((lab2::cfw<8, 0>), g, b, 0, s, ARGS); break;
        case 5: hipLaunchKernelGGL((lab2::cfw<2, 0>), g, b, 0, s, ARGS); break;
        case 6: hipLaunchKernelGGL((lab2::cfw<4, lab2::F_NOWS | lab2::F_ONEROUND>), g, b, 0, s, ARGS); break;
        case 7: hipLaunchKernelGGL((lab2::cfw<4, lab2::F_NOWS | lab2::F_FAKESEG>), g, b, 0, s, ARGS); break;
        case 8: hipLaunchKernelGGL((lab2::cfw<1, lab2::F_NOWS | lab2::F_FAKESEG | lab2::F_ONEROUND>), g, b, 0, s, ARGS); break;
        case 9: hipLaunchKernelGGL((lab2::cfw<8, lab2::F_NOWS>), g, b, 0, s, ARGS); break;
        case 10: hipLaunchKernelGGL(lab2::cfw_blk, g, b, 0, s, ARGS); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef ARGS
    return (int)hipGetLastError();
}
