// Diagnostic lab (not product code): variants of the train composite forward on the same inputs,
// timed by tools/composite_lab.py.  Every variant has the signature of ncn_composite_train_fw
// plus a variant id; the product kernel lives in normal-clustering-nerf_amd/csrc/vren.hip.
#include "../normal-clustering-nerf_amd/csrc/common.h"

using namespace ncn;

namespace lab {

constexpr int C = 3;

struct RayOut {
    float o, d, r[C];
    int total;
};

// One ray by one wave, rows of 64 samples, ROWS rows per round (the product's v2 body).
template <int ROWS, int MODE>
__device__ __forceinline__ void ray_body(const float* __restrict__ sigmas, const float* __restrict__ raws,
                                         const float* __restrict__ deltas, const float* __restrict__ ts,
                                         int64_t start, int N, float T_thr, float* __restrict__ ws, int lane,
                                         RayOut& out) {
    float Tc = 1.0f, acc_o = 0.f, acc_d = 0.f, acc_r[C] = {0.f, 0.f, 0.f};
    int total = N;
    bool done = false;
    for (int base = 0; base < N; base += 64 * ROWS) {
        float sg[ROWS], dl[ROWS], tt[ROWS], rr[ROWS][C];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int k = base + r * 64 + lane;
            const int64_t s = start + k;
            const bool v = k < N && !done;
            sg[r] = v ? sigmas[s] : 0.f;
            dl[r] = v ? deltas[s] : 0.f;
            tt[r] = v ? ts[s] : 0.f;
#pragma unroll
            for (int i = 0; i < C; i++) rr[r][i] = v ? raws[s * C + i] : 0.f;
        }
        if (MODE == 2) {  // loads only
            float t = 0.f;
#pragma unroll
            for (int r = 0; r < ROWS; r++) t += sg[r] + dl[r] + tt[r] + rr[r][0] + rr[r][1] + rr[r][2];
            acc_o += t;
            continue;
        }
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int k = base + r * 64 + lane;
            if (base + r * 64 >= N) break;
            const bool valid = k < N;
            if (done) {
                if (valid) ws[start + k] = 0.f;
                continue;
            }
            const float a = 1.0f - __expf(-sg[r] * dl[r]);
            const float om = 1.0f - a;
            const float incl = wave_incl_prod_dpp(valid ? om : 1.0f);
            const float Tb = Tc * wave_shr1_dpp(incl, 1.0f);
            const float Ta = Tb * om;
            const uint64_t stopm = __ballot(valid && Ta <= T_thr);
            const int stop_lane = stopm ? __builtin_ctzll(stopm) : 64;
            const bool inc = valid && lane <= stop_lane;
            const float w = inc ? a * Tb : 0.f;
            if (valid) ws[start + k] = w;
#pragma unroll
            for (int i = 0; i < C; i++) acc_r[i] = fmaf(w, rr[r][i], acc_r[i]);
            acc_d = fmaf(w, tt[r], acc_d);
            acc_o += w;
            if (stopm) {
                done = true;
                total = base + r * 64 + stop_lane;
            }
            Tc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Ta), 63));
        }
    }
    out.o = wave_sum_dpp(acc_o);
    out.d = wave_sum_dpp(acc_d);
#pragma unroll
    for (int i = 0; i < C; i++) out.r[i] = wave_sum_dpp(acc_r[i]);
    out.total = total;
}

__device__ __forceinline__ void store_ray(const RayOut& o, int64_t ray, int lane, int64_t* total_samples,
                                          float* opacity, float* depth, float* rend) {
    if (lane == 0) {
        opacity[ray] = o.o;
        depth[ray] = o.d;
#pragma unroll
        for (int i = 0; i < C; i++) rend[ray * C + i] = o.r[i];
        total_samples[ray] = o.total;
    }
}

// MODE 0: full; 1: per-ray loads + stores only; 2: sample loads, no compute/ws.  WPB waves/block.
template <int WPB, int ROWS, int MODE>
__global__ __launch_bounds__(64 * WPB) void wave_per_ray(const float* __restrict__ sigmas,
                                                         const float* __restrict__ raws,
                                                         const float* __restrict__ deltas,
                                                         const float* __restrict__ ts,
                                                         const int64_t* __restrict__ rays_a, int64_t R, float T_thr,
                                                         int64_t* __restrict__ total_samples,
                                                         float* __restrict__ opacity, float* __restrict__ depth,
                                                         float* __restrict__ rend, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t n = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * WPB + (threadIdx.x >> 6)));
    if (n >= R) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    RayOut o;
    if (MODE == 1) {
        o.o = (float)N; o.d = 0.f; o.r[0] = o.r[1] = o.r[2] = 0.f; o.total = N;
    } else {
        ray_body<ROWS, MODE>(sigmas, raws, deltas, ts, start, N, T_thr, ws, lane, o);
    }
    store_ray(o, ray, lane, total_samples, opacity, depth, rend);
}

// Grid-stride: each wave takes rays n, n + W, ... (W = waves in the grid); the next ray's triple
// is fetched before the current ray is composited.
template <int ROWS>
__global__ __launch_bounds__(256) void wave_multi_ray(const float* __restrict__ sigmas,
                                                      const float* __restrict__ raws,
                                                      const float* __restrict__ deltas,
                                                      const float* __restrict__ ts,
                                                      const int64_t* __restrict__ rays_a, int64_t R, float T_thr,
                                                      int64_t* __restrict__ total_samples,
                                                      float* __restrict__ opacity, float* __restrict__ depth,
                                                      float* __restrict__ rend, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t W = (int64_t)gridDim.x * 4;
    int64_t n = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (n >= R) return;
    int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    int N = (int)rays_a[3 * n + 2];
    while (true) {
        const int64_t nn = n + W;
        int64_t ray2 = 0, start2 = 0;
        int N2 = 0;
        if (nn < R) { ray2 = rays_a[3 * nn]; start2 = rays_a[3 * nn + 1]; N2 = (int)rays_a[3 * nn + 2]; }
        RayOut o;
        ray_body<ROWS, 0>(sigmas, raws, deltas, ts, start, N, T_thr, ws, lane, o);
        store_ray(o, ray, lane, total_samples, opacity, depth, rend);
        if (nn >= R) break;
        n = nn; ray = ray2; start = start2; N = N2;
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

// Per-ray buffer descriptors sized to the ray's segment: loads past N return 0 and stores past N
// are dropped by the hardware bounds check, so the row bodies carry no masks or branches.
template <int WPB, int ROWS, int KA = 0>
__global__ __launch_bounds__(64 * WPB) void wave_per_ray_buf(const float* __restrict__ sigmas,
                                                             const float* __restrict__ raws,
                                                             const float* __restrict__ deltas,
                                                             const float* __restrict__ ts,
                                                             const int64_t* __restrict__ rays_a, int64_t R,
                                                             float T_thr, int64_t* __restrict__ total_samples,
                                                             float* __restrict__ opacity, float* __restrict__ depth,
                                                             float* __restrict__ rend, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * WPB + (threadIdx.x >> 6)));
    const int64_t n = KA ? (n0 < R ? n0 : R - 1) : n0;
    if (!KA && n >= R) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    if (KA && n0 >= R) return;
    const uint32_t nb = (uint32_t)N * 4u;
    const auto r_s = rsrc(sigmas + start, nb), r_d = rsrc(deltas + start, nb), r_t = rsrc(ts + start, nb);
    const auto r_r = rsrc(raws + start * C, nb * C), r_w = rsrc(ws + start, nb);
    float Tc = 1.0f, acc_o = 0.f, acc_d = 0.f, acc_r[C] = {0.f, 0.f, 0.f};
    int total = N;
    for (int base = 0; base < N; base += 64 * ROWS) {
        float sg[ROWS], dl[ROWS], tt[ROWS], rr[ROWS][C];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint32_t k = (uint32_t)(base + r * 64 + lane);
            if (r == 0 || base + r * 64 < N) {
                sg[r] = bload(r_s, k * 4u);
                dl[r] = bload(r_d, k * 4u);
                tt[r] = bload(r_t, k * 4u);
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = bload(r_r, k * (4u * C) + 4u * i);
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
            const float incl = wave_incl_prod_dpp(om);
            const float Tb = Tc * wave_shr1_dpp(incl, 1.0f);
            const float Ta = Tb * om;
            const uint64_t stopm = __ballot(Ta <= T_thr);
            const int stop_lane = stopm ? __builtin_ctzll(stopm) : 64;
            const float w = lane <= stop_lane ? a * Tb : 0.f;
            bstore(r_w, (uint32_t)(kb + lane) * 4u, w);
#pragma unroll
            for (int i = 0; i < C; i++) acc_r[i] = fmaf(w, rr[r][i], acc_r[i]);
            acc_d = fmaf(w, tt[r], acc_d);
            acc_o += w;
            if (stopm) {
                total = kb + stop_lane;
                for (int k = kb + 64 + lane; k < N; k += 64) bstore(r_w, (uint32_t)k * 4u, 0.f);
                stopped = true;
                break;
            }
            Tc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Ta), 63));
        }
        if (stopped) break;
    }
    RayOut o;
    o.o = wave_sum_dpp(acc_o);
    o.d = wave_sum_dpp(acc_d);
#pragma unroll
    for (int i = 0; i < C; i++) o.r[i] = wave_sum_dpp(acc_r[i]);
    o.total = total;
    store_ray(o, ray, lane, total_samples, opacity, depth, rend);
}

// Inclusive product scan over the wave: v_mul_f32_dpp with the destination as both sources and no
// bound_ctrl, so a lane without a DPP source is simply not written (keeps its value = times 1).
__device__ __forceinline__ float wave_incl_prod_asm(float v) {
    asm volatile(
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_mul_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(v));
    return v;
}

__device__ __forceinline__ float f_swap32_sum(float a, float b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float f_swap16_sum(float a, float b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// every lane of a 16-lane row gets the row total (row_ror 8, 4, 2, 1)
__device__ __forceinline__ float row_total(float v) {
    v = dpp_add<0x128>(v);
    v = dpp_add<0x124>(v);
    v = dpp_add<0x122>(v);
    v = dpp_add<0x121>(v);
    return v;
}
// Five wave totals at once: two permlane32 swaps + one self swap halve the lanes, one permlane16
// swap + one self swap halve again, then 16-lane row totals on two registers.
__device__ __forceinline__ void wave_sum5(float& o, float& d, float& r0, float& r1, float& r2) {
    const float P = f_swap32_sum(o, d);     // lanes 0-31: o, 32-63: d
    const float Q = f_swap32_sum(r0, r1);   // lanes 0-31: r0, 32-63: r1
    const float Rr = f_swap32_sum(r2, r2);  // both halves: r2
    const float PQ = row_total(f_swap16_sum(P, Q));  // rows: o, r0, d, r1
    const float RR = row_total(f_swap16_sum(Rr, Rr));
    o = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(PQ), 0));
    r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(PQ), 16));
    d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(PQ), 32));
    r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(PQ), 48));
    r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(RR), 0));  // self swaps: every row = total
}

// v9 + asm product scan (SCAN=1) and/or the five-at-once reduction (RED=1); MODE 2 = loads only
template <int WPB, int ROWS, int SCAN, int RED, int MODE, int KA = 0>
__global__ __launch_bounds__(64 * WPB) void wave_per_ray_buf2(const float* __restrict__ sigmas,
                                                              const float* __restrict__ raws,
                                                              const float* __restrict__ deltas,
                                                              const float* __restrict__ ts,
                                                              const int64_t* __restrict__ rays_a, int64_t R,
                                                              float T_thr, int64_t* __restrict__ total_samples,
                                                              float* __restrict__ opacity, float* __restrict__ depth,
                                                              float* __restrict__ rend, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * WPB + (threadIdx.x >> 6)));
    const int64_t n = KA ? (n0 < R ? n0 : R - 1) : n0;
    if (!KA && n >= R) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    const bool live = !KA || n0 < R;
    const uint32_t nb = (uint32_t)N * 4u;
    const auto r_s = rsrc(sigmas + start, nb), r_d = rsrc(deltas + start, nb), r_t = rsrc(ts + start, nb);
    const auto r_r = rsrc(raws + start * C, nb * C), r_w = rsrc(ws + start, nb);
    float Tc = 1.0f, acc_o = 0.f, acc_d = 0.f, acc_r[C] = {0.f, 0.f, 0.f};
    int total = N;
    for (int base = 0; base == 0 || base < N; base += 64 * ROWS) {
        float sg[ROWS], dl[ROWS], tt[ROWS], rr[ROWS][C];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint32_t k = (uint32_t)(base + r * 64 + lane);
            if (r == 0 || base + r * 64 < N) {
                sg[r] = bload(r_s, k * 4u);
                dl[r] = bload(r_d, k * 4u);
                tt[r] = bload(r_t, k * 4u);
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = bload(r_r, k * (4u * C) + 4u * i);
            } else {
                sg[r] = dl[r] = tt[r] = 0.f;
#pragma unroll
                for (int i = 0; i < C; i++) rr[r][i] = 0.f;
            }
        }
        if (MODE == 2) {
#pragma unroll
            for (int r = 0; r < ROWS; r++) {
                acc_o += sg[r] * dl[r];
                acc_d += tt[r];
#pragma unroll
                for (int i = 0; i < C; i++) acc_r[i] += rr[r][i];
            }
            continue;
        }
        bool stopped = false;
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int kb = base + r * 64;
            if (kb >= N) break;
            const float a = 1.0f - __expf(-sg[r] * dl[r]);
            const float om = 1.0f - a;
            const float incl = SCAN ? wave_incl_prod_asm(om) : wave_incl_prod_dpp(om);
            const float Tb = Tc * wave_shr1_dpp(incl, 1.0f);
            const float Ta = Tb * om;
            const uint64_t stopm = __ballot(Ta <= T_thr);
            const int stop_lane = stopm ? __builtin_ctzll(stopm) : 64;
            const float w = lane <= stop_lane ? a * Tb : 0.f;
            bstore(r_w, (uint32_t)(kb + lane) * 4u, w);
#pragma unroll
            for (int i = 0; i < C; i++) acc_r[i] = fmaf(w, rr[r][i], acc_r[i]);
            acc_d = fmaf(w, tt[r], acc_d);
            acc_o += w;
            if (stopm) {
                total = kb + stop_lane;
                for (int k = kb + 64 + lane; k < N; k += 64) bstore(r_w, (uint32_t)k * 4u, 0.f);
                stopped = true;
                break;
            }
            Tc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Ta), 63));
        }
        if (stopped) break;
    }
    RayOut o;
    if (RED) {
        wave_sum5(acc_o, acc_d, acc_r[0], acc_r[1], acc_r[2]);
        o.o = acc_o; o.d = acc_d; o.r[0] = acc_r[0]; o.r[1] = acc_r[1]; o.r[2] = acc_r[2];
    } else {
        o.o = wave_sum_dpp(acc_o);
        o.d = wave_sum_dpp(acc_d);
#pragma unroll
        for (int i = 0; i < C; i++) o.r[i] = wave_sum_dpp(acc_r[i]);
    }
    o.total = total;
    if (live) store_ray(o, ray, lane, total_samples, opacity, depth, rend);
}

__global__ void empty_kernel(float* p) {
    if (p && threadIdx.x == 1234) p[0] = 1.f;
}

}  // namespace lab

extern "C" int lab_composite_fw(int variant, const float* sigmas, const float* raws, const float* deltas,
                                const float* ts, const int64_t* rays_a, int64_t R, float T_thr, int64_t* total,
                                float* opacity, float* depth, float* rend, float* ws, void* stream) {
    hipStream_t s = (hipStream_t)stream;
#define ARGS sigmas, raws, deltas, ts, rays_a, R, T_thr, total, opacity, depth, rend, ws
    switch (variant) {
        case 0: hipLaunchKernelGGL((lab::wave_per_ray<4, 4, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 1: hipLaunchKernelGGL((lab::wave_per_ray<16, 4, 0>), dim3(cdiv(R, 16)), dim3(1024), 0, s, ARGS); break;
        case 2: hipLaunchKernelGGL((lab::wave_per_ray<1, 4, 0>), dim3(R), dim3(64), 0, s, ARGS); break;
        case 3: hipLaunchKernelGGL((lab::wave_per_ray<4, 2, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 4: hipLaunchKernelGGL((lab::wave_per_ray<4, 4, 1>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 5: hipLaunchKernelGGL((lab::wave_per_ray<4, 4, 2>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 6: hipLaunchKernelGGL((lab::wave_multi_ray<2>), dim3(cdiv(R, 8)), dim3(256), 0, s, ARGS); break;
        case 7: hipLaunchKernelGGL((lab::wave_multi_ray<2>), dim3(cdiv(R, 16)), dim3(256), 0, s, ARGS); break;
        case 8: hipLaunchKernelGGL((lab::wave_per_ray<8, 4, 0>), dim3(cdiv(R, 8)), dim3(512), 0, s, ARGS); break;
        case 9: hipLaunchKernelGGL((lab::wave_per_ray_buf<4, 4>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 10: hipLaunchKernelGGL((lab::wave_per_ray_buf<4, 2>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 11: hipLaunchKernelGGL((lab::wave_per_ray_buf<4, 1>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 12: hipLaunchKernelGGL((lab::wave_per_ray_buf<16, 2>), dim3(cdiv(R, 16)), dim3(1024), 0, s, ARGS); break;
        case 13: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 2, 1, 0, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 14: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 2, 0, 1, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 15: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 2, 1, 1, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 16: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 2, 1, 1, 2>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 17: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 4, 1, 1, 0>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 18: hipLaunchKernelGGL((lab::wave_per_ray_buf2<2, 2, 1, 1, 0>), dim3(cdiv(R, 2)), dim3(128), 0, s, ARGS); break;
        case 19: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 4, 1, 1, 0, 1>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 20: hipLaunchKernelGGL((lab::wave_per_ray_buf2<4, 4, 1, 1, 2, 1>), dim3(cdiv(R, 4)), dim3(256), 0, s, ARGS); break;
        case 100: hipLaunchKernelGGL(lab::empty_kernel, dim3(cdiv(R, 4)), dim3(256), 0, s, nullptr); break;
        case 101: hipLaunchKernelGGL(lab::empty_kernel, dim3(cdiv(R, 16)), dim3(1024), 0, s, nullptr); break;
        case 102: hipLaunchKernelGGL(lab::empty_kernel, dim3(256), dim3(256), 0, s, nullptr); break;
        case 103: hipLaunchKernelGGL(lab::empty_kernel, dim3(cdiv(R, 1)), dim3(64), 0, s, nullptr); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef ARGS
    return (int)hipGetLastError();
}

// Speed-of-light reference (not a compositor): the same algorithmic bytes as the forward, streamed
// flat with 16-B loads and no per-ray structure: read sigmas/deltas/ts/raws (24 B/sample) and
// rays_a, write ws (4 B/sample) and the per-ray outputs.
namespace lab {
__global__ __launch_bounds__(256) void flat_stream(const float4* __restrict__ sg, const float4* __restrict__ dl,
                                                   const float4* __restrict__ tt, const float4* __restrict__ rw,
                                                   int64_t S4, const int64_t* __restrict__ rays_a, int64_t R,
                                                   float* __restrict__ opacity, float* __restrict__ depth,
                                                   float* __restrict__ rend, int64_t* __restrict__ total,
                                                   float4* __restrict__ ws) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = n; i < S4; i += stride) {
        const float4 a = sg[i], b = dl[i], c = tt[i], r0 = rw[3 * i], r1 = rw[3 * i + 1], r2 = rw[3 * i + 2];
        ws[i] = make_float4(a.x * b.x + c.x + r0.x + r1.x + r2.x, a.y * b.y + c.y + r0.y + r1.y + r2.y,
                            a.z * b.z + c.z + r0.z + r1.z + r2.z, a.w * b.w + c.w + r0.w + r1.w + r2.w);
    }
    for (int64_t r = n; r < R; r += stride) {
        const int64_t q = rays_a[3 * r + 2];
        opacity[r] = (float)q; depth[r] = 0.f;
        rend[3 * r] = rend[3 * r + 1] = rend[3 * r + 2] = 0.f;
        total[r] = q;
    }
}
}  // namespace lab

extern "C" int lab_flat_stream(int blocks, const float* sigmas, const float* raws, const float* deltas,
                               const float* ts, const int64_t* rays_a, int64_t R, int64_t S, int64_t* total,
                               float* opacity, float* depth, float* rend, float* ws, void* stream) {
    hipLaunchKernelGGL(lab::flat_stream, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)sigmas,
                       (const float4*)deltas, (const float4*)ts, (const float4*)raws, S / 4, rays_a, R, opacity,
                       depth, rend, total, (float4*)ws);
    return (int)hipGetLastError();
}
