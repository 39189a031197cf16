// Shared helpers for libncnerf.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

namespace ncn {

// Per-thread last-error message for ncn_last_error().
void set_error(const char* fmt, ...);

constexpr int WAVE = 64;
#define NCN_MAX_DEVICES 64  // per-device caches of host-side launch checks

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// Wave64 shuffles (ds_bpermute based; all 64 lanes participate).
__device__ __forceinline__ float shfl(float v, int src) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
__device__ __forceinline__ int shfl_i(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Inclusive scans across the 64 lanes (Hillis-Steele, 6 steps).
__device__ __forceinline__ int wave_incl_sum_i(int v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}

__device__ __forceinline__ float wave_incl_sum(float v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        float o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}
__device__ __forceinline__ float wave_incl_prod(float v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        float o = __shfl_up(v, off, 64);
        if (lane >= off) v *= o;
    }
    return v;
}

// DPP wave scans (GFX9 DPP: row_shr within 16-lane rows, then row_bcast:15 / row_bcast:31 across
// rows): 6 DPP ops with ~no latency, no LDS crossbar traffic (unlike __shfl_* = ds_bpermute).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROW_MASK, 0xF,
                                                      false));
}
__device__ __forceinline__ float wave_incl_prod_dpp(float v) {
    v *= dpp_f<0x111, 0xF>(1.0f, v);  // row_shr:1
    v *= dpp_f<0x112, 0xF>(1.0f, v);  // row_shr:2
    v *= dpp_f<0x114, 0xF>(1.0f, v);  // row_shr:4
    v *= dpp_f<0x118, 0xF>(1.0f, v);  // row_shr:8
    v *= dpp_f<0x142, 0xA>(1.0f, v);  // row_bcast:15 into rows 1, 3
    v *= dpp_f<0x143, 0xC>(1.0f, v);  // row_bcast:31 into rows 2, 3
    return v;
}
__device__ __forceinline__ float wave_incl_sum_dpp(float v) {
    v += dpp_f<0x111, 0xF>(0.0f, v);
    v += dpp_f<0x112, 0xF>(0.0f, v);
    v += dpp_f<0x114, 0xF>(0.0f, v);
    v += dpp_f<0x118, 0xF>(0.0f, v);
    v += dpp_f<0x142, 0xA>(0.0f, v);
    v += dpp_f<0x143, 0xC>(0.0f, v);
    return v;
}
// value of lane (l - 1), `first` for lane 0 (DPP wave_shr:1)
__device__ __forceinline__ float wave_shr1_dpp(float v, float first) { return dpp_f<0x138, 0xF>(first, v); }
// wave total via the inclusive DPP scan, read from lane 63 (uniform result)
__device__ __forceinline__ float wave_sum_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_incl_sum_dpp(v)), 63));
}

// Inclusive product scan as 6 fused v_mul_f32_dpp with the register as both sources and no
// bound_ctrl: a lane without a DPP source is not written, i.e. keeps its value (x 1).  The
// compiler's update_dpp form needs a v_mov of the identity + v_mov_dpp + v_mul per step.
// `s_nop 1` covers the VALU-write -> DPP-read hazard (2 wait states) before every step.
__device__ __forceinline__ float wave_incl_prod_dpp_fused(float v) {
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

// K independent inclusive product scans at once (rows of the same ray): one asm with the K
// registers' DPP steps interleaved, so for K >= 4 the VALU-write -> DPP-read wait states are filled
// by the other rows' steps instead of s_nops (K == 2 keeps one s_nop 0 per step).
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

// Four independent inclusive sum scans at once (v_add_f32_dpp, same no-bound_ctrl identity trick:
// a lane without a DPP source keeps its value, i.e. + 0); the 4-way interleave fills the wait states.
__device__ __forceinline__ void wave_incl_sum4(float& a, float& b, float& c, float& d) {
#define NCN_DPPA(R, CTRL) "v_add_f32_dpp %" #R ", %" #R ", %" #R " " CTRL "\n\t"
#define NCN_ASTEP4(C) NCN_DPPA(0, C) NCN_DPPA(1, C) NCN_DPPA(2, C) NCN_DPPA(3, C)
    asm volatile("s_nop 1\n\t" NCN_ASTEP4(NCN_S1) NCN_ASTEP4(NCN_S2) NCN_ASTEP4(NCN_S4) NCN_ASTEP4(NCN_S8)
                     NCN_ASTEP4(NCN_S15) NCN_ASTEP4(NCN_S31) "s_nop 1"
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#undef NCN_ASTEP4
#undef NCN_DPPA
}

// Wave totals of K values at once (CDNA4 permlane swaps): v_permlane32_swap pairs values so the
// lower half-wave carries one and the upper half the other, v_permlane16_swap halves again, then
// one 16-lane row total per register (row_ror 8/4/2/1).  ~3K+6 instructions instead of K full
// 64-lane DPP reductions (~8K + s_nops).  Result i is returned uniform in v[i].
__device__ __forceinline__ float swap32_sum(float a, float b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_sum(float a, float b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp_add_zero(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_total(float v) {
    v = dpp_add_zero<0x128>(v);  // row_ror:8
    v = dpp_add_zero<0x124>(v);  // row_ror:4
    v = dpp_add_zero<0x122>(v);  // row_ror:2
    v = dpp_add_zero<0x121>(v);  // row_ror:1
    return v;
}
template <int K>
__device__ __forceinline__ void wave_sum_multi(float (&v)[K]) {
    constexpr int K1 = (K + 1) / 2, K2 = (K1 + 1) / 2;
    float P[K1], Q[K2];
#pragma unroll
    for (int i = 0; i < K1; i++) P[i] = swap32_sum(v[2 * i], (2 * i + 1 < K) ? v[2 * i + 1] : v[2 * i]);
#pragma unroll
    for (int j = 0; j < K2; j++) Q[j] = row16_total(swap16_sum(P[2 * j], (2 * j + 1 < K1) ? P[2 * j + 1] : P[2 * j]));
    // value m sits in P[m/2], half m%2 (lanes 0-31 / 32-63); P[i] sits in Q[i/2], rows (i%2) + 2*half
#pragma unroll
    for (int m = 0; m < K; m++) {
        const int i = m / 2, h = (2 * i + 1 < K) ? (m & 1) : 0;
        const int row = (((2 * (i / 2) + 1) < K1) ? (i & 1) : 0) + 2 * h;
        v[m] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Q[i / 2]), row * 16));
    }
}

// A zero the compiler cannot see through: indexing loop-invariant LDS data with it keeps the
// loads inside the loop instead of hoisting them into (scarce) registers.
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

// Workgroup barrier that orders LDS only: waits for the wave's own LDS operations (lgkmcnt) but
// not for its outstanding global loads/stores/atomics (vmcnt), which __syncthreads() also drains.
// For phases that exchange data through LDS while fire-and-forget global stores / atomics or
// prefetch loads are in flight.
// XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs (block b runs on
// XCD b % 8), each with its own L2.  Renumbering blocks so that XCD x takes the contiguous logical
// range [x * G/8, (x+1) * G/8) keeps neighbouring work — the samples of one ray patch, which
// gather the same hash-table entries — inside one L2.  Identity when G is not a multiple of 8.
// (Placement is a performance hint only: nothing may depend on it for correctness.)
__device__ __forceinline__ int xcd_block(int b, int G) { return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3); }

// total_samples.sum() by one 1024-thread workgroup (+ optional f64 accumulators: acc[0] +=
// counter[0] (marched), acc[1] += the sum (composited)) — ncn_count_samples, and the extra
// workgroup of ncn_photo_normals_count_fwd.
__device__ __forceinline__ void count_samples_wg(const int64_t* __restrict__ total, int64_t R,
                                                 const int32_t* __restrict__ counter, int64_t* __restrict__ sum_out,
                                                 double* __restrict__ acc) {
    __shared__ long long part[16];
    long long v = 0;
    for (int64_t i = threadIdx.x; i < R; i += blockDim.x) v += total[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)v, off, 64), hi = __shfl_xor((unsigned)((unsigned long long)v >> 32), off, 64);
        v += (long long)(((unsigned long long)hi << 32) | lo);
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += part[w];
        *sum_out = t;
        if (acc) {
            acc[0] += counter ? (double)counter[0] : 0.0;
            acc[1] += (double)t;
        }
    }
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Raw buffer resources (T8): a descriptor sized to one segment makes the hardware bounds check
// return 0 for loads past it and drop stores past it, so row bodies carry no masks or branches.
// Build them from wave-uniform values only (scalar loads / kernargs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
__device__ __forceinline__ void buf_store(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, byte_off, 0, 0);
}

}  // namespace ncn

#define NCN_LAUNCH_CHECK(name)                                                         \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) {                                                       \
            ncn::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));     \
            return (int)e_;                                                           \
        }                                                                             \
    } while (0)

#define NCN_REQUIRE(cond, code, ...)                                                  \
    do {                                                                              \
        if (!(cond)) {                                                                \
            ncn::set_error(__VA_ARGS__);                                              \
            return (int)(code);                                                       \
        }                                                                             \
    } while (0)
