// Shared helpers for libncnerf.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

namespace ncn {

// Per-thread last-error message for ncn_last_error().
void set_error(const char* fmt, ...);

constexpr int WAVE = 64;

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
