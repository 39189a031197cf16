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
