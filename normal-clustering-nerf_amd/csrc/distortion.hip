// Distortion loss of Mip-NeRF 360 in DVGO-v2's O(N) form (reference: models/csrc/losses.cu,
// vren.distortion_loss_fw / _bw, losses.py:16-44): per ray
//   loss = sum_s 2 (wts_incl[s] ws_excl[s] - ws_incl[s] wts_excl[s]) + 1/3 ws[s]^2 deltas[s],
// wts = ws * ts, incl / excl = inclusive / exclusive prefix sums over the ray's segment.
// One wave per ray, the segment in rows of 64 samples; each row's prefix sums are a DPP wave scan
// plus the carry of the previous rows (the reference scans serially with thrust: fp32 rounding
// order differs, tolerance in tests/test_gpu_distortion.py).
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

__device__ __forceinline__ void dist_seg(const int64_t* __restrict__ rays_a, int64_t R, int64_t& ray, int64_t& start,
                                         int& N, bool& live) {
    const int64_t n0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    live = n0 < R;
    const int64_t n = live ? n0 : R - 1;
    ray = rays_a[3 * n];
    start = rays_a[3 * n + 1];
    N = (int)rays_a[3 * n + 2];
}

// losses.cu:47-100 (prefix sums + per-sample terms + per-ray reduce)
__global__ __launch_bounds__(256) void distortion_fw_kernel(const float* __restrict__ ws,
                                                            const float* __restrict__ deltas,
                                                            const float* __restrict__ ts,
                                                            const int64_t* __restrict__ rays_a, int64_t R,
                                                            float* __restrict__ loss, float* __restrict__ ws_incl,
                                                            float* __restrict__ wts_incl) {
    const int lane = threadIdx.x & 63;
    int64_t ray, start;
    int N;
    bool live;
    dist_seg(rays_a, R, ray, start, N, live);
    if (!live) return;
    float cw = 0.f, cwt = 0.f, acc = 0.f;  // carries of the prefix sums, per-lane loss terms
    for (int base = 0; base < N; base += 64) {
        const int k = base + lane;
        const bool in = k < N;
        const int64_t s = start + k;
        const float w = in ? ws[s] : 0.f, t = in ? ts[s] : 0.f, d = in ? deltas[s] : 0.f;
        const float wt = w * t;
        const float iw = cw + wave_incl_sum_dpp(w), iwt = cwt + wave_incl_sum_dpp(wt);
        const float ew = iw - w, ewt = iwt - wt;
        if (in) {
            ws_incl[s] = iw;
            wts_incl[s] = iwt;
            acc += 2.0f * (iwt * ew - iw * ewt) + (1.0f / 3.0f) * w * w * d;
        }
        cw = __shfl(iw, 63, 64);
        cwt = __shfl(iwt, 63, 64);
    }
    acc = wave_sum(acc);
    if (lane == 0) loss[ray] = acc;
}

// losses.cu:103-140
__global__ __launch_bounds__(256) void distortion_bw_kernel(const float* __restrict__ dL_dloss,
                                                            const float* __restrict__ ws_incl,
                                                            const float* __restrict__ wts_incl,
                                                            const float* __restrict__ ws,
                                                            const float* __restrict__ deltas,
                                                            const float* __restrict__ ts,
                                                            const int64_t* __restrict__ rays_a, int64_t R,
                                                            float* __restrict__ dL_dws) {
    const int lane = threadIdx.x & 63;
    int64_t ray, start;
    int N;
    bool live;
    dist_seg(rays_a, R, ray, start, N, live);
    if (!live || N <= 0) return;
    const float g = dL_dloss[ray];
    const int64_t end = start + N - 1;
    const float ws_sum = ws_incl[end], wts_sum = wts_incl[end];
    for (int base = 0; base < N; base += 64) {
        const int k = base + lane;
        if (k >= N) continue;
        const int64_t s = start + k;
        const float t = ts[s], iw = ws_incl[s], iwt = wts_incl[s];
        const float before = k == 0 ? 0.f : t * ws_incl[s - 1] - wts_incl[s - 1];
        float v = g * 2 * (before + (wts_sum - iwt - t * (ws_sum - iw)));
        v += g * (2.0f / 3.0f) * ws[s] * deltas[s];
        dL_dws[s] = v;
    }
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int ncn_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                           float* loss, float* ws_inclusive_scan, float* wts_inclusive_scan, void* stream) {
    if (n_rays <= 0) return 0;
    hipLaunchKernelGGL(distortion_fw_kernel, dim3(cdiv(n_rays, 4)), dim3(256), 0, (hipStream_t)stream, ws, deltas, ts,
                       rays_a, n_rays, loss, ws_inclusive_scan, wts_inclusive_scan);
    NCN_LAUNCH_CHECK("ncn_distortion_loss_fw");
    return 0;
}

int ncn_distortion_loss_bw(const float* dL_dloss, const float* ws_inclusive_scan, const float* wts_inclusive_scan,
                           const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* dL_dws, void* stream) {
    if (n_rays <= 0) return 0;
    hipLaunchKernelGGL(distortion_bw_kernel, dim3(cdiv(n_rays, 4)), dim3(256), 0, (hipStream_t)stream, dL_dloss,
                       ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a, n_rays, dL_dws);
    NCN_LAUNCH_CHECK("ncn_distortion_loss_bw");
    return 0;
}

}  // extern "C"
