// Optimizer step over the flat fp32 parameter buffer (reference: apex FusedAdam in AdamW mode with
// eps 1e-15 and per-group weight decay, train_nerf.py:262-285; gradient clipping by global L2 norm
// 0.05, train_nerf.py:955 via PL -> torch.nn.utils.clip_grad_norm_).  The clip factor is computed
// on device from the sum-of-squares partials, so the step has no host synchronisation.
#include <algorithm>
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

constexpr int SUMSQ_BLOCKS = 1024;

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ part,
                                                    int* __restrict__ step_inc) {
    __shared__ float red[4];
    if (step_inc && blockIdx.x == 0 && threadIdx.x == 0) *step_inc += 1;  // device step counter
    float s = 0.f;
    const int64_t n4 = n / 4;
    const float4* x4 = (const float4*)x;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 v = x4[i];
        s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
    if (blockIdx.x == 0)
        for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) s = fmaf(x[i], x[i], s);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ float clip_coef(const float* __restrict__ part, float max_norm) {
    __shared__ float c_s;
    if (threadIdx.x < 64) {
        float s = 0.f;
        for (int i = threadIdx.x; i < SUMSQ_BLOCKS; i += 64) s += part[i];
        s = wave_sum(s);
        if (threadIdx.x == 0) {
            const float norm = sqrtf(s);
            const float c = max_norm / (norm + 1e-6f);
            c_s = max_norm > 0.f ? fminf(c, 1.0f) : 1.0f;
        }
    }
    __syncthreads();
    return c_s;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const float* __restrict__ part, float max_norm, float lr, float b1,
                                                   float b2, float eps, float wd, float bc1, float bc2,
                                                   const float* __restrict__ lr_dev, const int* __restrict__ step_dev) {
    const float cf = part ? clip_coef(part, max_norm) : 1.0f;
    if (lr_dev) lr = *lr_dev;
    if (step_dev) {  // bias corrections from the device step (graph-captured step)
        const float st = (float)*step_dev;
        bc1 = 1.0f - powf(b1, st);
        bc2 = 1.0f - powf(b2, st);
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float gi = g[i] * cf;
        const float mi = b1 * m[i] + (1.f - b1) * gi;
        const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi / bc2) + eps;
        p[i] = p[i] - lr * ((mi / bc1) / denom + wd * p[i]);
    }
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int ncn_sumsq(const float* x, int64_t n, float* out_partial, int* step_inc, void* stream) {
    hipLaunchKernelGGL(sumsq_kernel, dim3(SUMSQ_BLOCKS), dim3(256), 0, (hipStream_t)stream, x, n, out_partial,
                       step_inc);
    NCN_LAUNCH_CHECK("ncn_sumsq");
    return 0;
}

int ncn_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
             const float* sumsq_partial, float max_norm, float lr, float beta1, float beta2, float eps,
             float weight_decay, int step, const float* lr_dev, const int* step_dev, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(step >= 1 || step_dev, hipErrorInvalidValue, "ncn_adam: step must be >= 1");
    const float bc1 = 1.0f - powf(beta1, (float)std::max(step, 1)), bc2 = 1.0f - powf(beta2, (float)std::max(step, 1));
    const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 2048);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg,
                       exp_avg_sq, n, sumsq_partial, max_norm, lr, beta1, beta2, eps, weight_decay, bc1, bc2, lr_dev,
                       step_dev);
    NCN_LAUNCH_CHECK("ncn_adam");
    return 0;
}

}  // extern "C"
