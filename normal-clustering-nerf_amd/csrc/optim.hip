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
    auto upd = [&](float& pi, float gr, float& mi, float& vi) {
        const float gi = gr * cf;
        mi = b1 * mi + (1.f - b1) * gi;
        vi = b2 * vi + (1.f - b2) * gi * gi;
        const float denom = sqrtf(vi / bc2) + eps;
        pi = pi - lr * ((mi / bc1) / denom + wd * pi);
    };
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
    const int64_t n4 = vec ? n / 4 : 0;
    for (int64_t i = tid; i < n4; i += nth) {  // 16-B accesses: 28 B/param at full width
        float4 P = ((float4*)p)[i], M = ((float4*)m)[i], V = ((float4*)v)[i];
        const float4 G = ((const float4*)g)[i];
        upd(P.x, G.x, M.x, V.x);
        upd(P.y, G.y, M.y, V.y);
        upd(P.z, G.z, M.z, V.z);
        upd(P.w, G.w, M.w, V.w);
        ((float4*)p)[i] = P;
        ((float4*)m)[i] = M;
        ((float4*)v)[i] = V;
    }
    for (int64_t i = 4 * n4 + tid; i < n; i += nth) upd(p[i], g[i], m[i], v[i]);
}

// ---------------------------------------------------------------------------------------------
// The optimizer step in two launches (train_nerf.py:262-285 + 955):
//  1. adam_prep_kernel: per-workgroup sums of squares of the gradient; the LAST workgroup to finish
//     (arrival counter) adds the partials in a fixed order and writes the step's scalars — clip
//     factor, bias corrections of the incremented device step, lr — then resets the counter;
//  2. adam_apply_kernel: Adam of both groups (index < n_group0: weight decay wd0, else wd1) with
//     16-B accesses, reading the four scalars; optionally zeroes the gradient it has consumed
//     (the next step's zero_grad fill folded into this pass: +4 B/param instead of a 4 B/param
//     fill launch).
// adam_prep runs ONE 1024-thread workgroup per CU (256 on MI355X): every arrival is an atomic on
// the same counter word, and same-address atomics serialise at the memory side (MI355X_MICROARCH.md
// "Global float atomics", contention row), so 2048 arrivals cost ~15-20 us where 256 cost ~2.
#ifndef NCN_ADAM_BLOCKS
#define NCN_ADAM_BLOCKS 256
#endif
#ifndef NCN_ADAM_UNROLL
#define NCN_ADAM_UNROLL 12
#endif
constexpr int ADAM_BLOCKS = NCN_ADAM_BLOCKS;  // workgroups of adam_prep (partials)
constexpr int ADAM_THREADS = 1024;
constexpr int ADAM_UNROLL = NCN_ADAM_UNROLL;  // float4 loads in flight per thread (45.8 MB: 11 per thread)
__global__ __launch_bounds__(ADAM_THREADS) void adam_prep_kernel(const float* __restrict__ g, int64_t n, float gscale,
                                                               float max_norm, double b1, double b2, float lr,
                                                               const float* __restrict__ lr_dev,
                                                               int* __restrict__ step_dev, float* __restrict__ work,
                                                               float* __restrict__ amp, const int* __restrict__ gate) {
    float* part = work;                                // [ADAM_BLOCKS]
    unsigned* cnt = (unsigned*)(work + ADAM_BLOCKS);   // arrival counter (left zero)
    float* sc = work + ADAM_BLOCKS + 4;                // cf, bc1, bc2, lr, skip (AMP)
    constexpr int NW = ADAM_THREADS / 64;
    __shared__ float red[NW];
    __shared__ bool last;
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * ADAM_THREADS;
    const float4* g4 = (const float4*)g;
    float s = 0.f;
    for (int64_t b = (int64_t)blockIdx.x * ADAM_THREADS + threadIdx.x; b < n4; b += ADAM_UNROLL * stride) {
        float4 x[ADAM_UNROLL];  // ADAM_UNROLL independent loads in flight per thread
#pragma unroll
        for (int u = 0; u < ADAM_UNROLL; u++) x[u] = b + u * stride < n4 ? g4[b + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < ADAM_UNROLL; u++) {
            s = fmaf(x[u].x, x[u].x, s); s = fmaf(x[u].y, x[u].y, s); s = fmaf(x[u].z, x[u].z, s); s = fmaf(x[u].w, x[u].w, s);
        }
    }
    if (blockIdx.x == 0)
        for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += ADAM_THREADS) s = fmaf(g[i], g[i], s);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    // Hand-off in the sc1 form of MI355X_MICROARCH.md "Correctness boundaries" (inter-workgroup
    // visibility): the partial is stored with an agent-scope (sc1) store and drained (vmcnt(0))
    // before the arrival add, and the last workgroup reads the partials with agent-scope (sc1)
    // loads.  This relies on gfx9's in-order completion of one wave's vector memory operations
    // after vmcnt(0), not on a HIP release/acquire pair: an agent-scope release fence writes back
    // the whole L2 (buffer_wbl2), which right after the table-gradient scatter measured ~40 us.
    // (The asm's "memory" clobber keeps the compiler from moving the store past the add.)
    if (threadIdx.x == 0) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; w++) t += red[w];
        __hip_atomic_store(&part[blockIdx.x], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the gridDim.x (<= ADAM_BLOCKS) partials, fixed-order sum in wave 0
    if (threadIdx.x < 64) {
        float q[ADAM_BLOCKS / 64];
#pragma unroll
        for (int u = 0; u < ADAM_BLOCKS / 64; u++) {
            const int i = u * 64 + threadIdx.x;
            q[u] = i < (int)gridDim.x ? __hip_atomic_load(&part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        }
        float t = 0.f;
#pragma unroll
        for (int u = 0; u < ADAM_BLOCKS / 64; u++) t += q[u];
        t = wave_sum(t);
        if (threadIdx.x == 0) {
            const float c = max_norm / (sqrtf(t) * gscale + 1e-6f);  // norm of the scaled gradient
            // GradScaler (AMP runs): a non-finite gradient skips the step and halves the scale;
            // NCN_AMP_GROWTH_INTERVAL finite steps in a row double it
            // gate == 0: no gradient is pending (a deferred optimizer step with nothing to apply):
            // the step is skipped without touching the scaler
            const bool gated_off = gate && *gate == 0;
            const bool skip = gated_off || (amp && !isfinite(t));
            if (amp && !gated_off) {
                float tr = skip ? 0.f : amp[1] + 1.f;
                float scale = skip ? amp[0] * 0.5f : amp[0];
                if (tr >= (float)NCN_AMP_GROWTH_INTERVAL) {
                    scale *= 2.f;
                    tr = 0.f;
                }
                amp[0] = scale;
                amp[1] = tr;
            }
            const int st = *step_dev + (skip ? 0 : 1);  // device step counter
            *step_dev = st;
            sc[4] = skip ? 1.f : 0.f;
            sc[0] = (max_norm > 0.f ? fminf(c, 1.0f) : 1.0f) * gscale;
            // bias corrections in double from the double betas, as apex's host code forms them
            // (1 - beta ** step in Python): 1 - 0.999f in f32 is off by 1.3e-5 relative
            sc[1] = (float)(1.0 - pow(b1, (double)st));
            sc[2] = (float)(1.0 - pow(b2, (double)st));
            sc[3] = lr_dev ? *lr_dev : lr;
            *cnt = 0u;
        }
    }
}
// (adam_apply takes 83 VGPRs: 5 waves/SIMD.  Measured with forced 6 / 8 waves per SIMD
// (tools/adam_probe.py, prep + apply over 11.45 M parameters): 72.7-73.1 / 75.0-75.7 us against
// 72.9-74.2 — HBM-bound.)
// Packed-fragment refresh folded into the Adam pass (PK: 0 none, 1 fp16, 2 bf16): parameter e in
// [poff, n) is master weight e - poff, written rounded to the operand type at its (up to two)
// packed positions pinv[2 (e - poff) + {0, 1}].
template <int PK>
__device__ __forceinline__ void adam_pack1(int64_t e, float x, const int32_t* __restrict__ pinv, int64_t poff,
                                           int64_t n, void* __restrict__ packed) {
    if (PK == 0 || e < poff || e >= n) return;
    const int64_t w = e - poff;
    const int2 q = ((const int2*)pinv)[w];
    if (PK == 1) {
        const _Float16 h = (_Float16)x;
        if (q.x >= 0) ((_Float16*)packed)[q.x] = h;
        if (q.y >= 0) ((_Float16*)packed)[q.y] = h;
    } else {
        const __bf16 h = (__bf16)x;
        if (q.x >= 0) ((__bf16*)packed)[q.x] = h;
        if (q.y >= 0) ((__bf16*)packed)[q.y] = h;
    }
}
template <bool ZERO, int PK>
__global__ __launch_bounds__(256) void adam_apply_kernel(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                         int64_t n0, float b1, float b2, float eps, float wd0,
                                                         float wd1, const float* __restrict__ sc,
                                                         const int32_t* __restrict__ pinv, int64_t poff,
                                                         void* __restrict__ packed) {
    const float cf = sc[0], bc1 = sc[1], bc2 = sc[2], lr = sc[3];
    if (sc[4] != 0.f) {  // (uniform) skipped AMP step: only the gradient is consumed
        if (PK) {  // (the packed fragments re-written from the unchanged weights: always consistent)
            const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
            for (int64_t e = poff + tid; e < n; e += nth) adam_pack1<PK>(e, p[e], pinv, poff, n, packed);
        }
        if (ZERO) {
            const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
            for (int64_t i = tid; i < n / 4; i += nth) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int64_t i = 4 * (n / 4) + tid; i < n; i += nth) g[i] = 0.f;
        }
        return;
    }
    auto upd = [&](float& pi, float gr, float& mi, float& vi, float wd) {
        const float gi = gr * cf;
        mi = b1 * mi + (1.f - b1) * gi;
        vi = b2 * vi + (1.f - b2) * gi * gi;
        const float denom = sqrtf(vi / bc2) + eps;
        pi = pi - lr * ((mi / bc1) / denom + wd * pi);
    };
    const int64_t n4 = n / 4, tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
#pragma unroll 2
    for (int64_t i = tid; i < n4; i += nth) {
        float4 P = ((float4*)p)[i], M = ((float4*)m)[i], V = ((float4*)v)[i];
        const float4 G = ((const float4*)g)[i];
        const int64_t e = 4 * i;
        upd(P.x, G.x, M.x, V.x, e < n0 ? wd0 : wd1);
        upd(P.y, G.y, M.y, V.y, e + 1 < n0 ? wd0 : wd1);
        upd(P.z, G.z, M.z, V.z, e + 2 < n0 ? wd0 : wd1);
        upd(P.w, G.w, M.w, V.w, e + 3 < n0 ? wd0 : wd1);
        ((float4*)p)[i] = P;
        ((float4*)m)[i] = M;
        ((float4*)v)[i] = V;
        if (PK && e + 3 >= poff) {
            adam_pack1<PK>(e, P.x, pinv, poff, n, packed);
            adam_pack1<PK>(e + 1, P.y, pinv, poff, n, packed);
            adam_pack1<PK>(e + 2, P.z, pinv, poff, n, packed);
            adam_pack1<PK>(e + 3, P.w, pinv, poff, n, packed);
        }
        // (the table gradient is sparse — most hash entries get no contribution in a step — so only
        // the non-zero float4s are written back as zeros: less HBM write traffic, same contents)
        if (ZERO && (G.x != 0.f || G.y != 0.f || G.z != 0.f || G.w != 0.f))
            ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int64_t i = 4 * n4 + tid; i < n; i += nth) {
        upd(p[i], g[i], m[i], v[i], i < n0 ? wd0 : wd1);
        adam_pack1<PK>(i, p[i], pinv, poff, n, packed);
        if (ZERO) g[i] = 0.f;
    }
}
// The step's inputs in one launch: up to NCN_STEP_MAX_BUFS buffer copies (the new batch into the
// captured graph's static input buffers) plus the device step counter the graph reads — instead of
// a multi-tensor copy launch and a fill launch ahead of every replay.  Workgroup b copies the 16-B
// chunks b, b + grid, ... of every buffer (bytes past the last whole chunk: byte copies).
constexpr int NCN_STEP_MAX_BUFS = 8;
struct StepCopies {
    const unsigned char* src[NCN_STEP_MAX_BUFS];
    unsigned char* dst[NCN_STEP_MAX_BUFS];
    int64_t bytes[NCN_STEP_MAX_BUFS];
};
__global__ __launch_bounds__(256) void step_inputs_kernel(StepCopies c, int nb, int64_t* step_dst, int64_t step,
                                                         int* flag_dst, int flag) {
    if (step_dst && blockIdx.x == 0 && threadIdx.x == 0) *step_dst = step;
    if (flag_dst && blockIdx.x == 0 && threadIdx.x == 0) *flag_dst = flag;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
    for (int b = 0; b < nb; b++) {
        const bool al = (((uintptr_t)c.src[b] | (uintptr_t)c.dst[b]) & 15) == 0;
        const int64_t n16 = al ? c.bytes[b] / 16 : 0;
        for (int64_t i = tid; i < n16; i += nth) ((uint4*)c.dst[b])[i] = ((const uint4*)c.src[b])[i];
        for (int64_t i = 16 * n16 + tid; i < c.bytes[b]; i += nth) c.dst[b][i] = c.src[b][i];
    }
}

// DDP gradient wire format (the data-parallel step's all-reduce): the reference's gradients are
// tcnn's fp16 parameter gradients at the GradScaler's scale S (tcnn modules keep fp16 params, and PL
// precision=16 scales the loss; train_nerf.py:944-955), and torch DDP's default communication hook
// divides every bucket by the world size BEFORE the all-reduce SUM ("Apply the division first to
// avoid overflow, especially for FP16": torch/distributed/algorithms/ddp_comm_hooks/default_hooks.py,
// _allreduce_fut).  So the wire carries fp16(fp16(S * g) / world): pack performs both roundings as
// DDP does (the bucket holds fp16(S * g); div_ rounds the quotient to fp16 again), the collective
// sums, and unpack writes float(w) / S — the world's average, so the optimizer takes no 1/world.
// Overflow -> inf, which the GradScaler step then skips on every rank alike, at the reference's
// magnitudes (a per-rank value near the fp16 maximum no longer overflows the 8-way sum).  8 elements
// per thread (two float4 loads, one 16-B store), a scalar tail.
__global__ __launch_bounds__(256) void grad_pack_f16_kernel(const float* __restrict__ g, int64_t n,
                                                            const float* __restrict__ scale, int world,
                                                            _Float16* __restrict__ w) {
    const float s = scale ? *scale : 1.f, wf = (float)world;
    // DDP's two roundings: the bucket's fp16(S g), then its in-place div_(world) (fp16 result)
    auto wire = [&](float x) { return (_Float16)((float)(_Float16)(x * s) / wf); };
    const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
        const float4 a = ((const float4*)g)[2 * i], b = ((const float4*)g)[2 * i + 1];
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
        const h8 o = {wire(a.x), wire(a.y), wire(a.z), wire(a.w), wire(b.x), wire(b.y), wire(b.z), wire(b.w)};
        ((h8*)w)[i] = o;
    }
    for (int64_t i = 8 * n8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) w[i] = wire(g[i]);
}
__global__ __launch_bounds__(256) void grad_unpack_f16_kernel(const _Float16* __restrict__ w, int64_t n,
                                                              const float* __restrict__ scale, float* __restrict__ g) {
    const float inv = scale ? 1.f / *scale : 1.f;
    const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * 256;
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
        const h8 v = ((const h8*)w)[i];
        ((float4*)g)[2 * i] = make_float4((float)v[0] * inv, (float)v[1] * inv, (float)v[2] * inv, (float)v[3] * inv);
        ((float4*)g)[2 * i + 1] = make_float4((float)v[4] * inv, (float)v[5] * inv, (float)v[6] * inv, (float)v[7] * inv);
    }
    for (int64_t i = 8 * n8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) g[i] = (float)w[i] * inv;
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int ncn_grad_pack_f16(const float* grad, int64_t n, const float* scale, int world, uint16_t* wire, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(world >= 1, hipErrorInvalidValue, "ncn_grad_pack_f16: world must be >= 1");
    NCN_REQUIRE(((((uintptr_t)grad) & 15) | (((uintptr_t)wire) & 15)) == 0, hipErrorInvalidValue,
                "ncn_grad_pack_f16: grad and wire must be 16-byte aligned");
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 2048)), 4096);
    hipLaunchKernelGGL(grad_pack_f16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, grad, n, scale,
                       world, (_Float16*)wire);
    NCN_LAUNCH_CHECK("ncn_grad_pack_f16");
    return 0;
}

int ncn_grad_unpack_f16(const uint16_t* wire, int64_t n, const float* scale, float* grad, void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(((((uintptr_t)grad) & 15) | (((uintptr_t)wire) & 15)) == 0, hipErrorInvalidValue,
                "ncn_grad_unpack_f16: grad and wire must be 16-byte aligned");
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 2048)), 4096);
    hipLaunchKernelGGL(grad_unpack_f16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const _Float16*)wire,
                       n, scale, grad);
    NCN_LAUNCH_CHECK("ncn_grad_unpack_f16");
    return 0;
}

int ncn_step_inputs(int n_bufs, const void* const* src, void* const* dst, const int64_t* n_bytes, int64_t* step_dst,
                    int64_t step, int32_t* flag_dst, int32_t flag, void* stream) {
    NCN_REQUIRE(n_bufs >= 0 && n_bufs <= NCN_STEP_MAX_BUFS, hipErrorInvalidValue,
                "ncn_step_inputs: at most 8 buffers");
    StepCopies c{};
    int64_t total = 0;
    for (int b = 0; b < n_bufs; b++) {
        NCN_REQUIRE(n_bytes[b] >= 0 && (n_bytes[b] == 0 || (src[b] && dst[b])), hipErrorInvalidValue,
                    "ncn_step_inputs: null buffer");
        c.src[b] = (const unsigned char*)src[b];
        c.dst[b] = (unsigned char*)dst[b];
        c.bytes[b] = n_bytes[b];
        total += n_bytes[b];
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(256, (total / 16 + 255) / 256));
    hipLaunchKernelGGL(step_inputs_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, c, n_bufs, step_dst, step,
                       flag_dst, flag);
    NCN_LAUNCH_CHECK("ncn_step_inputs");
    return 0;
}

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
    const int blocks = (int)std::min<int64_t>(cdiv(n, 1024), 2048);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg,
                       exp_avg_sq, n, sumsq_partial, max_norm, lr, beta1, beta2, eps, weight_decay, bc1, bc2, lr_dev,
                       step_dev);
    NCN_LAUNCH_CHECK("ncn_adam");
    return 0;
}

}  // extern "C"

template <int PK>
static void launch_apply(int zero, int blocks, hipStream_t st, float* params, float* grads, float* exp_avg,
                         float* exp_avg_sq, int64_t n, int64_t n_group0, double beta1, double beta2, float eps,
                         float wd0, float wd1, const float* sc, const int32_t* pinv, int64_t poff, void* packed) {
    if (zero)
        hipLaunchKernelGGL((adam_apply_kernel<true, PK>), dim3(blocks), dim3(256), 0, st, params, grads, exp_avg,
                           exp_avg_sq, n, n_group0, (float)beta1, (float)beta2, eps, wd0, wd1, sc, pinv, poff, packed);
    else
        hipLaunchKernelGGL((adam_apply_kernel<false, PK>), dim3(blocks), dim3(256), 0, st, params, grads, exp_avg,
                           exp_avg_sq, n, n_group0, (float)beta1, (float)beta2, eps, wd0, wd1, sc, pinv, poff, packed);
}

static int adam_step_impl(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t n_group0,
                          float grad_scale, float max_norm, float lr, double beta1, double beta2, float eps, float wd0,
                          float wd1, const float* lr_dev, int* step_dev, float* work, int zero_grads,
                          float* amp_state, const int* gate, const int32_t* pinv, int64_t poff, void* packed, int pk,
                          void* stream) {
    if (n <= 0) return 0;
    NCN_REQUIRE(((((uintptr_t)params) | ((uintptr_t)grads) | ((uintptr_t)exp_avg) | ((uintptr_t)exp_avg_sq)) & 15) == 0,
                hipErrorInvalidValue, "ncn_adam_step: buffers must be 16-byte aligned");
    NCN_REQUIRE(step_dev != nullptr && work != nullptr, hipErrorInvalidValue,
                "ncn_adam_step: needs the device step counter and the work buffer");
    const int prep_blocks = (int)std::min<int64_t>(ADAM_BLOCKS, std::max<int64_t>(1, cdiv(n / 4, ADAM_THREADS * 4)));
    hipLaunchKernelGGL(adam_prep_kernel, dim3(prep_blocks), dim3(ADAM_THREADS), 0, (hipStream_t)stream, grads, n,
                       grad_scale, max_norm, beta1, beta2, lr, lr_dev, step_dev, work, amp_state, gate);
    NCN_LAUNCH_CHECK("ncn_adam_step (prep)");
    // two float4 per thread (8 loads of p/g/m/v in flight): ~n/2048 workgroups
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(n, 2048)), 16384);
    const float* sc = work + ADAM_BLOCKS + 4;
    const hipStream_t st = (hipStream_t)stream;
    if (pk == 0)
        launch_apply<0>(zero_grads, blocks, st, params, grads, exp_avg, exp_avg_sq, n, n_group0, beta1, beta2, eps, wd0,
                        wd1, sc, nullptr, 0, nullptr);
    else if (pk == 1)
        launch_apply<1>(zero_grads, blocks, st, params, grads, exp_avg, exp_avg_sq, n, n_group0, beta1, beta2, eps, wd0,
                        wd1, sc, pinv, poff, packed);
    else
        launch_apply<2>(zero_grads, blocks, st, params, grads, exp_avg, exp_avg_sq, n, n_group0, beta1, beta2, eps, wd0,
                        wd1, sc, pinv, poff, packed);
    NCN_LAUNCH_CHECK("ncn_adam_step");
    return 0;
}

extern "C" {

int ncn_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t n_group0,
                  float grad_scale, float max_norm, float lr, double beta1, double beta2, float eps, float wd0, float wd1,
                  const float* lr_dev, int* step_dev, float* work, int zero_grads, float* amp_state, const int* gate,
                  void* stream) {
    return adam_step_impl(params, grads, exp_avg, exp_avg_sq, n, n_group0, grad_scale, max_norm, lr, beta1, beta2, eps,
                          wd0, wd1, lr_dev, step_dev, work, zero_grads, amp_state, gate, nullptr, 0, nullptr, 0, stream);
}

int ncn_adam_step_packed(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, int64_t n_group0,
                         float grad_scale, float max_norm, float lr, double beta1, double beta2, float eps, float wd0,
                         float wd1, const float* lr_dev, int* step_dev, float* work, int zero_grads, float* amp_state,
                         const int* gate, const int32_t* pack_inv, int64_t pack_off, uint16_t* packed, int pack_prec,
                         void* stream) {
    NCN_REQUIRE(pack_inv && packed && (pack_prec == NCN_PREC_F16 || pack_prec == NCN_PREC_BF16) && pack_off >= 0 &&
                    n - pack_off == NCN_FIELD_NW && (((uintptr_t)pack_inv) & 7) == 0,
                hipErrorInvalidValue, "ncn_adam_step_packed: pack_inv/packed/pack_prec/pack_off invalid");
    return adam_step_impl(params, grads, exp_avg, exp_avg_sq, n, n_group0, grad_scale, max_norm, lr, beta1, beta2, eps,
                          wd0, wd1, lr_dev, step_dev, work, zero_grads, amp_state, gate, pack_inv, pack_off, packed,
                          pack_prec == NCN_PREC_F16 ? 1 : 2, stream);
}

int64_t ncn_adam_step_work_floats(void) { return ADAM_BLOCKS + 12; }

}  // extern "C"
