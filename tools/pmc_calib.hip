// Diagnostic (not product): FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access patterns of
// the table scatter (MI355X_MICROARCH.md HBM section: "other access widths are uncalibrated: calibrate
// on a known byte count in your own access pattern").  Each kernel moves a known number of bytes over
// buffers far larger than the Infinity Cache, so the per-dispatch counters can be set against it:
//   stream16   16 B per lane, coalesced (the guide's reference: FETCH_SIZE reads half)
//   chunk48    48 B per lane as 3 x float4 at a 48-B lane stride (a coarse unit's position chunk)
//   chunk24    24 B per lane as 3 x float2 at a 24-B lane stride (a fine grab's position pair)
//   pair8      8 B per lane as one uint2 (a fine grab's dE pair)
//   atomics    f32 atomicAdd of adjacent (x, y) floats by lane pairs at random entries of a 46 MB
//              table, as the scatter's flush (2 atomics, one 8-B piece of one line per entry)
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); prints the bytes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__global__ void k_stream16(const float4* __restrict__ a, int64_t n4, float* __restrict__ out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void k_chunk48(const float4* __restrict__ a, int64_t nchunks, float* __restrict__ out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = a[3 * i], q = a[3 * i + 1], r = a[3 * i + 2];
        s += p.x + q.y + r.z + p.w + q.x + r.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void k_chunk24(const float2* __restrict__ a, int64_t nchunks, float* __restrict__ out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * blockDim.x) {
        const float2 p = a[3 * i], q = a[3 * i + 1], r = a[3 * i + 2];
        s += p.x + q.y + r.x + p.y;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void k_pair8(const uint2* __restrict__ a, int64_t n, float* __restrict__ out) {
    uint32_t s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint2 v = a[i];
        s += v.x ^ v.y;
    }
    if (s == 12345u) out[0] = (float)s;
}
__global__ void k_atomics(float* __restrict__ t, uint32_t entries, int64_t n_pairs) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n_pairs; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t e = hash32((uint32_t)(i >> 1) * 2654435761u + 12345u) % entries;
        atomicAdd(t + 2 * (size_t)e + (i & 1), 1.0f);
    }
}

int main() {
    const size_t big = 512ull << 20;  // 512 MB buffer: past the 256 MiB Infinity Cache
    char *a, *t;
    float* out;
    (void)hipMalloc(&a, big);
    (void)hipMalloc(&t, 46ull << 20);
    (void)hipMalloc(&out, 64);
    (void)hipMemset(a, 1, big);
    (void)hipMemset(t, 0, 46ull << 20);
    const int grid = 256 * 8, block = 256;
    const int64_t n_pairs = 2 << 20;  // 2 M entries (the scatter's flush claims ~1.7 M fine + coarse)
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(block), 0, 0, (const float4*)a, (int64_t)(256ull << 20) / 16, out);
        hipLaunchKernelGGL(k_chunk48, dim3(grid), dim3(block), 0, 0, (const float4*)a, (int64_t)(256ull << 20) / 48, out);
        hipLaunchKernelGGL(k_chunk24, dim3(grid), dim3(block), 0, 0, (const float2*)a, (int64_t)(256ull << 20) / 24, out);
        hipLaunchKernelGGL(k_pair8, dim3(grid), dim3(block), 0, 0, (const uint2*)a, (int64_t)(256ull << 20) / 8, out);
        hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(block), 0, 0, (float*)t, (uint32_t)((46ull << 20) / 8), n_pairs);
    }
    (void)hipDeviceSynchronize();
    printf("known bytes per dispatch: stream16/chunk48/chunk24/pair8 read %llu B each; atomics %lld f32 atomics "
           "(%lld B of operands, %lld entry pairs)\n",
           (unsigned long long)(256ull << 20), (long long)(2 * n_pairs), (long long)(8 * n_pairs), (long long)n_pairs);
    return 0;
}
