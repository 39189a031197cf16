// Diagnostic (not product): throughput of scattered f32 global atomics on gfx950 — table size,
// memory scope, duplicates — to size the table-gradient flush of the field scatter.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ __forceinline__ uint32_t hash32(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }
template <int SCOPE>
__global__ void k_atomic(float* t, uint32_t mask, int per_thread, uint32_t seed, int pairs) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < per_thread; i++) {
        uint32_t e = hash32(tid * 7919u + i * 104729u + seed) & mask;
        if (pairs) e &= ~1u;
        if (SCOPE == 0) atomicAdd(t + e, 1.0f);
        else if (SCOPE == 1) __hip_atomic_fetch_add(t + e, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else t[e] += 1.0f;  // plain RMW (wrong under races; bandwidth reference)
        if (pairs) atomicAdd(t + e + 1, 1.0f);
    }
}
int main() {
    float* t;
    const size_t N = 16u << 20;  // 16M floats = 64 MB
    (void)hipMalloc(&t, N * 4);
    (void)hipMemset(t, 0, N * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const int threads = 256 * 1024, per = 16;  // 4M atomics (x2 with pairs)
    for (uint32_t mask : {(1u << 20) - 1, (1u << 22) - 1, (1u << 24) - 1}) {
        for (int scope = 0; scope < 3; scope++) {
            for (int pairs = 0; pairs < 2; pairs++) {
                float best = 1e9;
                for (int rep = 0; rep < 5; rep++) {
                    (void)hipEventRecord(a);
                    if (scope == 0) hipLaunchKernelGGL(k_atomic<0>, dim3(threads / 256), dim3(256), 0, 0, t, mask, per, rep, pairs);
                    if (scope == 1) hipLaunchKernelGGL(k_atomic<1>, dim3(threads / 256), dim3(256), 0, 0, t, mask, per, rep, pairs);
                    if (scope == 2) hipLaunchKernelGGL(k_atomic<2>, dim3(threads / 256), dim3(256), 0, 0, t, mask, per, rep, pairs);
                    (void)hipEventRecord(b);
                    (void)hipEventSynchronize(b);
                    float ms; (void)hipEventElapsedTime(&ms, a, b);
                    best = ms < best ? ms : best;
                }
                const double n = (double)threads * per * (pairs ? 2 : 1);
                printf("table %6.1f MB scope %s pairs %d: %8.1f us  %6.2f G ops/s\n", (mask + 1) * 4.0 / 1e6,
                       scope == 0 ? "agent" : scope == 1 ? "wg   " : "plain", pairs, best * 1e3, n / (best * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
