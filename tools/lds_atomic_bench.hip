// Diagnostic microbenchmark: cost of LDS float atomics (ds_add_f32) vs plain LDS RMW on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHECK(x) do { hipError_t e = (x); if (e) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void k(float* out, int iters, int active) {
    __shared__ float buf[8192];
    for (int i = threadIdx.x; i < 8192; i += 512) buf[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t h = (threadIdx.x * 2654435761u) >> 19;  // random-ish slot
    float v = 1.0f + lane;
    for (int it = 0; it < iters; it++) {
        if (lane < active) {
            int slot;
            if (MODE == 0 || MODE >= 4) slot = (w * 64 + lane) & 8191;        // distinct, conflict-free
            else if (MODE == 1) slot = (h + it * 97) & 8191;       // random
            else if (MODE == 2) slot = w;                          // all lanes same address
            else slot = (w * 64 + (lane & 3)) & 8191;              // 16-way same address groups
            if (MODE == 4) atomicAdd((unsigned*)&buf[slot], (unsigned)lane);
            else if (MODE == 5) atomicCAS((unsigned*)&buf[slot], 0xFFFFFFFFu, (unsigned)lane);
            else if (MODE == 6) buf[slot] += v;  // plain RMW (racy; timing only)
            else if (MODE == 7) atomicAdd((unsigned long long*)&buf[slot & ~1], (unsigned long long)lane);
            else atomicAdd(&buf[slot], v);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = buf[0];
}

int main() {
    float* out;
    CHECK(hipMalloc(&out, 4096 * 4));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 2000, blocks = 512;
    const char* names[8] = {"distinct", "random", "same-addr", "4-addr", "u32 add", "u32 cas", "plain rmw", "u64 add"};
    for (int mode = 0; mode < 8; mode++)
        for (int active : {64, 16, 1}) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 6) hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
                if (mode == 7) hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(512), 0, 0, out, iters, active);
            };
            launch();
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            CHECK(hipEventSynchronize(b));
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // wave-instructions per CU: blocks*8 waves*iters / 256 CUs
            const double winst = (double)blocks * 8 * iters / 256;
            printf("%-10s active %2d: %8.3f ms  %6.1f cycles per wave-instruction per CU (2.4 GHz)\n", names[mode],
                   active, ms, ms * 1e-3 * 2.4e9 / winst);
        }
    return 0;
}
