// Diagnostic: launch cost of an empty 2048 x 256 grid, timed like the probes (HIP events).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void empty_k(float* p) { if (p && threadIdx.x == 1234) p[0] = 1.f; }
int main() {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int blocks : {1, 256, 2048, 8192}) {
        hipLaunchKernelGGL(empty_k, dim3(blocks), dim3(256), 0, 0, nullptr);
        (void)hipDeviceSynchronize();
        float tot = 0.f;
        for (int i = 0; i < 50; i++) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(empty_k, dim3(blocks), dim3(256), 0, 0, nullptr);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b); tot += ms;
        }
        printf("empty kernel %5d x 256: %.2f us (event-timed)\n", blocks, tot / 50 * 1e3);
    }
}
