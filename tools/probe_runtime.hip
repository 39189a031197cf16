#include <hip/hip_runtime.h>
extern "C" __global__ void k(float* x){ x[threadIdx.x] = __expf(x[threadIdx.x]); }
extern "C" int launch(float* x, hipStream_t s){ hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, x); return (int)hipGetLastError(); }
