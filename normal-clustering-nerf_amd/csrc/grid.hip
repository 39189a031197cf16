// Occupancy-grid refresh for gfx950: NGPMT.update_density_grid (ngp_mt.py:340-368) with its cell
// sampling sample_uniform_and_occupied_cells (ngp_mt.py:245-262), as five device passes with no
// host round trip (the reference runs ~50 torch ops, a nonzero() and a .item() sync):
//
//   grid_occ   : count of cells > threshold in the cascade -> hit probability of an occupied draw
//   grid_select: one thread per cell (Morton order = the cell index): hit test, decay of the cells
//                that are not hit, wave-aggregated append of the hit cells' jittered positions
//   (ncn_field_fwd density mode over the appended list, device count)
//   grid_apply : max(decay * grid, sigma) of the hit cells (the torch.where / torch.maximum update)
//   grid_mean + grid_pack: mean of the positive cells -> min(mean, threshold) -> packbits
//
// Sampling (documented deviation): the reference draws M = G^3/4 uniform cells and M
// cells from the occupied list, with replacement, and scatters the densities (duplicates: one of
// the writes survives).  What the update sees is the SET of cells hit; here every cell is hit
// independently with the same marginal probability, 1 - (1 - 1/N)^M for the uniform draws and
// 1 - (1 - 1/n_occ)^M for the occupied ones (N = G^3 cells, n_occ occupied).  The hit list is then
// produced in Morton order, so the hash-grid gathers of the density pass are spatially coherent
// (the reference's random order makes every gather a separate cache line).  Random numbers come
// from a counter-based hash of (seed, cascade, cell, stream): the refreshed grid is a
// deterministic function of the seed, independent of scheduling.
#pragma clang fp contract(off)

#include <algorithm>
#include "common.h"
#include "../../include/ncnerf.h"

namespace ncn {

constexpr int GR_BLOCKS = 256;   // workgroups of the two grid-wide reductions (one partial per thread of the last)
constexpr int GR_UNROLL = 8;   // float4 loads in flight per thread in the reductions
constexpr int GS_ITER = 8;       // grid_select: cells per thread (2048 per workgroup, one Morton block)

// Workspace (ncn_grid_work_bytes): per-workgroup partials, the arrival counter (left zero by every
// call), and the per-call scalars.
struct GridWork {
    double psum[GR_BLOCKS];
    unsigned long long pcnt[GR_BLOCKS];
    unsigned arrive;
    float p_occ;
    float pad[2];
};

__device__ __forceinline__ uint32_t gr_compact3(uint32_t x) {  // morton3D_invert, raymarching.cu:52-60
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

// 32-bit counter-based hash of (seed, cell, stream) (murmur3 finaliser over a seed-keyed mix:
// 32-bit multiplies only) -> uniform in [0, 1) with 24 random bits
__device__ __forceinline__ float gr_uniform(uint64_t seed, uint32_t cell, uint32_t stream) {
    uint32_t h = (uint32_t)seed ^ (cell * 0x9E3779B1u + stream * 0x85EBCA77u);
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    h += (uint32_t)(seed >> 32);
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// torch.maximum: NaN if either operand is NaN
__device__ __forceinline__ float torch_max(float a, float b) {
    if (a != a || b != b) return __int_as_float(0x7fc00000);
    return a > b ? a : b;
}

// Per-cell decay: `decay`, or with erode clamp(decay ** (1 / count_grid), 0.1, 0.95) (ngp_mt.py:356-357)
__device__ __forceinline__ float cell_decay(float decay, const float* __restrict__ count, uint32_t i) {
    if (!count) return decay;
    return fminf(fmaxf(powf(decay, 1.0f / count[i]), 0.1f), 0.95f);
}

// Agent-scope hand-off of per-workgroup partials to the last workgroup to arrive
// (MI355X_MICROARCH.md, inter-workgroup visibility): store, wait, one arrival add.
template <typename T>
__device__ __forceinline__ bool gr_arrive(T* slot, T v, unsigned* arrive) {
    __shared__ bool last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    return last;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)v, off, 64), hi = __shfl_xor((unsigned)(v >> 32), off, 64);
        v += ((unsigned long long)hi << 32) | lo;
    }
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Sum of the gridDim.x (<= 256) published partials by the 256 threads of the last workgroup: one
// agent-scope load per thread (a single round trip), wave sums, then 4 values through LDS.
template <typename T>
__device__ __forceinline__ T gr_final_sum(const T* part, T (*wsum)(T)) {
    __shared__ T red[4];
    T v = threadIdx.x < gridDim.x ? __hip_atomic_load(&part[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : (T)0;
    v = wsum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// 1. cells of the cascade with density > threshold (`torch.nonzero(grid[c] > thr)`, ngp_mt.py:256)
//    -> p_occ = 1 - (1 - 1/n_occ)^M (0 when none: the reference then draws no occupied cell);
//    the last workgroup also zeroes the hit-list count for grid_select.
__global__ __launch_bounds__(256) void grid_occ_kernel(const float* __restrict__ grid, int64_t n, float thr,
                                                       int64_t M, GridWork* __restrict__ w,
                                                       int32_t* __restrict__ n_list) {
    __shared__ unsigned long long red[4];
    unsigned long long c = 0;
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;  // n % 4 == 0 (checked on the host)
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n4; b += GR_UNROLL * stride) {
        float4 x[GR_UNROLL];  // GR_UNROLL loads in flight per thread
#pragma unroll
        for (int u = 0; u < GR_UNROLL; u++) x[u] = b + u * stride < n4 ? ((const float4*)grid)[b + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < GR_UNROLL; u++)
            c += (x[u].x > thr) + (x[u].y > thr) + (x[u].z > thr) + (x[u].w > thr);
    }
    c = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (!gr_arrive(&w->pcnt[blockIdx.x], red[0] + red[1] + red[2] + red[3], &w->arrive)) return;
    const unsigned long long t = gr_final_sum<unsigned long long>(w->pcnt, wave_sum_u64);
    if (threadIdx.x == 0) {
        const double p = t > 0 ? -expm1((double)M * log1p(-1.0 / (double)t)) : 0.0;
        w->p_occ = (float)p;
        *n_list = 0;
        w->arrive = 0;
    }
}

// 2. cells (index = Morton code of the coordinates, ngp_mt.py:255/260) in blocks of 2048 per
//    workgroup, 8 per thread.  Pass 1: hit test; cells not hit take the update with
//    density_grid_tmp = 0 (ngp_mt.py:323-324) right here; per (round, wave) hit counts to LDS.  One
//    atomic per workgroup reserves its slice of the hit list; pass 2 appends the hit cells' jittered
//    positions (ngp_mt.py:318-319) in Morton order within the block.
__global__ __launch_bounds__(256) void grid_select_kernel(float* __restrict__ grid, int64_t n, int G, float s_hg,
                                                          float hg, float thr, float p_u, int warmup, uint64_t seed,
                                                          float decay, const float* __restrict__ count,
                                                          const GridWork* __restrict__ w, float* __restrict__ xyzs,
                                                          int32_t* __restrict__ list_idx,
                                                          int32_t* __restrict__ n_list) {
    __shared__ int cnt[GS_ITER][4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t b0 = (int64_t)blockIdx.x * (256 * GS_ITER);
    const float p_o = warmup ? 1.0f : w->p_occ;
    float v[GS_ITER];
#pragma unroll
    for (int k = 0; k < GS_ITER; k++) {
        const int64_t i = b0 + k * 256 + threadIdx.x;
        v[k] = i < n ? grid[i] : 0.f;
    }
    uint32_t hits = 0;
#pragma unroll
    for (int k = 0; k < GS_ITER; k++) {
        const int64_t i = b0 + k * 256 + threadIdx.x;
        const uint32_t cell = (uint32_t)i;
        bool hit = i < n;
        if (hit && !warmup) hit = gr_uniform(seed, cell, 0) < p_u || (v[k] > thr && gr_uniform(seed, cell, 1) < p_o);
        if (i < n && !hit) grid[i] = v[k] < 0.f ? v[k] : torch_max(v[k] * cell_decay(decay, count, cell), 0.f);
        hits |= (uint32_t)hit << k;
        const uint64_t m = __ballot(hit);
        if (lane == 0) cnt[k][wv] = (int)__popcll(m);
    }
    __syncthreads();
    static_assert(GS_ITER * 4 <= 64, "one count per lane");
    if (threadIdx.x < 64) {  // exclusive scan of the GS_ITER*4 counts in (round, wave) order, one per lane
        const int c0 = lane < GS_ITER * 4 ? (&cnt[0][0])[lane] : 0;
        const int incl = wave_incl_sum_i(c0, lane);
        const int total = __shfl(incl, 63, 64);
        int base = 0;
        if (lane == 63 && total > 0) base = atomicAdd(n_list, total);
        base = __shfl(base, 63, 64);
        if (lane < GS_ITER * 4) (&cnt[0][0])[lane] = base + incl - c0;
    }
    __syncthreads();
    if (!hits) return;
    const uint64_t lt = (1ull << lane) - 1ull;
    const float gm1 = (float)(G - 1);
#pragma unroll
    for (int k = 0; k < GS_ITER; k++) {
        const bool hit = (hits >> k) & 1u;
        const uint64_t m = __ballot(hit);
        if (!hit) continue;
        const int pos = cnt[k][wv] + (int)__popcll(m & lt);
        const uint32_t cell = (uint32_t)(b0 + k * 256 + threadIdx.x);
        list_idx[pos] = (int32_t)cell;
        // (coords / (G-1) * 2 - 1) * (s - half_grid) + (rand * 2 - 1) * half_grid, in f32 as torch does
        const uint32_t c3[3] = {gr_compact3(cell), gr_compact3(cell >> 1), gr_compact3(cell >> 2)};
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float u = gr_uniform(seed, cell, 2 + q);
            float x = (float)c3[q] / gm1;
            x = x * 2.0f - 1.0f;
            x = x * s_hg;
            x = x + (u * 2.0f - 1.0f) * hg;
            xyzs[3 * (int64_t)pos + q] = x;
        }
    }
}

// 3. hit cells: grid = where(grid < 0, grid, max(grid * decay, sigma)) (ngp_mt.py:320-324)
__global__ __launch_bounds__(256) void grid_apply_kernel(float* __restrict__ grid, const int32_t* __restrict__ list_idx,
                                                         const float* __restrict__ sigmas,
                                                         const int32_t* __restrict__ n_list, int64_t cap, float decay,
                                                         const float* __restrict__ count) {
    const int64_t n = min((int64_t)*n_list, cap);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint32_t cell = (uint32_t)list_idx[i];
        const float v = grid[cell];
        grid[cell] = v < 0.f ? v : torch_max(v * cell_decay(decay, count, cell), sigmas[i]);
    }
}

// 4. mean of the positive cells (ngp_mt.py:365) -> threshold = min(mean, thr) (NaN when no cell is
//    positive: quirk q12, the bitfield is then cleared); partial sums in f64, summed in a fixed order.
__global__ __launch_bounds__(256) void grid_mean_kernel(const float* __restrict__ grid, int64_t n, double thr,
                                                        GridWork* __restrict__ w, float* __restrict__ thr_out) {
    __shared__ double rs[4];
    __shared__ unsigned long long rc[4];
    double s = 0.0;
    unsigned long long c = 0;
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;  // n % 8 == 0 (checked on the host)
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n4; b += GR_UNROLL * stride) {
        float4 x[GR_UNROLL];
#pragma unroll
        for (int u = 0; u < GR_UNROLL; u++) x[u] = b + u * stride < n4 ? ((const float4*)grid)[b + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < GR_UNROLL; u++) {
            const float e[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (e[q] > 0.f) { s += (double)e[q]; c++; }
        }
    }
    s = wave_sum_f64(s);
    c = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = s; rc[threadIdx.x >> 6] = c; }
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(&w->psum[blockIdx.x], rs[0] + rs[1] + rs[2] + rs[3], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (!gr_arrive(&w->pcnt[blockIdx.x], rc[0] + rc[1] + rc[2] + rc[3], &w->arrive)) return;
    const double ts = gr_final_sum<double>(w->psum, wave_sum_f64);
    const unsigned long long tc = gr_final_sum<unsigned long long>(w->pcnt, wave_sum_u64);
    {
        if (threadIdx.x == 0) {
            const float mean = tc > 0 ? (float)(ts / (double)tc) : __int_as_float(0x7fc00000);
            *thr_out = thr < (double)mean ? (float)thr : mean;  // Python min(mean, thr)
            w->arrive = 0;
        }
    }
}

// 5. packbits (raymarching.cu:133-161) against the device threshold
__global__ __launch_bounds__(256) void grid_pack_kernel(const float4* __restrict__ grid, int64_t n_bytes,
                                                        const float* __restrict__ thr_dev,
                                                        uint8_t* __restrict__ bitfield) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= n_bytes) return;
    const float thr = *thr_dev;
    const float4 lo = grid[2 * b], hi = grid[2 * b + 1];
    const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) bits |= (v[k] > thr) ? (1u << k) : 0u;
    bitfield[b] = (uint8_t)bits;
}

}  // namespace ncn

using namespace ncn;

extern "C" {

int64_t ncn_grid_work_bytes(void) { return (int64_t)sizeof(GridWork); }

int ncn_grid_sample(float* density_grid_c, int64_t n_cells, int grid_size, float s_minus_half_grid,
                    float half_grid, float threshold, int64_t M, int warmup, uint64_t seed, float decay,
                    const float* count_grid_c, float* list_xyzs, int32_t* list_idx, int32_t* n_list, void* work,
                    void* stream) {
    if (n_cells <= 0) return 0;
    NCN_REQUIRE(n_cells < (1ll << 31) && n_cells % 4 == 0 && grid_size > 1 && ((uintptr_t)density_grid_c & 15) == 0,
                hipErrorInvalidValue,
                "ncn_grid_sample: n_cells=%lld (multiple of 4, 16-B aligned grid) grid_size=%d", (long long)n_cells, grid_size);
    NCN_REQUIRE(work != nullptr && n_list != nullptr, hipErrorInvalidValue, "ncn_grid_sample: work / n_list required");
    hipStream_t s = (hipStream_t)stream;
    GridWork* w = (GridWork*)work;
    const int occ_blocks = (int)std::min<int64_t>(GR_BLOCKS, cdiv(n_cells, 4 * 256 * GR_UNROLL));
    hipLaunchKernelGGL(grid_occ_kernel, dim3(occ_blocks), dim3(256), 0, s, density_grid_c, n_cells, threshold, M, w,
                       n_list);
    NCN_LAUNCH_CHECK("ncn_grid_sample(occ)");
    const double N = (double)n_cells;
    const float p_u = (float)(-expm1((double)M * log1p(-1.0 / N)));
    hipLaunchKernelGGL(grid_select_kernel, dim3(cdiv(n_cells, 256 * GS_ITER)), dim3(256), 0, s, density_grid_c, n_cells, grid_size,
                       s_minus_half_grid, half_grid, threshold, p_u, warmup, seed, decay, count_grid_c, w, list_xyzs,
                       list_idx, n_list);
    NCN_LAUNCH_CHECK("ncn_grid_sample(select)");
    return 0;
}

int ncn_grid_apply(float* density_grid_c, const int32_t* list_idx, const float* sigmas, const int32_t* n_list,
                   int64_t capacity, float decay, const float* count_grid_c, void* stream) {
    if (capacity <= 0) return 0;
    const int blocks = (int)std::min<int64_t>(2048, cdiv(capacity, 256));
    hipLaunchKernelGGL(grid_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, density_grid_c, list_idx,
                       sigmas, n_list, capacity, decay, count_grid_c);
    NCN_LAUNCH_CHECK("ncn_grid_apply");
    return 0;
}

int ncn_grid_packbits(const float* density_grid, int64_t n_total, double threshold, uint8_t* bitfield,
                      float* thr_out, void* work, void* stream) {
    if (n_total <= 0) return 0;
    NCN_REQUIRE(n_total % 8 == 0 && ((uintptr_t)density_grid & 15) == 0, hipErrorInvalidValue,
                "ncn_grid_packbits: n_total must be a multiple of 8 and the grid 16-byte aligned");
    NCN_REQUIRE(work != nullptr && thr_out != nullptr, hipErrorInvalidValue, "ncn_grid_packbits: work / thr_out required");
    hipStream_t s = (hipStream_t)stream;
    const int blocks = (int)std::min<int64_t>(GR_BLOCKS, cdiv(n_total, 4 * 256 * GR_UNROLL));
    hipLaunchKernelGGL(grid_mean_kernel, dim3(blocks), dim3(256), 0, s, density_grid, n_total, threshold,
                       (GridWork*)work, thr_out);
    NCN_LAUNCH_CHECK("ncn_grid_packbits(mean)");
    const int64_t n_bytes = n_total / 8;
    hipLaunchKernelGGL(grid_pack_kernel, dim3(cdiv(n_bytes, 256)), dim3(256), 0, s, (const float4*)density_grid,
                       n_bytes, thr_out, bitfield);
    NCN_LAUNCH_CHECK("ncn_grid_packbits(pack)");
    return 0;
}

}  // extern "C"
