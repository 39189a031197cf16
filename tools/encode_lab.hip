// Diagnostic lab (not product code): the hash-grid encoding LEVEL-MAJOR — one launch whose
// workgroups take (level pair, block of samples) with the level pair outer, so the gathers in flight
// at any time hit one or two levels' tables (<= 4 MB each: L2-resident per XCD) instead of all 16
// (45.8 MB: Infinity-Cache traffic).  Writes the forward's enc_cache layout (fp16 fragments: lane
// (g, r) of a 16-sample group holds levels {2g, 2g+1 | 8+2g, 9+2g} of sample r), so its output is
// compared bit for bit with the product forward's cache by tools/encode_lab.py.
#include "../normal-clustering-nerf_amd/csrc/field.hip"

namespace lab {
using namespace ncn;

template <int SPT>  // samples per thread
__global__ __launch_bounds__(256) void encode_levels_kernel(const float* __restrict__ xyzs, int64_t n,
                                                            const float2* __restrict__ table, LevelTable Lt,
                                                            float xyz_min, float xyz_extent, int nbp,
                                                            _Float16* __restrict__ enc) {
    __shared__ LevelTable L;
    load_levels(L, Lt);
    __syncthreads();
    const int pair = blockIdx.x / nbp, blk = blockIdx.x % nbp;  // level pair outer
    const int l0 = 2 * pair;                                     // levels l0, l0 + 1
    const int g = pair & 3, half = pair >> 2;                     // fragment slot of this pair
#pragma unroll
    for (int u = 0; u < SPT; u++) {
        const int64_t s = ((int64_t)blk * SPT + u) * 256 + threadIdx.x;
        if (s >= n) break;
        const float x = (xyzs[3 * s] - xyz_min) / xyz_extent;
        const float y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
        const float z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
        const float2 a = encode_level(table, L, l0, x, y, z);
        const float2 b = encode_level(table, L, l0 + 1, x, y, z);
        const int64_t grp = s >> 4;
        const int lane = g * 16 + (int)(s & 15);
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *(h4*)(enc + (grp * 64 + lane) * 8 + half * 4) = h4{(_Float16)a.x, (_Float16)a.y, (_Float16)b.x, (_Float16)b.y};
    }
}
// XCD-partitioned: block b runs on XCD b % 8 (dispatch round-robin; a performance hint only), and
// XCD x encodes levels x and x + 8 for all points, so each L2 holds at most two levels' tables.
__global__ __launch_bounds__(256) void encode_xcd_kernel(const float* __restrict__ xyzs, int64_t n,
                                                         const float2* __restrict__ table, LevelTable Lt,
                                                         float xyz_min, float xyz_extent, int nb,
                                                         _Float16* __restrict__ enc) {
    __shared__ LevelTable L;
    load_levels(L, Lt);
    __syncthreads();
    const int x8 = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int l = j < nb ? x8 : x8 + 8, blk = j < nb ? j : j - nb;
    const int64_t s = (int64_t)blk * 256 + threadIdx.x;
    if (s >= n) return;
    const float x = (xyzs[3 * s] - xyz_min) / xyz_extent;
    const float y = (xyzs[3 * s + 1] - xyz_min) / xyz_extent;
    const float z = (xyzs[3 * s + 2] - xyz_min) / xyz_extent;
    const float2 a = encode_level(table, L, l, x, y, z);
    const int g = (l & 7) >> 1, half = l >> 3, sub = l & 1;
    const int64_t grp = s >> 4;
    const int lane = g * 16 + (int)(s & 15);
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    *(h2*)(enc + (grp * 64 + lane) * 8 + half * 4 + sub * 2) = h2{(_Float16)a.x, (_Float16)a.y};
}
}  // namespace lab

extern "C" int lab_encode_levels(const float* xyzs, int64_t n, const float* table, const uint32_t* levels,
                                 float xyz_min, float xyz_extent, int spt, void* enc, void* stream) {
    const ncn::LevelTable Lt = ncn::make_table(levels);
    const int per = 256 * (spt > 0 ? spt : 1);
    const int nbp = (int)((n + per - 1) / per);
    if (spt == 0) {
        const int nb = (int)((n + 255) / 256);
        hipLaunchKernelGGL(lab::encode_xcd_kernel, dim3(16 * nb), dim3(256), 0, (hipStream_t)stream, xyzs, n,
                           (const float2*)table, Lt, xyz_min, xyz_extent, nb, (_Float16*)enc);
    } else if (spt == 1)
        hipLaunchKernelGGL(lab::encode_levels_kernel<1>, dim3(8 * nbp), dim3(256), 0, (hipStream_t)stream, xyzs, n,
                           (const float2*)table, Lt, xyz_min, xyz_extent, nbp, (_Float16*)enc);
    else
        hipLaunchKernelGGL(lab::encode_levels_kernel<4>, dim3(8 * nbp), dim3(256), 0, (hipStream_t)stream, xyzs, n,
                           (const float2*)table, Lt, xyz_min, xyz_extent, nbp, (_Float16*)enc);
    return (int)hipGetLastError();
}
