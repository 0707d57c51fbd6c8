// r3dg_tilesort.h -- the per-tile (depth bits, Gaussian id) chunk sort shared by the depth-sort
// kernel (preprocess.hip) and the forward blend's fused sort (render_fwd.hip).
#pragma once

#include <rocprim/block/block_radix_sort.hpp>

#include "r3dg_common.h"

namespace r3dg {

constexpr int kSortBT = 256;  // threads of a tile-sorting workgroup
template <int IPT>
using TileSort = rocprim::block_radix_sort<uint32_t, kSortBT, IPT, uint32_t>;
template <int IPT>
union TileSortLds {
    typename TileSort<IPT>::storage_type sort;
    uint32_t keys[kSortBT * IPT];  // the sorted chunk's keys (tie test)
};

// One chunk of up to kSortBT * IPT (depth bits, Gaussian id) pairs held in the blocked arrangement
// (item t * IPT + k of thread t; the first n are real, pads are all-ones and sort last: visible
// depths < 0x7f800000), sorted by (depth bits, id) -- the reference's stable (tile << 32 | depth)
// sort of its Gaussian-major list breaks depth ties by Gaussian id. A rocPRIM block radix sort by
// depth over only the bits in which the chunk's keys differ (8 bits per pass: a tile's depths
// usually share their top 8 bits, so 3 passes instead of 4); a chunk in which two pairs share
// depth bits (cloned Gaussians do until they move) is sorted again, by id and then stably by
// depth. Called by every thread of the block, after a barrier that ends earlier uses of `lds`.
template <int IPT>
__device__ __forceinline__ void sort_pairs_chunk(uint32_t (&keys)[IPT], uint32_t (&vals)[IPT], int n,
                                                 TileSortLds<IPT>& lds) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    // the bit span in which the real keys differ: OR and AND over the chunk
    uint32_t ko = 0u, ka = 0xffffffffu;
#pragma unroll
    for (int k = 0; k < IPT; ++k)
        if (t * IPT + k < n) { ko |= keys[k]; ka &= keys[k]; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ko |= (uint32_t)__shfl_xor((int)ko, o);
        ka &= (uint32_t)__shfl_xor((int)ka, o);
    }
    if (l == 0) { lds.keys[2 * w] = ko; lds.keys[2 * w + 1] = ka; }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortBT / 64; ++k) { ko |= lds.keys[2 * k]; ka &= lds.keys[2 * k + 1]; }
    const uint32_t diff = ko ^ ka;
    const int b0 = diff ? __builtin_ctz(diff) : 0, b1 = diff ? 32 - __builtin_clz(diff) : 0;
    __syncthreads();  // lds.keys is the sort's storage too
    if (b1 > b0) TileSort<IPT>().sort(keys, vals, lds.sort, b0, b1);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IPT; ++k) lds.keys[t * IPT + k] = keys[k];
    __syncthreads();
    bool tie = false;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const int i = t * IPT + k;
        if (i + 1 < kSortBT * IPT && keys[k] != 0xffffffffu && lds.keys[i + 1] == keys[k]) tie = true;
    }
    if (__syncthreads_or(tie)) {  // block-uniform
        TileSort<IPT>().sort(vals, keys, lds.sort, 0, 32);
        __syncthreads();
        if (b1 > b0) TileSort<IPT>().sort(keys, vals, lds.sort, b0, b1);
    }
}

}  // namespace r3dg
