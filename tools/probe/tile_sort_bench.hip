// tile_sort_bench.hip -- variants of the per-tile depth sort (preprocess.hip tile_depth_sort_kernel)
// on an M1-shaped synthetic input: 8160 tiles of ~614 instances (max < 1024), Gaussian ids
// ascending within each tile, depth keys = float bits of U(3, 8). Median of 20 launches each.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/probe/tile_sort_bench.hip -o /tmp/tsb && /tmp/tsb
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/block/block_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

// MODE 0: load + gather + store only (memory / latency floor)
// MODE 1: rocPRIM block radix sort, bits [0, 32)
// MODE 2: same, bits trimmed to the tile's varying range (block OR/AND reduction first)
// MODE 3: 64-bit (depth << 32 | gid) keys over [0, 52) (what an unordered scatter would need)
template <int BS, int IPT, int MODE, int RB = 0,
          rocprim::block_radix_rank_algorithm ALG = rocprim::block_radix_rank_algorithm::default_for_radix_sort>
__global__ void __launch_bounds__(BS) sort_kernel(int T, const uint2* ranges, const uint32_t* depth_keys,
                                                  uint32_t* plist) {
    using Sort32 = rocprim::block_radix_sort<uint32_t, BS, IPT, uint32_t, 1, 1, RB, ALG>;
    using Sort64 = rocprim::block_radix_sort<uint64_t, BS, IPT>;
    __shared__ union {
        typename Sort32::storage_type s32;
        typename Sort64::storage_type s64;
    } st;
    __shared__ uint32_t s_or, s_and;
    const int tile = blockIdx.x;
    const uint2 rg = ranges[tile];
    const uint32_t s = rg.x, n = rg.y - rg.x;
    if (n <= 1) return;
    const int t = threadIdx.x;
    uint32_t keys[IPT], vals[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t i = (uint32_t)(t * IPT + k);
        const uint32_t g = i < n ? plist[s + i] : 0xffffffffu;
        vals[k] = g;
        keys[k] = i < n ? depth_keys[g] : 0xffffffffu;
    }
    if constexpr (MODE == 1) {
        Sort32().sort(keys, vals, st.s32, 0, 32);
    } else if constexpr (MODE == 2) {
        if (t == 0) { s_or = 0; s_and = 0xffffffffu; }
        __syncthreads();
        uint32_t o = 0, a = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < IPT; ++k)
            if ((uint32_t)(t * IPT + k) < n) { o |= keys[k]; a &= keys[k]; }
        atomicOr(&s_or, o);
        atomicAnd(&s_and, a);
        __syncthreads();
        const uint32_t diff = s_or ^ s_and;
        const int eb = diff ? 32 - __builtin_clz(diff) : 1;
        // pads must sort last: give them the all-ones pattern in the sorted bits
        Sort32().sort(keys, vals, st.s32, 0, eb);
    } else if constexpr (MODE == 3) {
        uint64_t kk[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) kk[k] = ((uint64_t)keys[k] << 32) | vals[k];
        Sort64().sort(kk, st.s64, 0, 52);
#pragma unroll
        for (int k = 0; k < IPT; ++k) vals[k] = (uint32_t)kk[k];
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t i = (uint32_t)(t * IPT + k);
        if (i < n) plist[s + i] = vals[k];
    }
}

template <typename K>
float timeit(const char* name, K kern, int T, const uint2* r, const uint32_t* dk, uint32_t* pl, const uint32_t* pl0,
             size_t L, int bs) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int it = 0; it < 23; ++it) {
        CK(hipMemcpy(pl, pl0, 4 * L, hipMemcpyDeviceToDevice));
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(kern, dim3(T), dim3(bs), 0, 0, T, r, dk, pl);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-40s median %.1f us\n", name, ts[ts.size() / 2] * 1e3);
    return ts[ts.size() / 2];
}

int main() {
    const int T = 8160, P = 1000000;
    std::mt19937 rng(1);
    std::poisson_distribution<int> pc(614);
    std::vector<uint2> ranges(T);
    std::vector<uint32_t> plist;
    for (int t = 0; t < T; ++t) {
        int c = std::min(pc(rng), 1000);
        std::vector<uint32_t> g(c);
        for (auto& x : g) x = rng() % P;
        std::sort(g.begin(), g.end());
        ranges[t] = make_uint2((uint32_t)plist.size(), (uint32_t)(plist.size() + c));
        plist.insert(plist.end(), g.begin(), g.end());
    }
    std::vector<uint32_t> dk(P);
    std::uniform_real_distribution<float> uz(3.f, 8.f);
    for (auto& k : dk) {
        float z = uz(rng);
        memcpy(&k, &z, 4);
    }
    const size_t L = plist.size();
    uint2* dr;
    uint32_t *ddk, *dpl, *dpl0;
    CK(hipMalloc(&dr, 8 * T));
    CK(hipMalloc(&ddk, 4 * P));
    CK(hipMalloc(&dpl, 4 * L));
    CK(hipMalloc(&dpl0, 4 * L));
    CK(hipMemcpy(dr, ranges.data(), 8 * T, hipMemcpyHostToDevice));
    CK(hipMemcpy(ddk, dk.data(), 4 * P, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpl0, plist.data(), 4 * L, hipMemcpyHostToDevice));
    printf("L = %zu\n", L);
    timeit("floor (load+gather+store) 256x4", sort_kernel<256, 4, 0>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("rocprim 32b 256x4", sort_kernel<256, 4, 1>, T, dr, ddk, dpl, dpl0, L, 256);
    std::vector<uint32_t> ref(L);
    CK(hipMemcpy(ref.data(), dpl, 4 * L, hipMemcpyDeviceToHost));
    timeit("rocprim trimmed bits 256x4", sort_kernel<256, 4, 2>, T, dr, ddk, dpl, dpl0, L, 256);
    std::vector<uint32_t> o2(L);
    CK(hipMemcpy(o2.data(), dpl, 4 * L, hipMemcpyDeviceToHost));
    printf("  trimmed == full: %d\n", (int)(o2 == ref));
    timeit("rocprim 32b 512x2", sort_kernel<512, 2, 1>, T, dr, ddk, dpl, dpl0, L, 512);
    timeit("rocprim 32b 128x8", sort_kernel<128, 8, 1>, T, dr, ddk, dpl, dpl0, L, 128);
    timeit("rocprim 32b 1024x1", sort_kernel<1024, 1, 1>, T, dr, ddk, dpl, dpl0, L, 1024);
    using A = rocprim::block_radix_rank_algorithm;
    timeit("match rb4 256x4", sort_kernel<256, 4, 1, 4, A::match>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("match rb6 256x4", sort_kernel<256, 4, 1, 6, A::match>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("match rb8 256x4", sort_kernel<256, 4, 1, 8, A::match>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("match rb11 256x4", sort_kernel<256, 4, 1, 11, A::match>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("basic rb4 256x4", sort_kernel<256, 4, 1, 4, A::basic>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("memoize rb4 256x4", sort_kernel<256, 4, 1, 4, A::basic_memoize>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("memoize rb8 256x4", sort_kernel<256, 4, 1, 8, A::basic_memoize>, T, dr, ddk, dpl, dpl0, L, 256);
    timeit("match rb8 128x8", sort_kernel<128, 8, 1, 8, A::match>, T, dr, ddk, dpl, dpl0, L, 128);
    timeit("match rb11 128x8", sort_kernel<128, 8, 1, 11, A::match>, T, dr, ddk, dpl, dpl0, L, 128);
    timeit("match rb8 64x16", sort_kernel<64, 16, 1, 8, A::match>, T, dr, ddk, dpl, dpl0, L, 64);
    timeit("rocprim 64b(52) 256x4", sort_kernel<256, 4, 3>, T, dr, ddk, dpl, dpl0, L, 256);
    CK(hipMemcpy(o2.data(), dpl, 4 * L, hipMemcpyDeviceToHost));
    printf("  64b == 32b stable: %d\n", (int)(o2 == ref));
    return 0;
}
