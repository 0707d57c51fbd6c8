// preprocess.hip -- per-Gaussian projection, tile binning keys and tile ranges (gfx950).
//
// Restates reference forward.cu:25-267 (preprocessCUDA, computeColorFromSH, computeCov3D,
// computeCov2D), rasterizer_impl.cu:56-140 (checkFrustum, duplicateWithKeys,
// identifyTileRanges). Everything that feeds the tile|depth keys is evaluated as plain IEEE
// ops in a fixed order with FP contraction OFF, matching oracle/r3dg_oracle.c bit for bit, so
// the keys and the sort order are reproducible (SURVEY.md §7 "Bit-exact keys").
#pragma clang fp contract(off)

#include <rocprim/block/block_radix_sort.hpp>

#include "r3dg_common.h"
#include "r3dg_kernels.h"

#ifndef R3DG_SORT_LONG_IPT
#define R3DG_SORT_LONG_IPT 8  // items per thread of the depth sort for tiles longer than 1024 instances
#endif

namespace r3dg {

// forward.cu:25-76.  Writes rgb and the clamp bits.
__device__ static void color_from_sh(int deg, float3 pos, const float* campos, const float* sh, float* rgb,
                                     uint8_t* clamped) {
    float dx = pos.x - campos[0], dy = pos.y - campos[1], dz = pos.z - campos[2];
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    float x = dx / len, y = dy / len, z = dz / len;
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, yz = y * z, xz = x * z;
    uint8_t cl = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float r = SH_C0 * sh[0 * 3 + c];
        if (deg > 0) {
            r = r - SH_C1 * y * sh[1 * 3 + c] + SH_C1 * z * sh[2 * 3 + c] - SH_C1 * x * sh[3 * 3 + c];
            if (deg > 1) {
                r = r + SH_C2_0 * xy * sh[4 * 3 + c] + SH_C2_1 * yz * sh[5 * 3 + c] +
                    SH_C2_2 * (2.0f * zz - xx - yy) * sh[6 * 3 + c] + SH_C2_3 * xz * sh[7 * 3 + c] +
                    SH_C2_4 * (xx - yy) * sh[8 * 3 + c];
                if (deg > 2) {
                    r = r + SH_C3_0 * y * (3.0f * xx - yy) * sh[9 * 3 + c] + SH_C3_1 * xy * z * sh[10 * 3 + c] +
                        SH_C3_2 * y * (4.0f * zz - xx - yy) * sh[11 * 3 + c] +
                        SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3 + c] +
                        SH_C3_4 * x * (4.0f * zz - xx - yy) * sh[13 * 3 + c] +
                        SH_C3_5 * z * (xx - yy) * sh[14 * 3 + c] + SH_C3_6 * x * (xx - 3.0f * yy) * sh[15 * 3 + c];
                }
            }
        }
        r += 0.5f;
        if (r < 0) cl |= (uint8_t)(1u << c);
        rgb[c] = r < 0.0f ? 0.0f : r;
    }
    *clamped = cl;
}

// forward.cu:124-158 (quaternion not normalised; R is the glm column-major matrix read as rows)
__device__ static void compute_cov3d(float3 s_in, float mod, float4 q, float* cov3D) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    float R[3][3];
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y + r * z); R[0][2] = 2.f * (x * z - r * y);
    R[1][0] = 2.f * (x * y - r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z + r * x);
    R[2][0] = 2.f * (x * z + r * y); R[2][1] = 2.f * (y * z - r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
    const float s[3] = {mod * s_in.x, mod * s_in.y, mod * s_in.z};
    float M[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) M[i][j] = s[i] * R[i][j];
    cov3D[0] = M[0][0] * M[0][0] + M[1][0] * M[1][0] + M[2][0] * M[2][0];
    cov3D[1] = M[0][0] * M[0][1] + M[1][0] * M[1][1] + M[2][0] * M[2][1];
    cov3D[2] = M[0][0] * M[0][2] + M[1][0] * M[1][2] + M[2][0] * M[2][2];
    cov3D[3] = M[0][1] * M[0][1] + M[1][1] * M[1][1] + M[2][1] * M[2][1];
    cov3D[4] = M[0][1] * M[0][2] + M[1][1] * M[1][2] + M[2][1] * M[2][2];
    cov3D[5] = M[0][2] * M[0][2] + M[1][2] * M[1][2] + M[2][2] * M[2][2];
}

// forward.cu:79-118: returns (a, b, c) of the low-pass-filtered 2D covariance.
__device__ static float3 compute_cov2d(float3 mean, float fx, float fy, float tanx, float tany, const float* cov3D,
                                       const float* view) {
    float3 t = xform_point4x3(mean, view);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float j00 = fx / t.z, j11 = fy / t.z;
    const float j20 = -(fx * t.x) / (t.z * t.z);
    const float j21 = -(fy * t.y) / (t.z * t.z);
    float g0[3], g1[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        g0[r] = view[4 * r + 0] * j00 + view[4 * r + 2] * j20;
        g1[r] = view[4 * r + 1] * j11 + view[4 * r + 2] * j21;
    }
    const float* c = cov3D;
    float u0 = c[0] * g0[0] + c[1] * g0[1] + c[2] * g0[2];
    float u1 = c[1] * g0[0] + c[3] * g0[1] + c[4] * g0[2];
    float u2 = c[2] * g0[0] + c[4] * g0[1] + c[5] * g0[2];
    float v0 = c[0] * g1[0] + c[1] * g1[1] + c[2] * g1[2];
    float v1 = c[1] * g1[0] + c[3] * g1[1] + c[4] * g1[2];
    float v2 = c[2] * g1[0] + c[4] * g1[1] + c[5] * g1[2];
    return make_float3(g0[0] * u0 + g0[1] * u1 + g0[2] * u2 + 0.3f, g1[0] * u0 + g1[1] * u1 + g1[2] * u2,
                       g1[0] * v0 + g1[1] * v1 + g1[2] * v2 + 0.3f);
}

// forward.cu:161-267 (preprocessCUDA) for one Gaussian. Returns whether it is visible; when it is,
// rec0/rec1/col/depth are the head of its render record (r3dg_kernels.h record_f4).
__device__ static bool preprocess_one(const PreprocessArgs& a, int idx, const float* sh, float4& rec0, float4& rec1,
                                      const float*& col, float& depth) {
    a.radii[idx] = 0;
    a.tiles_touched[idx] = 0;
    a.depth_keys[idx] = 0xffffffffu;
    const float3 p = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    const float3 pv = xform_point4x3(p, a.view);
    if (pv.z <= 0.2f) {  // auxiliary.h:154 (the reference __trap()s when prefiltered; we flag it)
        if (a.prefiltered && a.error_flag) a.error_flag[0] = 1u;  // same value from every writer
        return false;
    }
    const float4 ph = xform_point4x4(p, a.proj);
    const float p_w = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * p_w, ppy = ph.y * p_w;
    const float* cov3D;
    if (a.cov3D_precomp) {
        cov3D = a.cov3D_precomp + 6 * idx;
    } else {
        const float3 s = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
        const float4 q = make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2],
                                     a.rotations[4 * idx + 3]);
        compute_cov3d(s, a.scale_modifier, q, a.cov3D + 6 * idx);
        cov3D = a.cov3D + 6 * idx;
    }
    const float3 cov = compute_cov2d(p, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3D, a.view);
    const float det = cov.x * cov.z - cov.y * cov.y;
    if (det == 0.0f) return false;
    const float det_inv = 1.f / det;
    const float3 conic = make_float3(cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv);
    const float mid = 0.5f * (cov.x + cov.z);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const float px = ndc2pix(ppx, a.W), py = ndc2pix(ppy, a.H);
    int x0, y0, x1, y1;
    get_rect(px, py, (int)my_radius, a.grid_x, a.grid_y, x0, y0, x1, y1);
    if ((x1 - x0) * (y1 - y0) == 0) return false;
    if (!a.colors_precomp) color_from_sh(a.D, p, a.campos, sh, a.rgb + 3 * idx, a.clamped + idx);
    a.depths[idx] = pv.z;
    a.radii[idx] = (int)my_radius;
    a.means2D[idx] = make_float2(px, py);
    rec0 = make_float4(conic.x, conic.y, conic.z, a.opacity[idx]);
    a.conic_opacity[idx] = rec0;
    a.tiles_touched[idx] = (uint32_t)((y1 - y0) * (x1 - x0));
    a.depth_keys[idx] = __float_as_uint(pv.z);
    rec1 = make_float4(px, py, 0.0f, __int_as_float((int)my_radius));  // slot0 set by the duplicate pass
    col = a.colors_precomp ? a.colors_precomp + 3 * idx : a.rgb + 3 * idx;
    depth = pv.z;
    return true;
}

__global__ void __launch_bounds__(256) preprocess_kernel(PreprocessArgs a) {
    // LDS: first the block's SH coefficients (one coalesced copy, odd stride: conflict-free
    // per-thread reads), then the block's render records, assembled here and written out as one
    // contiguous, coalesced span.
    constexpr int SHS = 49;
    __shared__ float4 s_buf4[256 * SHS / 4 + 1];
    float* s_buf = reinterpret_cast<float*>(s_buf4);
    const int t = threadIdx.x;
    const int g0 = blockIdx.x * 256;
    const int idx = g0 + t;
    const int ng = min(256, a.P - g0);
    const int M3 = 3 * a.M;
    const bool use_sh = a.sh && !a.colors_precomp;
    if (use_sh) {
        const float* src = a.sh + (size_t)g0 * M3;
        for (int f = t; f < ng * M3; f += 256) {
            const int gg = f / M3;
            s_buf[gg * SHS + (f - gg * M3)] = src[f];
        }
    }
    __syncthreads();
    float4 rec0, rec1;
    const float* col = nullptr;
    float depth = 0.f;
    const bool vis = idx < a.P && preprocess_one(a, idx, s_buf + t * SHS, rec0, rec1, col, depth);
    if (!a.records) return;
    __syncthreads();  // SH consumed: the buffer now holds the records
    const int RF = 4 * a.rec4;  // floats per record
    if (vis) {
        float* r = s_buf + t * RF;
        reinterpret_cast<float4*>(r)[0] = rec0;
        reinterpret_cast<float4*>(r)[1] = rec1;
        reinterpret_cast<float4*>(r)[2] = make_float4(col[0], col[1], col[2], depth);
    }
    const int S = a.S, padf = RF - 12 - S;  // features at record float 12, then zero padding
    if (S > 0) {
        const float* src = a.features + (size_t)g0 * S;
        for (int f = t; f < ng * S; f += 256) {
            const int gg = f / S;
            s_buf[gg * RF + 12 + (f - gg * S)] = src[f];
        }
    }
    for (int f = t; f < ng * padf; f += 256) {
        const int gg = f / padf;
        s_buf[gg * RF + 12 + S + (f - gg * padf)] = 0.0f;
    }
    __syncthreads();
    float4* dst = a.records + (size_t)g0 * a.rec4;
    for (int f = t; f < ng * a.rec4; f += 256) dst[f] = s_buf4[f];
}

__global__ void __launch_bounds__(256) mark_visible_kernel(int P, const float* __restrict__ means3D,
                                                           const float* __restrict__ view, uint8_t* present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float3 p = make_float3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    present[idx] = xform_point4x3(p, view).z <= 0.2f ? 0 : 1;
}

// duplicateWithKeys (rasterizer_impl.cu:72-113). Block b expands the Gaussians [256b, 256b+256)
// into their tiles, row-major over each rect as the reference, at their Gaussian-major slots
// offsets[g-1] + k: the block's instances are one contiguous slot range, written cooperatively
// (coalesced; output position q finds its Gaussian by binary search over the block's instance
// offsets). The key is the tile alone: a stable sort by tile keeps each tile's instances in
// ascending Gaussian order, and tile_depth_sort_kernel then orders every tile by depth, stably --
// together the reference's stable sort by (tile << 32 | depth bits) over the Gaussian-major list.
// The four backward row flags of each slot (render_bwd.hip) are zeroed on the way.
__global__ void __launch_bounds__(256) duplicate_kernel(int P, const uint32_t* __restrict__ offsets,
                                                        const float2* __restrict__ means2D,
                                                        const int* __restrict__ radii, int grid_x, int grid_y,
                                                        uint32_t* __restrict__ tile_keys, uint32_t* __restrict__ gid_out,
                                                        uint32_t* __restrict__ flags, float4* __restrict__ records,
                                                        int rec4) {
    __shared__ uint32_t s_end[256];  // inclusive end of each Gaussian's instances, block-relative
    __shared__ int s_x0[256], s_y0[256], s_w[256];
    const int t = threadIdx.x;
    const int i0 = blockIdx.x * 256;
    const int n = min(256, P - i0);
    const uint32_t base = i0 == 0 ? 0u : offsets[i0 - 1];
    if (t < n) {
        const int g = i0 + t;
        s_end[t] = offsets[g] - base;
        const int r = radii[g];
        int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
        if (r > 0) {
            const float2 m = means2D[g];
            get_rect(m.x, m.y, r, grid_x, grid_y, x0, y0, x1, y1);
            if (records)  // the Gaussian's first slot, for the backward's rows
                reinterpret_cast<float*>(records + (size_t)g * rec4 + 1)[2] =
                    __uint_as_float(g == 0 ? 0u : offsets[g - 1]);
        }
        s_x0[t] = x0;
        s_y0[t] = y0;
        s_w[t] = max(x1 - x0, 1);
    }
    __syncthreads();
    const uint32_t total = s_end[n - 1];
    for (uint32_t q = t; q < total; q += 256) {
        int lo = 0, hi = n - 1;  // first Gaussian whose end > q
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_end[mid] > q) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t k = q - (lo == 0 ? 0u : s_end[lo - 1]);
        const int w = s_w[lo];
        const int x = s_x0[lo] + (int)(k % (uint32_t)w), y = s_y0[lo] + (int)(k / (uint32_t)w);
        tile_keys[base + q] = (uint32_t)(y * grid_x + x);
        gid_out[base + q] = (uint32_t)(i0 + lo);
        if (flags) flags[base + q] = 0u;
    }
}

// identifyTileRanges (rasterizer_impl.cu:118-140) as one binary search per tile over the sorted
// tile ids: every tile's range is written (empty tiles (0, 0), the reference's memset value), so no
// memset is needed.
__global__ void __launch_bounds__(256) tile_ranges_kernel(int T, int L, const uint32_t* __restrict__ tiles,
                                                          uint2* __restrict__ ranges) {
    const int tile = blockIdx.x * blockDim.x + threadIdx.x;
    if (tile >= T) return;
    auto lower = [&](uint32_t key) {
        int lo = 0, hi = L;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tiles[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return (uint32_t)lo;
    };
    const uint32_t b = lower((uint32_t)tile), e = lower((uint32_t)tile + 1u);
    ranges[tile] = b < e ? make_uint2(b, e) : make_uint2(0u, 0u);  // empty: (0, 0) as the reference's memset
}

// Backward (and depth-sort) launch order, longest tiles first: one workgroup bucket-sorts the
// tiles by instance count (bucket = count / 4, capped; descending). Only the schedule depends on
// this order, so the order within a bucket, which LDS atomics leave unspecified, changes no result.
__global__ void __launch_bounds__(1024) tile_order_kernel(int T, const uint2* __restrict__ ranges,
                                                          uint32_t* __restrict__ order) {
    constexpr int NBK = 1024;
    __shared__ uint32_t hist[NBK];
    __shared__ uint32_t scan[2][NBK];
    const int t = threadIdx.x;
    hist[t] = 0;
    __syncthreads();
    auto bucket = [&](int tile) {
        const uint2 r = ranges[tile];
        return (int)min((r.y - r.x) >> 2, (uint32_t)(NBK - 1));
    };
    for (int i = t; i < T; i += 1024) atomicAdd(&hist[bucket(i)], 1u);
    __syncthreads();
    // exclusive scan in descending bucket order (Hillis-Steele over the reversed histogram)
    const uint32_t v = hist[NBK - 1 - t];
    int cur = 0;
    scan[0][t] = v;
    __syncthreads();
    for (int o = 1; o < NBK; o <<= 1) {
        const uint32_t x = scan[cur][t] + (t >= o ? scan[cur][t - o] : 0u);
        scan[cur ^ 1][t] = x;
        cur ^= 1;
        __syncthreads();
    }
    hist[NBK - 1 - t] = scan[cur][t] - v;  // now the cursor of bucket NBK-1-t
    __syncthreads();
    for (int i = t; i < T; i += 1024) order[atomicAdd(&hist[bucket(i)], 1u)] = (uint32_t)i;
}

// The depth half of the reference's (tile << 32 | depth bits) sort: every tile's instances,
// ascending Gaussian ids after the stable tile sort, sorted stably by the Gaussians' depth bits
// (the reference's order: depth, ties by Gaussian id). One workgroup per tile, longest tiles
// first. A chunk of the tile is sorted in registers / LDS (rocPRIM block radix sort, 4 passes of
// 8 bits) -- 1024-instance chunks for tiles of up to 1024 instances, 2048-instance chunks for
// longer ones (both sorters share one LDS union: 16 KB, still 8 waves/SIMD); a tile longer than
// one chunk sorts each chunk into a run and merges run pairs (stable merge path) through the
// scratch buffers, ping-pong, landing in point_list.
constexpr int kSortBT = 256;
using TileDepthSort4 = rocprim::block_radix_sort<uint32_t, kSortBT, 4, uint32_t>;
using TileDepthSortL = rocprim::block_radix_sort<uint32_t, kSortBT, R3DG_SORT_LONG_IPT, uint32_t>;
union TileDepthSortStorage {
    typename TileDepthSort4::storage_type s4;
    typename TileDepthSortL::storage_type sl;
};

__device__ __forceinline__ uint32_t nt_load(const uint32_t* p) { return __builtin_nontemporal_load(p); }

// chunks of kSortBT * IPT instances of the tile [s, s + n) sorted into runs at (rk, rv)
template <int IPT, class Sort, class Storage>
__device__ __forceinline__ void sort_tile_chunks(uint32_t s, uint32_t n, uint32_t nchunks, const uint32_t* depth_keys,
                                                 const uint32_t* point_list, uint32_t* rk, uint32_t* rv,
                                                 Storage& storage) {
    constexpr uint32_t kChunk = kSortBT * IPT;
    const int t = threadIdx.x;
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t c0 = c * kChunk;
        uint32_t keys[IPT], vals[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {  // blocked arrangement: item index = t * IPT + k
            const uint32_t i = c0 + (uint32_t)(t * IPT + k);
            const uint32_t g = i < n ? point_list[s + i] : 0xffffffffu;
            vals[k] = g;
            keys[k] = i < n ? depth_keys[g] : 0xffffffffu;  // visible depths < 0x7f800000: pads sort last
        }
        if (c > 0) __syncthreads();  // storage reuse
        Sort().sort(keys, vals, storage, 0, 32);
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t i = c0 + (uint32_t)(t * IPT + k);
            if (i < n) {
                if (nchunks > 1) rk[s + i] = keys[k];
                rv[s + i] = vals[k];
            }
        }
    }
}

__global__ void __launch_bounds__(kSortBT) __attribute__((amdgpu_waves_per_eu(8))) tile_depth_sort_kernel(int T, const uint2* __restrict__ ranges,
                                                                  const uint32_t* __restrict__ order,
                                                                  const uint32_t* __restrict__ depth_keys,
                                                                  uint32_t* __restrict__ point_list, uint32_t* kA,
                                                                  uint32_t* vA, uint32_t* kB) {
    __shared__ TileDepthSortStorage storage;
    const int b = blockIdx.x;
    if (b >= T) return;
    const int tile = order ? (int)order[b] : b;
    const uint2 rg = ranges[tile];
    const uint32_t s = rg.x, n = rg.y - rg.x;
    if (n <= 1) return;
    const int t = threadIdx.x;
    // sorter capacity by tile length (block-uniform); a 2-item sorter for tiles of up to 512
    // instances measured no faster (M1: 0.086 vs 0.083 ms, it spills one VGPR)
    const uint32_t kChunk = n <= kSortBT * 4 ? kSortBT * 4 : kSortBT * R3DG_SORT_LONG_IPT;
    const uint32_t nchunks = (n + kChunk - 1) / kChunk;
    int rounds = 0;
    while ((1u << rounds) < nchunks) ++rounds;
    // runs go where an even number of merge rounds leaves the result in (kB, point_list)
    uint32_t* rk = (rounds & 1) ? kA : kB;
    uint32_t* rv = (rounds & 1) ? vA : point_list;
    if (kChunk == kSortBT * 4) sort_tile_chunks<4, TileDepthSort4>(s, n, nchunks, depth_keys, point_list, rk, rv, storage.s4);
    else sort_tile_chunks<R3DG_SORT_LONG_IPT, TileDepthSortL>(s, n, nchunks, depth_keys, point_list, rk, rv, storage.sl);
    if (nchunks == 1) return;
    __syncthreads();
    uint32_t *sk = rk, *sv = rv, *dk = (rk == kA) ? kB : kA, *dv = (rk == kA) ? point_list : vA;
    for (uint32_t w = kChunk; w < n; w *= 2) {
        for (uint32_t a0 = 0; a0 < n; a0 += 2 * w) {
            const uint32_t a1 = min(a0 + w, n), b1 = min(a0 + 2 * w, n);
            const uint32_t la = a1 - a0, lb = b1 - a1, tot = b1 - a0;
            const uint32_t per = (tot + kSortBT - 1) / kSortBT;
            const uint32_t d0 = min((uint32_t)t * per, tot), d1 = min(d0 + per, tot);
            if (d0 >= d1) continue;
            const uint32_t* A = sk + s + a0;
            const uint32_t* B = sk + s + a1;
            // merge path: i = number of A items among the first d0 outputs (ties: A first)
            uint32_t lo = d0 > lb ? d0 - lb : 0u, hi = min(d0, la);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (nt_load(A + mid) <= nt_load(B + (d0 - 1 - mid))) lo = mid + 1;
                else hi = mid;
            }
            uint32_t i = lo, j = d0 - lo;
            uint32_t ka = i < la ? nt_load(A + i) : 0xffffffffu, kb = j < lb ? nt_load(B + j) : 0xffffffffu;
            for (uint32_t d = d0; d < d1; ++d) {
                const bool takeA = j >= lb || (i < la && ka <= kb);
                if (takeA) {
                    dk[s + a0 + d] = ka;
                    dv[s + a0 + d] = nt_load(sv + s + a0 + i);
                    ++i;
                    ka = i < la ? nt_load(A + i) : 0xffffffffu;
                } else {
                    dk[s + a0 + d] = kb;
                    dv[s + a0 + d] = nt_load(sv + s + a1 + j);
                    ++j;
                    kb = j < lb ? nt_load(B + j) : 0xffffffffu;
                }
            }
        }
        __syncthreads();
        uint32_t* tk = sk; sk = dk; dk = tk;
        uint32_t* tv = sv; sv = dv; dv = tv;
    }
}

hipError_t launch_tile_depth_sort(int T, const uint2* ranges, const uint32_t* order, const uint32_t* depth_keys,
                                  uint32_t* point_list, uint32_t* kA, uint32_t* vA, uint32_t* kB, hipStream_t st) {
    hipLaunchKernelGGL(tile_depth_sort_kernel, dim3(T), dim3(kSortBT), 0, st, T, ranges, order, depth_keys, point_list,
                       kA, vA, kB);
    return hipGetLastError();
}

}  // namespace r3dg
