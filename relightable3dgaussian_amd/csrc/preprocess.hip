// preprocess.hip -- per-Gaussian projection, tile binning keys and tile ranges (gfx950).
//
// Restates reference forward.cu:25-267 (preprocessCUDA, computeColorFromSH, computeCov3D,
// computeCov2D), rasterizer_impl.cu:56-140 (checkFrustum, duplicateWithKeys,
// identifyTileRanges). Everything that feeds the tile|depth keys is evaluated as plain IEEE
// ops in a fixed order with FP contraction OFF, matching oracle/r3dg_oracle.c bit for bit, so
// the keys and the sort order are reproducible (SURVEY.md §7 "Bit-exact keys").
#pragma clang fp contract(off)

#include "r3dg_common.h"
#include "r3dg_kernels.h"
#include "r3dg_tilesort.h"

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
    rec1 = make_float4(px, py, 0.0f, __int_as_float((int)my_radius));
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
    // the per-tile counters of the atomic binning (bin_atomic_kernel) start at zero
    if (a.tile_count)
        for (int i = idx; i < a.num_tiles; i += (int)(gridDim.x * 256)) a.tile_count[i] = 0u;
    // the single-pass scan's status words and ticket (rasterizer.hip scan_touched_kernel) start at zero
    if (a.scan_status)
        for (int i = idx; i < a.scan_words; i += (int)(gridDim.x * 256)) a.scan_status[i] = 0ull;
    if (a.work_hist)
        for (int i = idx; i < kWorkBuckets; i += (int)(gridDim.x * 256)) a.work_hist[i] = 0u;
    if (use_sh) {
        const float* src = a.sh + (size_t)g0 * M3;
        // (a plain division here: the multiply-high of gather_bwd_kernel measured 2-5 % slower in
        // this kernel)
        block_load4<256>(src, ng * M3, t, [&](int f, float v) {
            const int gg = f / M3;
            s_buf[gg * SHS + (f - gg * M3)] = v;
        });
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
        // the blends' staged conic is (-a/2, -b, -c/2): exact (powers of two), so gauss_power is
        // dx (A dx + B dy) + C dy^2 (r3dg_common.h) and the cull recovers (a, b, c) exactly
        reinterpret_cast<float4*>(r)[0] = make_float4(-0.5f * rec0.x, -rec0.y, -0.5f * rec0.z, rec0.w);
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

// Binning: duplicateWithKeys + SortPairs + identifyTileRanges (rasterizer_impl.cu:72-140, 343-383).
// The reference writes one (tile << 32 | depth) key per instance in Gaussian-major slot order and
// radix-sorts all L of them (45 bits, stable). Its result is every tile's instances ordered by
// (depth bits, Gaussian id): a stable sort of a Gaussian-major list breaks depth ties by Gaussian.
// Here the tile grouping is a counting sort with no order inside a tile, and
// tile_depth_sort_kernel then orders every tile by (depth bits, Gaussian id):
//   1. bin_count_kernel: workgroup b (one per CU) counts the instances of its Gaussian range per
//      tile with LDS counters and writes its row hist[b, :];
//   2. bin_colscan_kernel: per-tile totals and, in place, each workgroup's offset inside its tiles
//      (column prefix sums of hist);
//   3. tile_ranges_kernel: exclusive scan of the totals -> ranges (the reference's (0, 0) for
//      empty tiles) and each tile's first position;
//   4. bin_scatter_kernel: every instance takes the next position of its (workgroup, tile) from
//      an LDS counter and writes (depth bits, Gaussian id) there -- one 8-byte store, and the
//      depth sort reads its keys coalesced instead of gathering them per instance (also zeroes
//      row flags when given them; the rows reduction reads each Gaussian's first slot from the
//      scan, offsets[g - 1], not from a record store here: 1 M scattered 4-byte stores fewer);
//      one extra workgroup of its grid computes the longest-first tile order meanwhile.
// No global atomics: they execute at the memory side (MI355X_MICROARCH.md "Global float
// atomics"), one 64-B request per scattered lane -- a first version with one per instance took
// 0.18 ms per pass at M1. Steps 1-3 need only the scan of tiles touched, so they run while the
// host reads num_rendered back and allocates the binning state. Workgroups enumerate their
// instances load-balanced, kBinSub Gaussians at a time: slot q finds its Gaussian by binary search
// over the staged instance offsets, and its tile is the row-major index of q - the Gaussian's first
// slot in its rect (duplicateWithKeys' order). Above kBinMaxTiles tiles the LDS counters do not
// fit and bin_atomic_kernel takes one global atomic per instance instead (same result).

// The instances of Gaussians [g0, g0 + n), n <= kBinSub, staged in LDS: visit(tile, g, key) once per
// instance (key: the Gaussian's depth bits, scatter passes only). Every thread takes a contiguous run of the range's slots: one binary search for the
// run's first Gaussian, then the rect walked row-major (duplicateWithKeys' order) -- the search's
// dependent LDS reads are paid once per run, not once per instance. Scatter passes also zero the
// backward's row flags of the range's slots (coalesced).
template <class Visit>
__device__ __forceinline__ void bin_enumerate(const BinArgs& a, int g0, int n, uint32_t* s_end, int* s_x0, int* s_y0,
                                              int* s_w, bool scatter, Visit visit) {
    const int t = threadIdx.x, nt = blockDim.x;
    const uint32_t base = g0 == 0 ? 0u : a.offsets[g0 - 1];
    __syncthreads();  // the previous range's enumeration is done with the staging arrays
    for (int i = t; i < n; i += nt) {
        const int g = g0 + i;
        s_end[i] = a.offsets[g] - base;
        const int r = a.radii[g];
        const float2 m = a.means2D[g];  // loaded with the radius, not behind it: one round trip
        asm volatile("" ::"v"(m.x), "v"(m.y));  // (kept here: the compiler sinks it into the branch)
        int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
        if (r > 0) get_rect(m.x, m.y, r, a.grid_x, a.grid_y, x0, y0, x1, y1);
        s_x0[i] = x0;
        s_y0[i] = y0;
        s_w[i] = max(x1 - x0, 1);
    }
    __syncthreads();
    const uint32_t total = s_end[n - 1];
    if (scatter && a.flags)
        for (uint32_t q = t; q < total; q += nt) a.flags[base + q] = 0u;
    const uint32_t per = (total + nt - 1) / nt;
    uint32_t q = min((uint32_t)t * per, total);
    const uint32_t q1 = min(q + per, total);
    if (q >= q1) return;
    int lo = 0, hi = n - 1;  // first Gaussian whose end > q
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_end[mid] > q) hi = mid;
        else lo = mid + 1;
    }
    uint32_t end = s_end[lo];
    const uint32_t k = q - (lo == 0 ? 0u : s_end[lo - 1]);
    int w = s_w[lo], x0 = s_x0[lo];
    int x = x0 + (int)(k % (uint32_t)w), y = s_y0[lo] + (int)(k / (uint32_t)w);
    uint32_t key = scatter ? a.depth_keys[g0 + lo] : 0u;
    for (;;) {
        visit((uint32_t)(y * a.grid_x + x), (uint32_t)(g0 + lo), key);
        if (++q >= q1) break;
        if (q < end) {
            if (++x == x0 + w) { x = x0; ++y; }
        } else {  // next Gaussian with instances
            do { ++lo; } while (s_end[lo] <= q);
            end = s_end[lo];
            w = s_w[lo]; x0 = s_x0[lo]; x = x0; y = s_y0[lo];
            if (scatter) key = a.depth_keys[g0 + lo];
        }
    }
}

// Gaussian range of binning workgroup b: whole kBinSub sub-ranges, split evenly
__device__ __forceinline__ void bin_range(const BinArgs& a, int& g_begin, int& g_end) {
    const int nsub = (a.P + kBinSub - 1) / kBinSub;
    const int b = blockIdx.x;
    g_begin = (int)((long long)b * nsub / a.nblk) * kBinSub;
    g_end = min((int)((long long)(b + 1) * nsub / a.nblk) * kBinSub, a.P);
}

__global__ void __launch_bounds__(kBinThreads) bin_count_kernel(BinArgs a) {
    extern __shared__ uint32_t s_dyn[];
    uint32_t* s_cnt = s_dyn;  // [T]
    uint32_t* s_end = s_dyn + a.T;
    int* s_x0 = reinterpret_cast<int*>(s_end + kBinSub);
    int* s_y0 = s_x0 + kBinSub;
    int* s_w = s_y0 + kBinSub;
    for (int i = threadIdx.x; i < a.T; i += kBinThreads) s_cnt[i] = 0u;
    // bin_colscan_kernel's look-back status words and ticket start at zero
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < (a.T + 63) / 64 + 1; i += kBinThreads) a.tile_scan[i] = 0ull;
    int gb, ge;
    bin_range(a, gb, ge);
    for (int g0 = gb; g0 < ge; g0 += kBinSub)
        bin_enumerate(a, g0, min(kBinSub, ge - g0), s_end, s_x0, s_y0, s_w, false,
                      [&](uint32_t tile, uint32_t, uint32_t) { atomicAdd(s_cnt + tile, 1u); });
    __syncthreads();
    uint32_t* row = a.hist + (size_t)blockIdx.x * a.T;
    for (int i = threadIdx.x; i < a.T; i += kBinThreads) row[i] = s_cnt[i];
}

// Column scan of the per-workgroup tile counts: hist[b, t] = sum of hist[b', t] over b' < b (workgroup
// b's first position inside tile t's range) and tile_work[t] = the column total (the tile's
// instance count, which tile_ranges_kernel turns into its first position). 64 tiles per workgroup
// (one per lane), wave w of 16 owns the contiguous rows [w nblk / 16, (w + 1) nblk / 16). One launch
// for what were two (the totals, then the offsets after the ranges: round 6, one kernel boundary
// fewer on the binning's critical path); the scatter adds the tile's first position.
//
// Round 6: the tiles' ranges and first positions as well (what tile_ranges_kernel computed in a
// launch of its own, one 1024-thread workgroup scanning all T counts: 11 us at M1), by a decoupled
// look-back over the workgroups' 64-tile totals (status words a.tile_scan, zeroed by bin_count_kernel;
// the workgroup's logical id from a ticket, as scan_touched_kernel's).
constexpr uint64_t kTileScanAggregate = 1ull << 62, kTileScanInclusive = 2ull << 62;
__global__ void __launch_bounds__(1024) bin_colscan_kernel(BinArgs a, uint2* __restrict__ ranges) {
    __shared__ uint32_t s_part[16][64];
    __shared__ int s_blk;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int nbk = (a.T + 63) / 64;
    if (threadIdx.x == 0)
        s_blk = (int)__hip_atomic_fetch_add(a.tile_scan + nbk, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int blk = s_blk;
    const int tile = blk * 64 + l;
    const int r0 = w * a.nblk / 16, r1 = (w + 1) * a.nblk / 16;
    // the wave's rows of the column held in registers: all loads in flight at once, and the offsets
    // pass below writes from them (a loop of dependent loads, twice: 20.2 -> 15.5 us at M1,
    // profiles/r06/colscan_regs/)
    constexpr int kRows = (R3DG_BIN_BLOCKS_MAX + 15) / 16;  // r1 - r0 <= ceil(nblk / 16)
    uint32_t c[kRows];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
        c[k] = (tile < a.T && r0 + k < r1) ? a.hist[(size_t)(r0 + k) * a.T + tile] : 0u;
        s += c[k];
    }
    s_part[w][l] = s;
    __syncthreads();
    uint32_t run = 0;
    for (int k = 0; k < w; ++k) run += s_part[k][l];
    if (w == 15) {
        // the column totals of this workgroup's 64 tiles -> their first positions
        const uint32_t cnt = tile < a.T ? run + s : 0u;
        uint32_t x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (l >= o) x += y;
        }
        const uint32_t agg = __shfl(x, 63);
        if (blk > 0 && l == 0)
            __hip_atomic_store(a.tile_scan + blk, kTileScanAggregate | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t prefix = lookback_prefix(a.tile_scan, blk);
        if (l == 0)
            __hip_atomic_store(a.tile_scan + blk, kTileScanInclusive | (prefix + agg), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t start = prefix + x - cnt;
        if (tile < a.T) {
            a.tile_work[tile] = start;  // the tile's first position
            ranges[tile] = cnt ? make_uint2(start, start + cnt) : make_uint2(0u, 0u);
        }
    }
    if (tile >= a.T) return;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
        if (r0 + k < r1) a.hist[(size_t)(r0 + k) * a.T + tile] = run;
        run += c[k];
    }
}

// Longest-first launch order of the tiles (the backward, the long-tile depth sort): a bucket sort by
// instance count (bucket = count / 4, capped; descending). Only the schedule depends on the order,
// so the order within a bucket, which LDS atomics leave unspecified, changes no result (measured:
// exact-count buckets, which scatter the tiles of a bucket spatially, slowed the backward by 3 %).
// One 1024-thread workgroup; the padded grid's last slots name no tile (T).
__device__ __forceinline__ uint32_t block_exclusive_scan_1024(uint32_t v, uint32_t* s_wave);
__device__ void tile_order_block(int T, const uint2* __restrict__ ranges, uint32_t* __restrict__ order) {
    constexpr int NBK = 1024;
    __shared__ uint32_t hist[NBK];
    __shared__ uint32_t s_wave[16];
    const int t = threadIdx.x;
    const int per = (T + 1023) / 1024;
    const int b0 = min(t * per, T), b1 = min(b0 + per, T);
    auto bucket = [](uint32_t c) { return (int)min(c >> 2, (uint32_t)(NBK - 1)); };
    hist[t] = 0;
    __syncthreads();
    for (int i = b0; i < b1; ++i) {
        const uint2 r = ranges[i];
        atomicAdd(&hist[bucket(r.y - r.x)], 1u);
    }
    __syncthreads();
    // exclusive scan in descending bucket order (over the reversed histogram)
    const uint32_t v = hist[NBK - 1 - t];
    const uint32_t ex = block_exclusive_scan_1024(v, s_wave);
    hist[NBK - 1 - t] = ex;  // now the cursor of bucket NBK-1-t
    __syncthreads();
    for (int i = b0; i < b1; ++i) {
        const uint2 r = ranges[i];
        order[atomicAdd(&hist[bucket(r.y - r.x)], 1u)] = (uint32_t)i;
    }
    const int TP = padded_tile_grid(T);
    if (t < TP - T) order[T + t] = (uint32_t)T;
}

// tile_order_block on its own, when the LDS binning scattered nothing (no instances)
__global__ void __launch_bounds__(1024) tile_order_kernel(int T, const uint2* __restrict__ ranges,
                                                          uint32_t* __restrict__ order) {
    tile_order_block(T, ranges, order);
}

// The scatter grid has one workgroup more than the binning's: it computes the tiles' longest-first
// order (tile_order_block) beside the scatter, off the binning's critical path (round 6: the ranges
// kernel 14.9 -> 11.5 us). (Every scatter workgroup scanning the tile counts itself, so that no
// ranges kernel runs at all, measured slower: the scatter 69 -> 80 us, and the host, which must
// allocate the binning state between the count readback and the scatter launch, then left the GPU
// idle 6 us; profiles/r06/README.md.)
__global__ void __launch_bounds__(kBinThreads) bin_scatter_kernel(BinArgs a, const uint2* __restrict__ ranges,
                                                                  uint32_t* __restrict__ order) {
    if ((int)blockIdx.x == a.nblk) {
        tile_order_block(a.T, ranges, order);
        return;
    }
    extern __shared__ uint32_t s_dyn[];
    uint32_t* s_pos = s_dyn;  // [T] next position of this workgroup's instances of each tile (bucket)
    uint32_t* s_end = s_dyn + a.T;
    int* s_x0 = reinterpret_cast<int*>(s_end + kBinSub);
    int* s_y0 = s_x0 + kBinSub;
    int* s_w = s_y0 + kBinSub;
    const uint32_t* row = a.hist + (size_t)blockIdx.x * a.T;
    int gb, ge;
    bin_range(a, gb, ge);
    if (a.stage) {
        // two-pass scatter, pass 1: the workgroup's first position in each bucket of kBinBucket tiles
        // is the bucket's first position + its column offsets summed over the bucket's tiles, so a
        // workgroup writes one run per bucket (~40 pairs at M1) instead of one per tile (~2.4)
        const int nbk = (a.T + kBinBucket - 1) / kBinBucket;
        for (int b = threadIdx.x; b < nbk; b += kBinThreads) {
            const int t0 = b * kBinBucket, t1 = min(t0 + kBinBucket, a.T);
            uint32_t s = a.tile_work[t0];
            if (t1 - t0 == kBinBucket) {  // all 16 loads in flight at once (a dependent loop: 8 round trips)
#pragma unroll
                for (int k = 0; k < kBinBucket; ++k) s += row[t0 + k];
            } else {
                for (int t = t0; t < t1; ++t) s += row[t];
            }
            s_pos[b] = s;
        }
        for (int g0 = gb; g0 < ge; g0 += kBinSub)
            bin_enumerate(a, g0, min(kBinSub, ge - g0), s_end, s_x0, s_y0, s_w, true,
                          [&](uint32_t tile, uint32_t g, uint32_t key) {
                              const uint32_t b = tile / kBinBucket;
                              a.stage[atomicAdd(s_pos + b, 1u)] =
                                  make_uint2(key, g | ((tile - b * kBinBucket) << kBinBucketShift));
                          });
        return;
    }
    // the workgroup's first position in each tile: the tile's first position + its column offset
    for (int i = threadIdx.x; i < a.T; i += kBinThreads) s_pos[i] = a.tile_work[i] + row[i];
    for (int g0 = gb; g0 < ge; g0 += kBinSub)
        bin_enumerate(a, g0, min(kBinSub, ge - g0), s_end, s_x0, s_y0, s_w, true,
                      [&](uint32_t tile, uint32_t g, uint32_t key) {
                          a.pairs[atomicAdd(s_pos + tile, 1u)] = make_uint2(key, g);
                      });
}

// Two-pass scatter, pass 2: one workgroup per bucket moves the bucket's staged pairs (one contiguous
// range of the list, in pass 1's order) to their tiles' ranges inside it, so every line of the
// bucket's range is written through one L2 (pass 1's runs per (workgroup, tile) were ~2.4 pairs:
// each line was written in pieces by ~7 workgroups on different XCDs). A wave ranks its 64 pairs
// per tile by ballots; one lane per (wave, tile) claims the wave's positions from the tile's LDS
// cursor. The order inside a tile is left unspecified, as the one-pass scatter's: the depth sort
// (tile_depth_sort_kernel / the forward's fused sort) orders every tile by (depth bits, id).
__global__ void __launch_bounds__(1024) bin_bucket_kernel(BinArgs a) {
    __shared__ uint32_t s_cur[kBinBucket];
    const int b = blockIdx.x;
    const int t0 = b * kBinBucket, nt = min(kBinBucket, a.T - t0);
    const int t = threadIdx.x, l = t & 63;
    if (t < nt) s_cur[t] = a.tile_work[t0 + t];
    const uint32_t s0 = a.tile_work[t0];
    const uint32_t s1 = t0 + kBinBucket < a.T ? a.tile_work[t0 + kBinBucket] : a.L;
    __syncthreads();
    const uint32_t idmask = (1u << kBinBucketShift) - 1u;
    for (uint32_t i0 = s0; i0 < s1; i0 += 1024) {
        const uint32_t i = i0 + (uint32_t)t;
        const bool valid = i < s1;
        const uint2 kv = valid ? a.stage[i] : make_uint2(0u, 0u);
        const int sub = valid ? (int)(kv.y >> kBinBucketShift) : -1;
        // rank of the lane among the wave's pairs of its tile; lane s < kBinBucket counts tile s
        uint32_t rank = 0, cnt = 0;
#pragma unroll
        for (int s = 0; s < kBinBucket; ++s) {
            const unsigned long long m = __ballot(sub == s);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (sub == s) rank = r;
            if (l == s) cnt = (uint32_t)__builtin_popcountll(m);
        }
        // lanes 0..15 claim the wave's positions of their tile (one LDS atomic instruction)
        const uint32_t base_l = cnt ? atomicAdd(&s_cur[l & (kBinBucket - 1)], cnt) : 0u;
        const uint32_t base = (uint32_t)__shfl((int)base_l, sub & (kBinBucket - 1));
        if (valid) a.pairs[base + rank] = make_uint2(kv.x, kv.y & idmask);
    }
}

// Fallback above kBinMaxTiles tiles: one global atomic per instance on the per-tile counters
// (counting pass; preprocess zeroed them) or cursors (scatter pass).
template <bool SCATTER>
__global__ void __launch_bounds__(256) bin_atomic_kernel(BinArgs a) {
    __shared__ uint32_t s_end[256];
    __shared__ int s_x0[256], s_y0[256], s_w[256];
    const int g0 = blockIdx.x * 256;
    bin_enumerate(a, g0, min(256, a.P - g0), s_end, s_x0, s_y0, s_w, SCATTER,
                  [&](uint32_t tile, uint32_t g, uint32_t key) {
                      if constexpr (SCATTER) a.pairs[atomicAdd(a.tile_work + tile, 1u)] = make_uint2(key, g);
                      else atomicAdd(a.tile_work + tile, 1u);
                  });
}

static size_t bin_lds_bytes(int T) { return sizeof(uint32_t) * ((size_t)T + 4 * kBinSub); }

// dynamic LDS above 64 KiB must be allowed per kernel (T > 12288 tiles, e.g. 4K frames)
template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

// Exclusive scan of one value per thread over a 1024-thread block: wave scans by lane shuffles,
// then the 16 wave totals (two barriers).
__device__ __forceinline__ uint32_t block_exclusive_scan_1024(uint32_t v, uint32_t* s_wave) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    if (l == 63) s_wave[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < w; ++k) pre += s_wave[k];
    __syncthreads();  // s_wave may be reused
    return pre + x - v;
}

// identifyTileRanges (rasterizer_impl.cu:118-140) from the per-tile counts: one workgroup scans
// them (tile t's range starts after every lower tile's instances, as in the sorted list), writes
// every tile's range (empty tiles (0, 0), the reference's memset value) and turns the counts into
// the tiles' first positions. Then the backward / depth-sort launch order, longest tiles first: a
// bucket sort by instance count (bucket = count / 4, capped; descending). Only the schedule depends
// on the order, so the order within a bucket, which LDS atomics leave unspecified, changes no result
// (measured: exact-count buckets, which scatter the tiles of a bucket spatially, slowed the
// backward by 3 %). Thread t owns the PER tiles [t PER, t PER + PER), held in registers: one round of
// independent loads (PER = 0: any T, counts re-read).
template <int PER>
__global__ void __launch_bounds__(1024) tile_ranges_kernel(int T, uint32_t* __restrict__ work,
                                                           uint2* __restrict__ ranges, uint32_t* __restrict__ order) {
    constexpr int NBK = 1024;
    __shared__ uint32_t hist[NBK];
    __shared__ uint32_t s_wave[16];
    const int t = threadIdx.x;
    const int per = PER > 0 ? PER : (T + 1023) / 1024;
    const int b0 = min(t * per, T), b1 = min(b0 + per, T);
    auto bucket = [](uint32_t c) { return (int)min(c >> 2, (uint32_t)(NBK - 1)); };
    hist[t] = 0;
    uint32_t c[PER > 0 ? PER : 1];
    uint32_t sum = 0;
    if constexpr (PER > 0) {
#pragma unroll
        for (int k = 0; k < PER; ++k) c[k] = b0 + k < b1 ? work[b0 + k] : 0u;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += c[k];
    } else {
        for (int i = b0; i < b1; ++i) sum += work[i];
    }
    uint32_t run = block_exclusive_scan_1024(sum, s_wave);
    if constexpr (PER > 0) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = b0 + k;
            if (i < b1) {
                ranges[i] = c[k] ? make_uint2(run, run + c[k]) : make_uint2(0u, 0u);
                work[i] = run;
                run += c[k];
                if (order) atomicAdd(&hist[bucket(c[k])], 1u);
            }
        }
    } else {
        for (int i = b0; i < b1; ++i) {
            const uint32_t ci = work[i];
            ranges[i] = ci ? make_uint2(run, run + ci) : make_uint2(0u, 0u);
            work[i] = run;
            run += ci;
            if (order) atomicAdd(&hist[bucket(ci)], 1u);
        }
    }
    if (!order) return;  // block-uniform
    __syncthreads();
    // exclusive scan in descending bucket order (over the reversed histogram)
    const uint32_t v = hist[NBK - 1 - t];
    const uint32_t ex = block_exclusive_scan_1024(v, s_wave);
    hist[NBK - 1 - t] = ex;  // now the cursor of bucket NBK-1-t
    __syncthreads();
    if constexpr (PER > 0) {
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if (b0 + k < b1) order[atomicAdd(&hist[bucket(c[k])], 1u)] = (uint32_t)(b0 + k);
    } else {
        for (int i = b0; i < b1; ++i) {
            const uint2 r = ranges[i];
            order[atomicAdd(&hist[bucket(r.y - r.x)], 1u)] = (uint32_t)i;
        }
    }
    const int TP = padded_tile_grid(T);
    if (t < TP - T) order[T + t] = (uint32_t)T;  // the padded grid's last workgroups: no tile
}

hipError_t launch_bin_prepare(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st) {
    if (a.T <= 0) return hipSuccess;
    // with the LDS binning the tile order comes with the scatter (bin_scatter_kernel's extra
    // workgroup, or tile_order_kernel when nothing is scattered: launch_bin_order)
    const bool lds = a.P > 0 && a.hist;
    if (a.P > 0) {
        if (lds) {
            const hipError_t e = allow_lds(bin_count_kernel, bin_lds_bytes(a.T));
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(bin_count_kernel, dim3(a.nblk), dim3(kBinThreads), bin_lds_bytes(a.T), st, a);
            // column scan + the tiles' ranges and first positions (no tile_ranges_kernel)
            hipLaunchKernelGGL(bin_colscan_kernel, dim3((a.T + 63) / 64), dim3(1024), 0, st, a, ranges);
            return hipGetLastError();
        } else {
            hipLaunchKernelGGL(bin_atomic_kernel<false>, dim3((a.P + 255) / 256), dim3(256), 0, st, a);
        }
    }
    uint32_t* ord = lds ? nullptr : order;
    if (a.T <= 8 * 1024)
        hipLaunchKernelGGL(tile_ranges_kernel<8>, dim3(1), dim3(1024), 0, st, a.T, a.tile_work, ranges, ord);
    else if (a.T <= 40 * 1024)
        hipLaunchKernelGGL(tile_ranges_kernel<40>, dim3(1), dim3(1024), 0, st, a.T, a.tile_work, ranges, ord);
    else
        hipLaunchKernelGGL(tile_ranges_kernel<0>, dim3(1), dim3(1024), 0, st, a.T, a.tile_work, ranges, ord);
    return hipGetLastError();
}

hipError_t launch_bin_scatter(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st) {
    if (a.P <= 0 || a.T <= 0) return hipSuccess;
    if (a.hist) {
        const hipError_t e = allow_lds(bin_scatter_kernel, bin_lds_bytes(a.T));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(bin_scatter_kernel, dim3(a.nblk + 1), dim3(kBinThreads), bin_lds_bytes(a.T), st, a, ranges,
                           order);
        if (a.stage)  // pass 2: the bucketed pairs to their tiles
            hipLaunchKernelGGL(bin_bucket_kernel, dim3((a.T + kBinBucket - 1) / kBinBucket), dim3(1024), 0, st, a);
    } else {
        hipLaunchKernelGGL(bin_atomic_kernel<true>, dim3((a.P + 255) / 256), dim3(256), 0, st, a);
    }
    return hipGetLastError();
}

// the tile order when the LDS binning ran but nothing was scattered (no instances)
hipError_t launch_bin_order(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st) {
    if (a.T <= 0 || !(a.P > 0 && a.hist)) return hipSuccess;
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, a.T, ranges, order);
    return hipGetLastError();
}

// The depth half of the binning: every tile's instances, in whatever order the scatter left them,
// sorted by (depth bits, Gaussian id) -- the reference's stable (tile << 32 | depth) sort of the
// Gaussian-major list orders a tile by depth and breaks ties by Gaussian id. One workgroup per tile,
// longest tiles first. A chunk of the tile is sorted in registers / LDS (rocPRIM block radix sort,
// 4 passes of 8 bits) -- 1024-instance chunks for tiles of up to 1024 instances, 2048-instance
// chunks for longer ones (both sorters share one LDS union: 16 KB, still 8 waves/SIMD). A chunk
// with equal depth bits (cloned Gaussians share a depth until they move) is sorted again: by
// Gaussian id, then stably by depth. A tile longer than one chunk sorts each chunk into a run and
// merges run pairs (merge path, (depth, id) compared lexicographically) through the scratch
// buffers, ping-pong, landing in point_list.
union TileDepthSortStorage {
    TileSortLds<4> s4;
    TileSortLds<R3DG_SORT_LONG_IPT> sl;
};

__device__ __forceinline__ uint32_t nt_load(const uint32_t* p) { return __builtin_nontemporal_load(p); }

// (depth bits, Gaussian id) order; Gaussian ids are unique within a tile
__device__ __forceinline__ bool kv_less(uint32_t ka, uint32_t va, uint32_t kb, uint32_t vb) {
    return ka < kb || (ka == kb && va < vb);
}

// chunks of kSortBT * IPT instances of the tile [s, s + n) sorted into runs at (rk, rv)
template <int IPT>
__device__ __forceinline__ void sort_tile_chunks(uint32_t s, uint32_t n, uint32_t nchunks, const uint2* pairs,
                                                 uint32_t* rk, uint32_t* rv, TileSortLds<IPT>& lds) {
    constexpr uint32_t kChunk = kSortBT * IPT;
    const int t = threadIdx.x;
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t c0 = c * kChunk;
        uint32_t keys[IPT], vals[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {  // blocked arrangement: item index = t * IPT + k
            const uint32_t i = c0 + (uint32_t)(t * IPT + k);
            const uint2 kv = i < n ? pairs[s + i] : make_uint2(0xffffffffu, 0xffffffffu);
            keys[k] = kv.x;
            vals[k] = kv.y;
        }
        if (c > 0) __syncthreads();  // storage reuse
        sort_pairs_chunk<IPT>(keys, vals, (int)min(kChunk, n - c0), lds);
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

#ifndef R3DG_SORT_WAVES
#define R3DG_SORT_WAVES 6  // waves per SIMD the long-tile sorter's registers target (80 VGPR; 8: 64, spills)
#endif
__global__ void __launch_bounds__(kSortBT) __attribute__((amdgpu_waves_per_eu(R3DG_SORT_WAVES)))
tile_depth_sort_kernel(int T, const uint2* __restrict__ ranges, const uint32_t* __restrict__ order,
                       const uint2* __restrict__ pairs, uint32_t* __restrict__ point_list,
                       uint32_t* kA, uint32_t* vA, uint32_t* kB, int min_n) {
    __shared__ TileDepthSortStorage storage;
    const int b = blockIdx.x;
    if (b >= T) return;
    const int tile = order ? (int)order[b] : b;
    const uint2 rg = ranges[tile];
    const uint32_t s = rg.x, n = rg.y - rg.x;
    const int t = threadIdx.x;
    if (n <= (uint32_t)min_n) return;  // sorted by the forward blend (fused)
    if (n == 1) {
        if (t == 0) point_list[s] = pairs[s].y;
        return;
    }
    // sorter capacity by tile length (block-uniform); a 2-item sorter for tiles of up to 512
    // instances measured no faster (M1: 0.086 vs 0.083 ms, it spills one VGPR)
    const uint32_t kChunk = n <= kSortBT * 4 ? kSortBT * 4 : kSortBT * R3DG_SORT_LONG_IPT;
    const uint32_t nchunks = (n + kChunk - 1) / kChunk;
    int rounds = 0;
    while ((1u << rounds) < nchunks) ++rounds;
    // runs go where an even number of merge rounds leaves the result in (kB, point_list)
    uint32_t* rk = (rounds & 1) ? kA : kB;
    uint32_t* rv = (rounds & 1) ? vA : point_list;
    if (kChunk == kSortBT * 4)
        sort_tile_chunks<4>(s, n, nchunks, pairs, rk, rv, storage.s4);
    else
        sort_tile_chunks<R3DG_SORT_LONG_IPT>(s, n, nchunks, pairs, rk, rv, storage.sl);
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
            const uint32_t* Av = sv + s + a0;
            const uint32_t* Bv = sv + s + a1;
            // merge path: i = number of A items among the first d0 outputs
            uint32_t lo = d0 > lb ? d0 - lb : 0u, hi = min(d0, la);
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1, o = d0 - 1 - mid;
                if (!kv_less(nt_load(B + o), nt_load(Bv + o), nt_load(A + mid), nt_load(Av + mid))) lo = mid + 1;
                else hi = mid;
            }
            uint32_t i = lo, j = d0 - lo;
            uint32_t ka = 0xffffffffu, va = 0xffffffffu, kb = 0xffffffffu, vb = 0xffffffffu;
            if (i < la) { ka = nt_load(A + i); va = nt_load(Av + i); }
            if (j < lb) { kb = nt_load(B + j); vb = nt_load(Bv + j); }
            for (uint32_t d = d0; d < d1; ++d) {
                const bool takeA = j >= lb || (i < la && kv_less(ka, va, kb, vb));
                if (takeA) {
                    dk[s + a0 + d] = ka;
                    dv[s + a0 + d] = va;
                    ++i;
                    if (i < la) { ka = nt_load(A + i); va = nt_load(Av + i); }
                } else {
                    dk[s + a0 + d] = kb;
                    dv[s + a0 + d] = vb;
                    ++j;
                    if (j < lb) { kb = nt_load(B + j); vb = nt_load(Bv + j); }
                }
            }
        }
        __syncthreads();
        uint32_t* tk = sk; sk = dk; dk = tk;
        uint32_t* tv = sv; sv = dv; dv = tv;
    }
}

hipError_t launch_tile_depth_sort(int T, const uint2* ranges, const uint32_t* order, const uint2* pairs,
                                  uint32_t* point_list, uint32_t* kA, uint32_t* vA,
                                  uint32_t* kB, int min_n, hipStream_t st) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(tile_depth_sort_kernel, dim3(T), dim3(kSortBT), 0, st, T, ranges, order, pairs, point_list,
                       kA, vA, kB, min_n);
    return hipGetLastError();
}

}  // namespace r3dg
