// r3dg_kernels.h -- kernel argument blocks and launch helpers shared between the kernel
// translation units and the host orchestration (rasterizer.hip).
#pragma once

#include <hip/hip_ext.h>

#include <algorithm>

#include "r3dg_common.h"

namespace r3dg {

struct PreprocessArgs {
    int P, D, M, W, H, grid_x, grid_y, prefiltered;
    float focal_x, focal_y, tan_fovx, tan_fovy, scale_modifier;
    const float* means3D;
    const float* scales;
    const float* rotations;
    const float* opacity;
    const float* sh;
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    int* radii;
    uint32_t* tiles_touched;
    uint32_t* depth_keys;  // float bits of the view depth, 0xffffffff when not visible
    float4* records;       // [P, rec4] render records (see record_f4)
    int rec4, S;
    const float* features; // [P, S]
    float* depths;
    float2* means2D;
    float* cov3D;
    float4* conic_opacity;
    float* rgb;
    uint8_t* clamped;
    unsigned int* error_flag;
    uint32_t* tile_count;  // [num_tiles] zeroed here for the atomic binning (bin_atomic_kernel), or null
    int num_tiles;
    uint64_t* scan_status; // [scan_words] zeroed here for the single-pass scan (scan_touched_kernel), or null
    int scan_words;
    uint32_t* work_hist;   // [kWorkBuckets] zeroed here for the forward's work buckets (RenderFwdArgs::bwd_hist)
};

// Binning (duplicateWithKeys + SortPairs + identifyTileRanges, rasterizer_impl.cu:72-140, 343-383)
// as two passes over the instances with per-tile counters instead of a radix sort over L keys:
// see preprocess.hip bin_count_kernel.
struct BinArgs {
    int P, grid_x, grid_y, rec4, T;
    int nblk;                 // binning workgroups (bin_blocks); each owns a contiguous Gaussian range
    const uint32_t* offsets;  // inclusive scan of tiles touched
    const float2* means2D;
    const int* radii;
    uint32_t* tile_work;      // [T] instance count per tile, then the tile's first position
    uint32_t* hist;           // [nblk, T] per-workgroup tile counts, then positions; null: T too large
                              // for the LDS counters, every instance takes a global atomic instead
    const uint32_t* depth_keys;  // [P] float bits of each Gaussian's view depth
    uint2* pairs;             // [L] scatter pass: (depth bits, Gaussian) of each instance, grouped by tile
    uint32_t* flags;          // [L] scatter pass: backward row flags of each slot, zeroed
    uint2* stage;             // [L] two-pass scatter: the pairs grouped by tile bucket (Gaussian id | the
                              // tile's index in its bucket << 28); null: one pass straight to the tiles
    uint32_t L;               // scatter passes: instances in all
    uint64_t* tile_scan;      // [T / 64 + 1] bin_colscan_kernel's look-back status words and ticket
};
// Two-pass scatter: buckets of kBinBucket consecutive tiles (one contiguous range of the sorted list)
constexpr int kBinBucket = 16;
constexpr int kBinBucketShift = 28;  // the tile's index in its bucket above the Gaussian id (P < 2^28)
constexpr int kBinThreads = 1024;                  // binning workgroup (one per CU)
constexpr int kBinSub = 1024;                      // Gaussians staged in LDS at a time
constexpr int kBinMaxTiles = (163840 - 16 * kBinSub) / 4;  // LDS counters per workgroup (160 KiB)
// binning workgroups for T tiles: the [nblk, T] count matrix stays <= 4 * R3DG_BIN_MATRIX entries
#ifndef R3DG_BIN_BLOCKS_MAX
#define R3DG_BIN_BLOCKS_MAX 256
#endif
#ifndef R3DG_BIN_MATRIX
#define R3DG_BIN_MATRIX (1 << 21)
#endif
inline int bin_blocks_max(int T) {
    return T > kBinMaxTiles ? 0 : std::max(1, std::min(R3DG_BIN_BLOCKS_MAX, R3DG_BIN_MATRIX / std::max(T, 1)));
}

struct RenderFwdArgs {
    const float4* records;     // render records (record_f4), used by the default-shader kernel
    const uint2* ranges;
    const uint32_t* point_list;
    const float2* means2D;
    const float4* conic_opacity;
    const float* depths;
    const float* colors;
    const float* shader_colors;
    const float* features;
    const float* bg;
    int S, W, H, grid_x, num_tiles, cull;
    const uint32_t* tile_order;  // launch order of the tiles (longest first), or null
    float* final_T;
    uint32_t* n_contrib;
    float* out_color;
    float* out_opacity;
    float* out_depth;
    float* out_feature;
    float* out_shader_color;
    float* zero_stencil;  // stencil output to zero (default splat shaders), or null
    // the backward's per-Gaussian atomic sums (in the geometry state), zeroed here so the backward
    // needs no memset: tile t's workgroup zeroes float4s [t * zero_chunk, (t + 1) * zero_chunk) of
    // the zero_n4 after its outputs (the stores drain under the other workgroups' blends); null: none
    float4* zero_sums;
    uint32_t zero_n4, zero_chunk;
    uint8_t* contrib;     // [L] per sorted position: bit 2q + h set when a pixel of half h (rows 0-3 / 4-7) of quadrant q blended it
    FeatureLayout flay;
    // fused depth sort (default-shader kernel): tiles of up to kFusedSortMax instances are sorted
    // from the binning's (depth bits, id) pairs in the blend's prologue and their sorted ids written
    // to point_list_out; null pairs: every tile was sorted by tile_depth_sort_kernel
    const uint2* pairs;
    uint32_t* point_list_out;
    // non-default splat shaders: per Gaussian float4 [shader r, g, b, 0] (refresh_record_opacity
    // writes it after the splat shaders), staged as one more record column
    const float4* shader_rec;
    // [T] the backward's work per tile (the most visits of any of its quadrants), or null; with it
    // each tile's rank in its work bucket (bwd_rank [T]) from the bucket counts bwd_hist
    // [kWorkBuckets] (zeroed by preprocess_kernel)
    uint32_t* bwd_work;
    uint32_t* bwd_rank;
    uint32_t* bwd_hist;
};
constexpr int kWorkBuckets = 1024;
__host__ __device__ inline int work_bucket(uint32_t work) { return (int)(work >> 2 < 1023u ? work >> 2 : 1023u); }
constexpr int kFusedSortMax = 1024;

// Per-Gaussian gradient sums the gather kernel assembles (LDS, one row per Gaussian):
// [mean2D x,y,z | conic x,y,w | opacity | colour r,g,b | features 0..S-1 | pad].
constexpr int kRowMean = 0, kRowConic = 3, kRowOpacity = 6, kRowColor = 7, kRowFeat = 10;

// Partial gradient row written by the backward blend for one (instance, 8x8 quadrant) pair --
// the reduction of one wave's 64 pixels, at index 4 * slot + quadrant:
//   [0, XW)      X part: sum_px w * [dL/dcolour 0..2, dL/dfeature 0..S-1, dL/ddepth], zero pad
//   [XW, XW+6)   moments of q = G * dL/dalpha about the quadrant centre (pixel offsets x, y in
//                -3.5 .. 3.5): sum q * [1, x, y, x^2, xy, y^2]
//   [XW+6, XW+8) the quadrant centre (pixel coordinates): the row sum expands the moments about
//                the Gaussian's mean without decoding the row's tile
// with w = alpha * T and XW = 16 * bwd_xblocks(S). A row exists only where the wave blended the
// instance; flags[4 * slot + quadrant] = 1 marks it (the gather reads flagged rows only).
__host__ __device__ inline int bwd_xblocks(int S);
__host__ __device__ inline int part_row_stride(int S);

struct RenderBwdArgs {
    const float4* records;     // render records (record_f4)
    const uint2* ranges;
    const uint32_t* point_list;
    const uint32_t* offsets;   // inclusive scan of tiles touched: Gaussian g owns slots [offsets[g-1], offsets[g])
    const int* radii;
    const float2* means2D;
    const float4* conic_opacity;
    const float* depths;
    const float* colors;
    const float* features;
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;      // colour grads, channel c of pixel p at ca[c] + p * cm[c]
    int ca[3], cm[3];
    const float* dL_dpix_o;
    const float* dL_dpix_d;
    const float* dL_dpix_f;    // feature grads, layout gflay
    FeatureLayout gflay;
    int S, W, H, grid_x, grid_y, num_tiles, cull, backward_geometry, RS;
    const uint32_t* tile_order;  // launch order of the tiles (longest first), or null
    float* rows;               // [4L, RS] partial rows (part_row_stride)
    uint8_t* flags;            // [4L] 1 where a partial row was written (zeroed by the forward's binning scatter)
    const uint8_t* contrib;    // [L] the forward's contribution bits (RenderFwdArgs::contrib)
    int sums_atomic;           // 1: flush straight into `sums` with f32 atomics (no rows / flags)
    float* sums;               // [P, SRS] per-Gaussian sums, zeroed before the launch (sums_atomic)
    int SRS;
    // kernel variant (host side; r3dg_options test_bwd_dpp / test_bwd_wterms): 0 the default
    int variant_dpp, wterms;
};

struct GatherBwdArgs {
    int P, D, M, S, RS, W, H, grid_x, grid_y;
    int g_begin, g_end;       // Gaussian range of this launch (outputs indexed by global id)
    const float* rows;        // partial rows (RenderBwdArgs)
    float* sums;              // [P, RS] per-Gaussian sums (row_sum_kernel -> gather_bwd_kernel)
    int sums_moments;         // 1: sums hold the raw moments about the mean (atomic flush), stride SRS
    int SRS;
    const uint32_t* flags;    // one word per slot: byte q set when quadrant q's row exists
    const float2* means2D;
    const float4* conic_opacity;
    const uint32_t* offsets;
    const int* radii;
    const float* means3D;
    const float* sh;
    const uint8_t* clamped;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    const float* cov3D;       // precomputed or geom-state cov3D
    const float* view;
    const float* proj;
    const float* campos;
    float focal_x, focal_y, tan_fovx, tan_fovy;
    int use_scales;           // scales/rotations given (cov3D not precomputed)
    float* dL_dmeans2D;
    float* dL_dcolors;
    float* dL_dopacity;
    float* dL_dmeans3D;
    float* dL_dfeatures;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dscales;
    float* dL_drotations;
    // row strides (floats) of dL_dmeans3D / dL_dopacity / dL_dscales / dL_drotations / dL_dfeatures:
    // 3, 1, 3, 4, S, or one packed [P, 11 + S] row each (r3dg_backward_outputs.dense_stride)
    int ld_m3, ld_op, ld_sc, ld_rot, ld_f;
};

struct XyzNormalArgs {
    int W, H;
    const float* view;
    float focal_x, focal_y, cx, cy;
    const float* opacity;
    const float* depth;
    float* normal;
    float* xyz;
    // the backward's launch order, computed by the grid's extra column from the forward's per-tile
    // work (RenderFwdArgs::bwd_work), or null
    int num_tiles, blocks_x;   // blocks_x: pixel workgroups per row of the 1-D grid
    const uint32_t* bwd_work;
    const uint32_t* bwd_rank;
    const uint32_t* bwd_hist;
    uint32_t* bwd_order;
};

struct IntermediateArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    const float2* means2D;
    const float4* conic_opacity;
    const float* depths;
    const float* stencils;
    const float* stencil_opacity;
    int W, H, grid_x, num_tiles;
    float* out_depth;
    float* out_stencil;
    const float4* records;  // render records (intermediate_glds_kernel stages conic + opacity, position)
    int rec4;
    float4* inter_rec;      // [P] scratch: [depth, stencil, stencil opacity, 0], packed per launch
    const uint32_t* tile_order;  // launch order of the tiles (longest first), or null (XCD-aware spatial)
};

// kernels (defined in the .hip translation units)
__global__ void preprocess_kernel(PreprocessArgs a);
__global__ void mark_visible_kernel(int P, const float* means3D, const float* view, uint8_t* present);
// counts, tile ranges, the longest-first tile order and every workgroup's scatter positions
hipError_t launch_bin_prepare(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st);
hipError_t launch_bin_scatter(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st);
hipError_t launch_bin_order(const BinArgs& a, uint2* ranges, uint32_t* order, hipStream_t st);
// sorts the tiles longer than min_n instances (the forward sorts the others when fused)
hipError_t launch_tile_depth_sort(int T, const uint2* ranges, const uint32_t* order, const uint2* pairs,
                                  uint32_t* point_list, uint32_t* kA, uint32_t* vA, uint32_t* kB, int min_n,
                                  hipStream_t st);

// Slot of an instance from its Gaussian's render record word 1 (x, y, -, radius), the Gaussian's
// first slot slot0 = offsets[g-1] and the tile (the rows reduction's partial-row index).
__device__ __forceinline__ uint32_t record_slot(float4 r1, uint32_t slot0, int tx, int ty, int grid_x, int grid_y) {
    int x0, y0, x1, y1;
    get_rect(r1.x, r1.y, __float_as_int(r1.w), grid_x, grid_y, x0, y0, x1, y1);
    return slot0 + (uint32_t)((ty - y0) * (x1 - x0) + (tx - x0));
}

// Slot of the instance (Gaussian g, tile) in the reference's unsorted, Gaussian-contiguous order:
// offsets[g-1] + row-major index of the tile in g's rect (duplicateWithKeys, rasterizer_impl.cu:92-107).
__device__ __forceinline__ uint32_t instance_slot(const uint32_t* offsets, float2 xy, int radius, uint32_t g,
                                                  int tx, int ty, int grid_x, int grid_y) {
    int x0, y0, x1, y1;
    get_rect(xy.x, xy.y, radius, grid_x, grid_y, x0, y0, x1, y1);
    return (g == 0 ? 0u : offsets[g - 1]) + (uint32_t)((ty - y0) * (x1 - x0) + (tx - x0));
}
#ifndef R3DG_XYZ_R
#define R3DG_XYZ_R 4  // tile rows per xyz_normal_kernel workgroup (render_fwd.hip; 1 / 2 / 4 / 8: 25.7 / 25.0 / 21.7 / 24.9 us at M1)
#endif
__global__ void xyz_normal_kernel(XyzNormalArgs a);
constexpr int kOrderSlices = 16;  // xyz_normal_kernel's leading workgroups that sort the backward's tile order
// RenderIntermediateTextures: packs the per-Gaussian depth / stencil record, then the DMA-staged blend
hipError_t launch_intermediate(const IntermediateArgs& a, int P, const int* radii, hipStream_t st);
hipError_t launch_bwd_order(int T, const uint32_t* work, const uint32_t* rank, const uint32_t* hist, uint32_t* order,
                            hipStream_t st);

// host launchers for the templated blend kernels
hipError_t launch_render_forward(const RenderFwdArgs& a, bool shader, hipStream_t stream);
hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t stream);
hipError_t launch_row_sum(const GatherBwdArgs& a, hipStream_t stream);
hipError_t launch_gather_backward(const GatherBwdArgs& a, hipStream_t stream);
hipError_t launch_sh_color_grads(int n, const uint8_t* clamped, const float* dcol, float* out, hipStream_t st);
hipError_t launch_sh_grad_views(int g0, int n, int deg, int M, int N, const float* means3D, const float* campos,
                                const float* drgb, float* dsh, hipStream_t st);

// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so block b runs on the
// same XCD as b+8. Give each XCD a contiguous band of tiles (neighbouring tiles share
// Gaussians, so their attribute gathers hit the same L2). Grid is padded to a multiple of 8.
// Feature-count bucket of the templated blend kernels (launch_* dispatch) and the per-Gaussian
// render record the blend kernels stage from: float4 [conic.x, conic.y, conic.z, opacity],
// float4 [x, y, 0, radius bits], then the attribute row [r, g, b, depth, f0 .. f_{SMAX-1}]
// zero-padded to (4 + SMAX + 3) / 4 float4. Written by preprocess_kernel for visible Gaussians
// only; the blend kernels never stage an invisible one.
__host__ __device__ inline int smax_of(int S) {
    return S == 0 ? 0 : S <= 4 ? 4 : S <= 8 ? 8 : S <= 12 ? 12 : S <= 16 ? 16 : S <= 24 ? 24 : 32;
}
__host__ __device__ inline int record_f4(int S) { return 2 + (4 + smax_of(S) + 3) / 4; }
__host__ __device__ inline int bwd_xblocks(int S) { return (4 + smax_of(S) + 15) / 16; }
// partial-row stride (floats): X part + 6 moments + 2 pad, rounded up to R3DG_ROW_ALIGN floats.
// Rows of whole 128-byte lines (R3DG_ROW_ALIGN 32) measured slower: row-sum 0.235 -> 0.246 ms,
// gather 0.144 -> 0.152 ms at M1 (more bytes per present row, no fewer lines touched).
#ifndef R3DG_ROW_ALIGN
#define R3DG_ROW_ALIGN 8
#endif
__host__ __device__ inline int part_row_stride(int S) {
    return (16 * bwd_xblocks(S) + 8 + R3DG_ROW_ALIGN - 1) / R3DG_ROW_ALIGN * R3DG_ROW_ALIGN;
}

__host__ __device__ inline int padded_tile_grid(int num_tiles) { return (num_tiles + 7) & ~7; }
__device__ __forceinline__ int xcd_tile(int b, int grid) {
    const int per = grid >> 3;
    return (b & 7) * per + (b >> 3);
}
// Tile of workgroup b: from a launch order when one is given (padded_tile_grid entries, num_tiles
// marking a slot without a tile): the longest tiles first (workgroups are dispatched in index
// order, so the heaviest tiles start first and the tail is made of short tiles;
// tile_ranges_kernel), else the XCD-aware spatial order.
__device__ __forceinline__ int block_tile(const uint32_t* order, int num_tiles) {
    const int b = blockIdx.x;
    if (order) return (int)order[b];
    return xcd_tile(b, gridDim.x);
}
#ifdef R3DG_EXP_COUNT  // timing/counting experiment builds only (tools/exp_build.sh)
static __device__ unsigned long long g_exp_cnt[8];  // one copy per translation unit
#define R3DG_EXP_READER(name)                                                        \
    extern "C" void name(unsigned long long* out) {                                  \
        hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp_cnt), sizeof(g_exp_cnt));         \
    }
#define R3DG_EXP_ADD(i, v) atomicAdd(&g_exp_cnt[i], (unsigned long long)(v))
#else
#define R3DG_EXP_ADD(i, v) ((void)0)
#endif

// ---- profiled launches ----------------------------------------------------------------------
// While r3dg_profile_enable is active, a profiled stage (rasterizer.hip ProfScope) hands its
// start / stop events to the stage's kernel launch, which records them as part of the dispatch
// (hipExtLaunchKernelGGL): device-side timestamps with no separate marker packets between
// kernels, so profiling does not add gaps to the timed steps.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents take_launch_events();  // the pending pair (cleared), or nulls when none is pending

template <typename K, typename... Args>
inline void launch_kernel(K kernel, dim3 grid, dim3 block, hipStream_t stream, Args... args) {
    const LaunchEvents e = take_launch_events();
    if (e.start)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, e.start, e.stop, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, stream, args...);
}

}  // namespace r3dg
