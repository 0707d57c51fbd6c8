// r3dg_common.h -- device-side constants, math helpers and the opaque state-buffer layouts
// shared by the HIP kernels of the relightable splat rasterizer (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "r3dg_hip.h"

namespace r3dg {

constexpr int kTileX = 16;  // screen tile (reference config.h:15-16)
constexpr int kTileY = 16;
constexpr int kBlock = kTileX * kTileY;  // one pixel per thread, 4 wave64 per tile
constexpr int kWave = 64;
constexpr int kMaxFeatures = 32;  // S limit of this build (reference bwd caps S at 24, backward.cu:449)

// Spherical-harmonic constants (reference auxiliary.h:22-39).
__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

// Feature output layout: channel c of pixel pix lives at a[c] + pix * m[c] (r3dg_feature_groups).
struct FeatureLayout {
    int a[kMaxFeatures];
    int m[kMaxFeatures];
};
FeatureLayout make_feature_layout(int S, long long HW, bool native);

// ---- opaque state buffers ------------------------------------------------------------------
// Layouts are pure functions of (P), (L) and (H, W) so the backward can re-derive the pointers
// from the buffers the autograd context kept (the reference does the same with fromChunk,
// rasterizer_impl.cu:157-201). Every array starts on a 256-byte boundary.
struct GeomState {
    float* depths;          // [P]   view-space z
    int* internal_radii;    // [P]   used when the caller passes no radii output
    float2* means2D;        // [P]
    float* cov3D;           // [P,6]
    float4* conic_opacity;  // [P]
    float* rgb;             // [P,3]
    float* shader_rgb;      // [P,3] splat-shader colour (only written when a splat shader runs)
    float* stencils;        // [P]
    float* stencil_opacity; // [P]
    uint8_t* clamped;       // [P] bit c: SH colour channel c clamped at 0
    uint32_t* tiles_touched;// [P]
    uint32_t* point_offsets;// [P] inclusive scan of tiles_touched (Gaussian-contiguous slots)
    uint32_t* depth_keys;   // [P] depth bits (0xffffffff: not visible)
    void* scan_temp;
    size_t scan_temp_bytes;
    // [P, record_f4(S)] render records, last in the buffer (r3dg_kernels.h): only set when the
    // state is carved with S
    float4* records;
};

struct BinningState {
    // Instances grouped by tile with per-tile counters, then every tile sorted by (depth bits,
    // Gaussian id): the reference's stable sort by (tile << 32 | depth bits) of its Gaussian-major
    // instance list (preprocess.hip bin_count_kernel / tile_depth_sort_kernel).
    uint32_t* point_list;   // [L] Gaussian ids in sorted order (reference point_list)
    uint2* pairs;           // [L] (depth bits, Gaussian) grouped by tile, unsorted within a tile
    uint32_t* sort_k1;      // [L] depth-sort scratch (tiles longer than one sort chunk)
    uint32_t* sort_v1;      // [L]
    uint32_t* sort_k2;      // [L]
    uint32_t* flags;        // [L] backward row flags, one byte per (slot, quadrant) (render_bwd.hip)
    uint8_t* contrib;       // [L] per sorted position: bit 2q + h = a pixel of half h of quadrant q blended it (forward)
};
struct ImageState {
    float* final_T;     // [H*W]
    uint32_t* n_contrib;// [H*W]
    uint2* ranges;      // [tiles]
    uint32_t* tile_order;        // [padded tiles] tiles by descending instance count (blend launch order)
    uint32_t* tile_work;         // [tiles] binning: instance count per tile, then its first position
    uint32_t* bwd_work;          // [tiles] the forward's count of the backward's work per tile
    uint32_t* bwd_rank;          // [tiles] the tile's rank in its work bucket
    uint32_t* bwd_hist;          // [1024] the work buckets' counts
    uint32_t* bwd_order;         // [padded tiles] the backward's launch order (most work first)
    uint32_t* bin_hist;          // [bin_blocks_max(tiles), tiles] binning: per-workgroup counts / positions
};

size_t geom_state_bytes(size_t P, int S);
size_t binning_state_bytes(size_t L);
size_t image_state_bytes(int H, int W, bool with_hist = true);
GeomState geom_state_from(void* base, size_t P, int S = -1);
BinningState binning_state_from(void* base, size_t L);
ImageState image_state_from(void* base, int H, int W);

// ---- error handling --------------------------------------------------------------------------
void set_error(const std::string& msg);

// the library options (r3dg_set_options; include/r3dg_hip.h): a snapshot, never the environment
r3dg_options options();

#define R3DG_CHECK_HIP(expr)                                                                    \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            ::r3dg::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " at " +      \
                              __FILE__ + ":" + std::to_string(__LINE__));                       \
            return R3DG_ERR_HIP;                                                                \
        }                                                                                       \
    } while (0)

#define R3DG_CHECK_LAUNCH(debug, stream)                                                        \
    do {                                                                                        \
        R3DG_CHECK_HIP(hipGetLastError());                                                      \
        if (debug) R3DG_CHECK_HIP(hipStreamSynchronize(stream));                                \
    } while (0)

#define R3DG_REQUIRE(cond, msg)                                                                 \
    do {                                                                                        \
        if (!(cond)) {                                                                          \
            ::r3dg::set_error(msg);                                                             \
            return R3DG_ERR_ARG;                                                                \
        }                                                                                       \
    } while (0)

// ---- device math -----------------------------------------------------------------------------
__device__ __forceinline__ float ndc2pix(float v, int S) {
    // auxiliary.h:41-44 evaluates in double (the literals are double)
    return (float)((((double)v + 1.0) * S - 1.0) * 0.5);
}

__device__ __forceinline__ void get_rect(float px, float py, int max_radius, int gx, int gy, int& x0, int& y0,
                                         int& x1, int& y1) {
    // auxiliary.h:46-56
    x0 = min(gx, max(0, (int)((px - (float)max_radius) / kTileX)));
    y0 = min(gy, max(0, (int)((py - (float)max_radius) / kTileY)));
    x1 = min(gx, max(0, (int)((px + (float)max_radius + kTileX - 1) / kTileX)));
    y1 = min(gy, max(0, (int)((py + (float)max_radius + kTileY - 1) / kTileY)));
}

__device__ __forceinline__ float3 xform_point4x3(float3 p, const float* m) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}

__device__ __forceinline__ float4 xform_point4x4(float3 p, const float* m) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// Wave-wide sum over 64 lanes with DPP (result valid in lane 63).

template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND = false>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, BANK_MASK, BOUND));
}

__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    v += dpp_mov<0xB1>(v);          // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);          // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);         // row_half_mirror
    v += dpp_mov<0x140>(v);         // row_mirror        -> every lane: its 16-lane row sum
    v += dpp_mov<0x142, 0xA>(v);    // row_bcast:15      -> rows 1,3 += row 0,2
    v += dpp_mov<0x143, 0xC>(v);    // row_bcast:31      -> rows 2,3 += lane 31
    return v;                       // lane 63 holds the total
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Copies of a workgroup's contiguous span of n floats (float4 accesses when 16-byte aligned) between global memory and
// an LDS layout: float4 global accesses, kCopyU of them in flight per thread before the LDS side
// (the per-Gaussian kernels' SH staging; one dword per access kept 8 loads in flight). put(f, v) /
// get(f) map element f to its LDS slot.
constexpr int kCopyU = 6;
// floor(f / d) by one multiply-high, m = fastdiv_magic(d) = ceil(2^32 / d): exact while f * d < 2^32
// (the SH staging: f < 256 * d, d = 3 M < 4096). The copies below map every element through such a
// quotient; a plain `/` by a runtime divisor is a ~15-instruction sequence per element (round 5:
// half the VALU of the gather and preprocess kernels).
__host__ __device__ inline uint32_t fastdiv_magic(uint32_t d) { return d > 1 ? 0xFFFFFFFFu / d + 1u : 0u; }
__device__ __forceinline__ int fastdiv(int f, uint32_t m) { return m ? (int)__umulhi((uint32_t)f, m) : f; }
template <int BT, class F>
__device__ __forceinline__ void block_load4(const float* __restrict__ src, int n, int t, F&& put) {
    const int n4 = (reinterpret_cast<uintptr_t>(src) & 15u) ? 0 : n >> 2;  // unaligned: dword copies
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int b = t; b < n4; b += BT * kCopyU) {
        float4 v[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int i = b + u * BT;
            v[u] = i < n4 ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int i = b + u * BT;
            if (i < n4) {
                put(4 * i, v[u].x);
                put(4 * i + 1, v[u].y);
                put(4 * i + 2, v[u].z);
                put(4 * i + 3, v[u].w);
            }
        }
    }
    for (int f = 4 * n4 + t; f < n; f += BT) put(f, src[f]);
}
template <int BT, class F>
__device__ __forceinline__ void block_store4(float* __restrict__ dst, int n, int t, F&& get) {
    const int n4 = (reinterpret_cast<uintptr_t>(dst) & 15u) ? 0 : n >> 2;  // unaligned: dword copies
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i = t; i < n4; i += BT) d4[i] = make_float4(get(4 * i), get(4 * i + 1), get(4 * i + 2), get(4 * i + 3));
    for (int f = 4 * n4 + t; f < n; f += BT) dst[f] = get(f);
}

typedef float floatx4 __attribute__((ext_vector_type(4)));  // MFMA accumulator fragment
typedef float f32x2 __attribute__((ext_vector_type(2)));    // packed fp32 pair (v_pk_* ops)

// Exponent of the 2D Gaussian at offset (dx, dy) from its centre: -0.5 (a dx^2 + c dy^2) - b dx dy
// (forward.cu:468, backward.cu:526). The reference's nvcc build contracts this expression into
// FMAs (fmad is on by default; the pattern is the compiler's choice); here one fixed FMA
// pattern, restated operation for operation by the oracle (oracle/r3dg_oracle.c gauss_power), so
// every call site -- forward, backward, either instance of an unrolled pair -- and the oracle
// produce the same bits, and the `power > 0` test resolves identically everywhere. `co` is the
// STAGED conic of the render records, (A, B, C) = (-a/2, -b, -c/2) (exact scalings, written by
// preprocess_kernel): power = dx (A dx + B dy) + C dy^2, five operations after the two offsets
// (round 4's pattern on (a, b, c) took seven).
__device__ __forceinline__ float gauss_power(float4 co, float dx, float dy) {
#pragma clang fp contract(off)
    const float f = __builtin_fmaf(co.x, dx, co.y * dy);
    return __builtin_fmaf(dx, f, (co.z * dy) * dy);
}
// (a, b, c, opacity) of a staged conic (exact)
__device__ __forceinline__ float4 unstage_conic(float4 co) {
    return make_float4(-2.0f * co.x, -co.y, -2.0f * co.z, co.w);
}

// The blend's exp (forward.cu:477 / backward.cu:527 `exp(power)`, i.e. CUDA expf: <= 2 ulp,
// implementation-defined bits). One bit-reproducible f32 statement shared with the oracle
// (oracle/r3dg_oracle.c r3dg_expf, the same operations in the same order): k = rint(x / ln2)
// by the 1.5 * 2^23 shift, Cody-Waite reduction r = x - k ln2 (ln2 split 16 + 24 bits, both
// products exact / singly rounded by the FMAs), degree-6 polynomial for e^r with 1 + r exact,
// scaling by 2^k as an integer add to the exponent field (the shifted kf carries k in its low
// bits and (0x4B400000 << 23) == 0 mod 2^32). Max error 0.90 ulp over every float in [-80, 0],
// correctly rounded on 99.54 % of them (tests/test_oracle.py pins the oracle's copy). Inputs
// clamp to [-80, 0]: every consumer has power <= 0, and e^-80 lies far below the alpha
// threshold. With it, alpha -- and so T, the early stop and n_contrib -- are bit-identical to
// the oracle's (tests/test_gpu_parity.py asserts n_contrib equal).
__device__ __forceinline__ float r3dg_expf(float x) {
#pragma clang fp contract(off)
    x = __builtin_amdgcn_fmed3f(x, -80.0f, 0.0f);
    const float kf = __builtin_fmaf(x, 0x1.715476p+0f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = __builtin_fmaf(k, -0x1.62e400p-1f, x);
    r = __builtin_fmaf(k, -0x1.7f7d1cp-20f, r);
    float p = 0x1.6a959cp-10f;
    p = __builtin_fmaf(p, r, 0x1.123a0ap-7f);
    p = __builtin_fmaf(p, r, 0x1.555850p-5f);
    p = __builtin_fmaf(p, r, 0x1.555492p-3f);
    p = __builtin_fmaf(p, r, 0x1.fffffcp-2f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return __uint_as_float(__float_as_uint(p) + (__float_as_uint(kf) << 23));
}

// The render equation's exp (render_equation.cu:151 / :351 `expf(sharp * (h_d_n - 1))`: the
// argument reaches -2e7 at the roughness floor and a few ulp above 0 when |h|·|n| rounds above 1).
// r3dg_expf's operations over [-87, 88] -- where p·2^k stays a normal float, so the exponent add
// is exact -- and 0 below -87 (e^-87 = 1.6e-38: the reference's denormal results differ from 0 by
// less than amp · 2^-126). Restated by oracle/r3dg_oracle.c r3dg_expf_wide.
__device__ __forceinline__ float r3dg_expf_wide(float x) {
#pragma clang fp contract(off)
    if (x < -87.0f) return 0.0f;
    x = fminf(x, 88.0f);
    const float kf = __builtin_fmaf(x, 0x1.715476p+0f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = __builtin_fmaf(k, -0x1.62e400p-1f, x);
    r = __builtin_fmaf(k, -0x1.7f7d1cp-20f, r);
    float p = 0x1.6a959cp-10f;
    p = __builtin_fmaf(p, r, 0x1.123a0ap-7f);
    p = __builtin_fmaf(p, r, 0x1.555850p-5f);
    p = __builtin_fmaf(p, r, 0x1.555492p-3f);
    p = __builtin_fmaf(p, r, 0x1.fffffcp-2f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return __uint_as_float(__float_as_uint(p) + (__float_as_uint(kf) << 23));
}

// sin and cos of the Fibonacci sample angle (render_equation.cu:93-94 `cosf(theta)`, `sinf(theta)`;
// CUDA's are implementation-defined to 2 ulp). One bit-reproducible f32 statement shared with the
// oracle (oracle/r3dg_oracle.c r3dg_sincosf): k = rint(x · 2/π) by the 1.5 · 2^23 shift,
// three-term Cody-Waite reduction r = x - k·π/2 (π/2 = C1 + C2 + C3, each product singly rounded
// by an FMA), the Cephes minimax polynomials for sin / cos on [-π/4, π/4], quadrant k mod 4.
// |x| < 2^15 (angles reach 2.4 · Ns + 2π).
__device__ __forceinline__ void r3dg_sincosf(float x, float* s_out, float* c_out) {
#pragma clang fp contract(off)
    const float kf = __builtin_fmaf(x, 0x1.45f306p-1f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = __builtin_fmaf(k, -0x1.921fb6p+0f, x);
    r = __builtin_fmaf(k, 0x1.777a5cp-25f, r);
    r = __builtin_fmaf(k, 0x1.ee59dap-50f, r);
    const float r2 = r * r;
    float ps = __builtin_fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f);
    ps = __builtin_fmaf(ps, r2, -1.6666654611e-1f);
    const float sn = __builtin_fmaf(ps * r2, r, r);
    float pc = __builtin_fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f);
    pc = __builtin_fmaf(pc, r2, 4.166664568298827e-2f);
    const float cs = __builtin_fmaf(pc * r2, r2, __builtin_fmaf(-0.5f, r2, 1.0f));
    const unsigned q = __float_as_uint(kf) & 3u;
    const float a = (q & 1u) ? cs : sn, b = (q & 1u) ? sn : cs;
    *s_out = (q & 2u) ? -a : a;
    *c_out = ((q + 1u) & 2u) ? -b : b;
}

// r3dg_expf on two values with packed f32 ops (v_pk_fma_f32 / v_pk_add_f32): per component the
// same IEEE operations in the same order, so each result is bit-identical to r3dg_expf.
__device__ __forceinline__ f32x2 r3dg_expf2(float x0, float x1) {
#pragma clang fp contract(off)
    const f32x2 x = {__builtin_amdgcn_fmed3f(x0, -80.0f, 0.0f), __builtin_amdgcn_fmed3f(x1, -80.0f, 0.0f)};
    const f32x2 sh = {0x1.8p+23f, 0x1.8p+23f};
    const f32x2 kf = __builtin_elementwise_fma(x, f32x2{0x1.715476p+0f, 0x1.715476p+0f}, sh);
    const f32x2 k = kf - sh;
    f32x2 r = __builtin_elementwise_fma(k, f32x2{-0x1.62e400p-1f, -0x1.62e400p-1f}, x);
    r = __builtin_elementwise_fma(k, f32x2{-0x1.7f7d1cp-20f, -0x1.7f7d1cp-20f}, r);
    f32x2 p = {0x1.6a959cp-10f, 0x1.6a959cp-10f};
    p = __builtin_elementwise_fma(p, r, f32x2{0x1.123a0ap-7f, 0x1.123a0ap-7f});
    p = __builtin_elementwise_fma(p, r, f32x2{0x1.555850p-5f, 0x1.555850p-5f});
    p = __builtin_elementwise_fma(p, r, f32x2{0x1.555492p-3f, 0x1.555492p-3f});
    p = __builtin_elementwise_fma(p, r, f32x2{0x1.fffffcp-2f, 0x1.fffffcp-2f});
    p = __builtin_elementwise_fma(p, r, f32x2{1.0f, 1.0f});
    p = __builtin_elementwise_fma(p, r, f32x2{1.0f, 1.0f});
    return f32x2{__uint_as_float(__float_as_uint(p.x) + (__float_as_uint(kf.x) << 23)),
                 __uint_as_float(__float_as_uint(p.y) + (__float_as_uint(kf.y) << 23))};
}

// Fast approximate exp for the backward's gradient values (v_exp_f32 on x * log2 e; ~4e-7
// relative at |x| <= 6). Decisions never rest on it alone: see alpha_ok_bwd.
__device__ __forceinline__ float fast_expf(float x) {
    return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
}

// The reference's alpha test `alpha < 1/255` (forward.cu:478, backward.cu:529) for the backward,
// which must skip exactly the instances the forward skipped. oG = opacity * fast_expf(power);
// its relative error is < 1e-6 for any alpha near the threshold (power >= ln(1/255) there), so
// away from a 4e-6 band the decision equals the exact one; inside the band the step re-evaluates
// with r3dg_expf (rare; one wave-uniform branch). Returns the exact-decision G.
__device__ __forceinline__ float settle_threshold(float power, float opacity, float G) {
#ifdef R3DG_HWEXP
    return G;
#endif
    const bool near = fabsf(__builtin_fmaf(opacity * G, 255.0f, -1.0f)) < 4e-6f;
#ifndef R3DG_NOSETTLE
    if (__builtin_expect(__ballot(near) != 0ull, 0)) {
        if (near) G = r3dg_expf(power);
    }
#else
    (void)near;
#endif
    return G;
}

// The blend's G = exp(power) in the forward kernels. Default: the shared bit-reproducible
// r3dg_expf (n_contrib / final_T bit-exact against the oracle). R3DG_HWEXP (experiment build,
// DESIGN.md §4): the hardware v_exp_f32 on power * log2(e) -- the backward's fast_expf, so forward
// and backward take identical alpha decisions without the backward's settle step, but the bits are
// not the oracle's (v_exp_f32 is not correctly rounded: tools/probe/vexp_cr.hip).
__device__ __forceinline__ float blend_expf(float x) {
#ifdef R3DG_HWEXP
    return fast_expf(x);
#else
    return r3dg_expf(x);
#endif
}

// settle_threshold for a pair of steps with one wave-uniform branch.
__device__ __forceinline__ void settle_threshold2(float pw0, float o0, float& G0, float pw1, float o1, float& G1) {
#ifdef R3DG_HWEXP
    return;  // the forward used the same fast_expf: its decisions are these
#endif
    const bool n0 = fabsf(__builtin_fmaf(o0 * G0, 255.0f, -1.0f)) < 4e-6f;
    const bool n1 = fabsf(__builtin_fmaf(o1 * G1, 255.0f, -1.0f)) < 4e-6f;
    if (__builtin_expect(__ballot(n0 || n1) != 0ull, 0)) {
        if (n0) G0 = r3dg_expf(pw0);
        if (n1) G1 = r3dg_expf(pw1);
    }
}

// Minimum of Q(d) = a dx^2 + 2b dx dy + c dy^2 (positive definite) over mean - pixel offsets with
// the pixel in the rectangle [xa, xb] x [ya, yb]: 0 if the mean lies inside, else the smallest of
// the four edge minima (each a clamped 1-D convex quadratic).
__device__ __forceinline__ float qform_min_rect(float a, float b, float c, float ia, float ic, float mx, float my,
                                                float xa, float xb, float ya, float yb) {
    if (mx >= xa && mx <= xb && my >= ya && my <= yb) return 0.0f;
    auto q = [&](float dx, float dy) { return a * dx * dx + 2.0f * b * dx * dy + c * dy * dy; };
    auto edge_x = [&](float px) {  // pixel column fixed
        const float dx = mx - px;
        const float dy = fminf(fmaxf(-b * dx * ic, my - yb), my - ya);
        return q(dx, dy);
    };
    auto edge_y = [&](float py) {  // pixel row fixed
        const float dy = my - py;
        const float dx = fminf(fmaxf(-b * dy * ia, mx - xb), mx - xa);
        return q(dx, dy);
    };
    return fminf(fminf(edge_x(xa), edge_x(xb)), fminf(edge_y(ya), edge_y(yb)));
}

// Cull margin on the threshold t = 2 ln(255 o) of Q = -2 power: t (1 + m) + m + e * Mmax.
// (1 + m) + m (m = 0.01) absorbs the exp / log errors (r3dg_expf <= 0.9 ulp, __logf). The term
// e * Mmax absorbs the fp32 rounding of Q itself: the blend's gauss_power rounds ~7 times and the
// cull's own minimum ~5 times, each error bounded by 2^-24 times the term magnitudes
// |a| dx^2 + 2 |b dx dy| + |c| dy^2 <= (|a| + |b|) dx^2 + (|c| + |b|) dy^2, whose maximum over the
// quadrant rectangle is Mmax. For compact splats Mmax is small and the term vanishes; for large,
// needle-shaped splats far from their mean the terms reach ~1e6 and cancel to a few units, and the
// term keeps the cull conservative there (tests/test_gpu_parity.py test_cull_exact_needles:
// cull on == off bit for bit on 1920x1080 needles with sigma up to 1000 px). Round 1 used m = 0.1.
#ifndef R3DG_CULL_MARGIN
#define R3DG_CULL_MARGIN 0.01f
#endif
#ifndef R3DG_CULL_REL
#define R3DG_CULL_REL 1e-6f  // e: 16 * 2^-24 rounded up
#endif
// Forward blend: read a staged attribute row's last float4 whole even when its last channel is
// padding (S = 11: 15 channels), so it is one ds_read_b128 rather than a ds_read_b96 (twice the
// LDS-array cycles, MI355X_MICROARCH.md §LDS): render_fwd 0.515 -> 0.507 ms at M1 (three same-box
// pairs, profiles/r06/b128_prio_ab; the backward measured +0.4 % with it and keeps the b96).
// 0 restores the narrow read (experiment builds).
#ifndef R3DG_ATTR_B128
#define R3DG_ATTR_B128 1
#endif

// Is min Q over the pixel rectangle [xa, xb] x [ya, yb] above t (1 + m) + m + e * Mmax, i.e. does
// alpha = o exp(-Q/2) stay below 1/255 at every pixel of the rectangle, in the blend's own fp32
// arithmetic? (a, b, c) = conic, (mx, my) = mean, lt = 2 ln(255 o).
__device__ __forceinline__ bool rect_culled(float4 co, float mx, float my, float xa, float xb, float ya,
                                            float yb) {
    const float ia = __builtin_amdgcn_rcpf(co.x), ic = __builtin_amdgcn_rcpf(co.z);
    const float qmin = qform_min_rect(co.x, co.y, co.z, ia, ic, mx, my, xa, xb, ya, yb);
    const float dxa = mx - xa, dxb = mx - xb, dya = my - ya, dyb = my - yb;
    const float ab = fabsf(co.y);
    const float mmax = (co.x + ab) * fmaxf(dxa * dxa, dxb * dxb) + (co.z + ab) * fmaxf(dya * dya, dyb * dyb);
    const float t = 2.0f * __logf(255.0f * co.w) * (1.0f + R3DG_CULL_MARGIN) + R3DG_CULL_MARGIN +
                    R3DG_CULL_REL * mmax;
    return qmin > t;  // false for a NaN / infinite bound: keep
}

// The exact per-quadrant cull: may alpha = o exp(-Q/2) reach 1/255 anywhere in the 8x8 quadrant with
// top-left pixel (qx, qy) (rect_culled's margin), so a dropped instance fails the reference's alpha
// test on every pixel of the quadrant (tests/test_gpu_parity.py: cull on == off bitwise). Takes the
// render record's staged conic (gauss_power).
__device__ __forceinline__ bool quadrant_live(float2 xy, float4 staged, float qx, float qy, int cull) {
    if (!cull) return true;
    const float4 co = unstage_conic(staged);
    if (co.w < 1.0f / 255.0f) return false;
    const float det = co.x * co.z - co.y * co.y;
    if (!(det > 0.0f) || !(co.x > 0.0f) || !(co.z > 0.0f)) return true;
    return !rect_culled(co, xy.x, xy.y, qx, qx + 7.0f, qy, qy + 7.0f);
}

// quadrant_live for the quadrant's two 8x4 halves (rows qy..qy+3, qy+4..qy+7): the threshold, the
// conic's reciprocals and Mmax over the whole quadrant (an upper bound of each half's: still
// conservative) are shared; the form's minimum is taken over each half's rectangle.
// The rectangle's edges come in wave-uniform (SGPR: readfirstlane by the caller), so they cost
// no VGPRs in the 64-VGPR forward.
__device__ __forceinline__ float uniform_f(float x) {
    return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(x)));
}
__device__ __forceinline__ void half_live(float2 xy, float4 staged, float xa, float xb, float ya, float ym0,
                                          float ym1, float yb, int cull, bool& top, bool& bot) {
    top = bot = true;
    if (!cull) return;
    const float4 co = unstage_conic(staged);
    if (co.w < 1.0f / 255.0f) {
        top = bot = false;
        return;
    }
    const float det = co.x * co.z - co.y * co.y;
    if (!(det > 0.0f) || !(co.x > 0.0f) || !(co.z > 0.0f)) return;
    const float mx = xy.x, my = xy.y;
    const float ia = __builtin_amdgcn_rcpf(co.x), ic = __builtin_amdgcn_rcpf(co.z);
    const float dxa = mx - xa, dxb = mx - xb, dya = my - ya, dyb = my - yb;
    const float ab = fabsf(co.y);
    const float mmax = (co.x + ab) * fmaxf(dxa * dxa, dxb * dxb) + (co.z + ab) * fmaxf(dya * dya, dyb * dyb);
    const float t = 2.0f * __logf(255.0f * co.w) * (1.0f + R3DG_CULL_MARGIN) + R3DG_CULL_MARGIN +
                    R3DG_CULL_REL * mmax;
    top = !(qform_min_rect(co.x, co.y, co.z, ia, ic, mx, my, xa, xb, ya, ym0) > t);
    bot = !(qform_min_rect(co.x, co.y, co.z, ia, ic, mx, my, xa, xb, ym1, yb) > t);
}

}  // namespace r3dg

namespace r3dg {
// Decoupled look-back by one wave (single-pass scans, rasterizer.hip scan_touched_kernel /
// preprocess.hip bin_colscan_kernel): the exclusive prefix of workgroup b from the 64-bit status
// words of its predecessors ([flag: 62-63 | value: 0-31], flag 1 = the workgroup's aggregate, 2 = its
// inclusive prefix, 0 = not published yet). Lane k polls predecessor b - 1 - k, so a window of 64
// predecessors costs one round of device-scope loads (each one crosses the XCDs' L2s): the window
// is summed up to its nearest inclusive prefix once every word up to it is published, else polled
// again. Called by all 64 lanes of one wave; returns the prefix in every lane.
__device__ __forceinline__ uint32_t lookback_prefix(const uint64_t* status, int b) {
    const int l = threadIdx.x & 63;
    uint32_t prefix = 0;
    int hi = b;  // predecessors [0, hi) not summed yet
    while (hi > 0) {
        const int p = hi - 1 - l;
        const uint64_t s = p >= 0 ? __hip_atomic_load(status + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                  : (2ull << 62);  // before workgroup 0: an inclusive prefix of 0
        const uint32_t flag = (uint32_t)(s >> 62);
        const unsigned long long incl = __ballot(flag == 2u), ready = __ballot(flag != 0u);
        const int stop = incl ? (int)__builtin_ctzll(incl) : 63;  // the nearest inclusive prefix, or the window
        const unsigned long long need = stop == 63 ? ~0ull : ((2ull << stop) - 1ull);
        if ((ready & need) != need) continue;  // a word up to it is not published yet: poll again
        uint32_t v = l <= stop ? (uint32_t)s : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
        prefix += v;
        if (incl) break;
        hi -= 64;
    }
    return prefix;
}
}  // namespace r3dg
