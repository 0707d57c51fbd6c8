// render_bwd.hip -- backward of the tile blend and of the per-Gaussian preprocessing (gfx950).
//
// Restates reference backward.cu:401-614 (renderCUDA backward), :144-276 (computeCov2DCUDA),
// :20-139 (SH backward), :280-343 (cov3D backward), :348-398 (preprocessCUDA backward).
//
// MI355X design (replaces the reference's per-pixel float atomicAdd scatter, ~(10+S) atomics
// per contributing pixel, backward.cu:552-611):
//   1. render_bwd_glds_kernel: one workgroup per tile (longest tiles first) replays the forward's
//      per-quadrant contribution lists back to front, the render records LDS-DMA-staged one batch
//      ahead; wave w owns the tile's 8x8 quadrant w. Per visited (instance, wave) pair a predicated
//      blend step yields two per-pixel scalars w = alpha*T and q = G*dL/dalpha; a wave's 64-pixel
//      reductions of 13 instances are bf16-split MFMA products (w x [colour, feature, depth grads],
//      q x pixel moments about the quadrant centre). Default (ATOM): each (instance, wave) row is
//      expanded about the Gaussian's mean in the lanes and added into the per-Gaussian sums
//      [P, SRS] with no-return atomics (X part f32, the six moments expanded and summed in f64) --
//      the reference's accumulation at 1/64 of its atomics; the last bits of the X part depend on
//      the atomics' arrival order, as the reference's do. w is split into
//      two bf16 terms (|w - h - m| <= 2^-16 |w|), q into three (exact).
//      R3DG_BWD_REDUCE=rows (!ATOM): one partial row per (instance, quadrant) at 4 * slot +
//      quadrant, flagged, summed by
//   2. row_sum_kernel: one 8-lane group per Gaussian sums its flagged partial rows (contiguous:
//      slots are Gaussian-major, duplicateWithKeys order) in a fixed order and expands the
//      quadrant-centred moments -- bitwise reproducible run to run.
//      render_bwd_dpp_kernel (R3DG_BWD=dpp) is the DPP-reduction cross-check writing the same rows.
//   3. gather_bwd_kernel: one thread per Gaussian expands the sums into the mean2D / conic / opacity
//      gradients and runs the cov2D / projection / SH / cov3D backward.
#include "r3dg_common.h"
#include "r3dg_kernels.h"

namespace r3dg {

#ifdef R3DG_EXP_COUNT
R3DG_EXP_READER(r3dg_exp_counters_bwd)
#endif

__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Pixel setup shared by both variants: lane l of wave w owns pixel (l & 7, l >> 3) of the tile's
// 8x8 quadrant w; the upstream gradients of that pixel.
#define R3DG_BWD_PIXEL_SETUP()                                                                          \
    const int tile = block_tile(a.tile_order, a.num_tiles);                                             \
    if (tile >= a.num_tiles) return;                                                                    \
    const int t = threadIdx.x, w = t >> 6, l = t & 63;                                                  \
    R3DG_BWD_PIXELS()

// Pixel (l & 7, l >> 3) of quadrant w of `tile` and its upstream gradients (tile, w, l defined).
#define R3DG_BWD_PIXELS()                                                                               \
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;                                               \
    const int px = tx * kTileX + (w & 1) * 8 + (l & 7);                                                 \
    const int py = ty * kTileY + (w >> 1) * 8 + (l >> 3);                                               \
    const bool inside = px < a.W && py < a.H;                                                           \
    const int pix = inside ? py * a.W + px : 0;                                                         \
    const float pfx = (float)px, pfy = (float)py;                                                       \
    const uint2 range = a.ranges[tile];                                                                 \
    const int S = a.S;                                                                                  \
    const float T_final = inside ? a.final_T[pix] : 0.f;                                                \
    const int last = inside ? (int)a.n_contrib[pix] : 0;                                                \
    float g[3], gf[SMAX > 0 ? SMAX : 1], gd = 0.f, go = 0.f;                                            \
    _Pragma("unroll") for (int c = 0; c < 3; ++c) g[c] = inside ? a.dL_dpix[a.ca[c] + pix * a.cm[c]] : 0.f; \
    _Pragma("unroll") for (int c = 0; c < SMAX; ++c) gf[c] =                                            \
        (inside && c < S) ? a.dL_dpix_f[a.gflay.a[c] + pix * a.gflay.m[c]] : 0.f;                       \
    if (inside) {                                                                                       \
        gd = a.dL_dpix_d[pix];                                                                          \
        go = a.dL_dpix_o[pix];                                                                          \
    }                                                                                                   \
    const float bg_dot = a.bg[0] * g[0] + a.bg[1] * g[1] + a.bg[2] * g[2];

// Block-wide max of n_contrib: tile positions >= it are never blended (and never staged).
__device__ __forceinline__ int block_max_last(int wmax, int* s_max_last) {
    if (threadIdx.x == 0) *s_max_last = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(s_max_last, wmax);
    __syncthreads();
    return *s_max_last;
}

// One wave's pixel moments of q, sum q * [1, x, y, x^2, xy, y^2] with (x, y) = pixel - quadrant
// centre, expanded about the Gaussian's mean ("expand_moments"): with (d0x, d0y) = mean - quadrant
// centre the pixel's offset from the mean is (d0x - x, d0y - y), so
//   sum q dx = d0x S0 - Sx,  sum q dx^2 = d0x^2 S0 - 2 d0x Sx + Sxx,  sum q dx dy = d0x d0y S0 - d0x Sy
//   - d0y Sx + Sxy  (and y alike): the partial row's moments (r3dg_kernels.h), what
// backward.cu:583-611 sums per pixel through dG/ddelx, dG/ddely and the conic terms. Both
// reductions (the atomic flush and row_sum_kernel) evaluate and sum it in double: for a mean ~1e3
// px from its pixels the terms are ~1e6 times the result.

// DPP variant (cross-check of the MFMA default, R3DG_BWD=dpp): the reference's per-channel
// recurrences (backward.cu:544-579) step by step; every wave reduces its 64 pixels' values of an
// instance with DPP and lane 63 writes the wave's partial row.
template <int SMAX>
__global__ void __launch_bounds__(kBlock) render_bwd_dpp_kernel(RenderBwdArgs a) {
    constexpr int NA4 = (4 + SMAX + 3) / 4;      // attribute row: colour, depth, features
    constexpr int NXB = (4 + SMAX + 15) / 16;
    constexpr int XW = 16 * NXB;
    constexpr int RF4 = 2 + NA4;
    __shared__ float2 s_xy[kBlock];
    __shared__ float4 s_co[kBlock];
    __shared__ uint32_t s_mask[kBlock];
    __shared__ uint32_t s_slot[kBlock];
    __shared__ float4 s_attr[kBlock * NA4];
    __shared__ int s_max_last;

    R3DG_BWD_PIXEL_SETUP()
    float T = T_final;
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    const float xr = (float)(l & 7) - 3.5f, yr = (float)(l >> 3) - 3.5f;  // offset from the quadrant centre
    const float qcx = (float)(tx * kTileX + (w & 1) * 8) + 3.5f, qcy = (float)(ty * kTileY + (w >> 1) * 8) + 3.5f;

    float acc[3] = {0.f, 0.f, 0.f}, acc_f[SMAX > 0 ? SMAX : 1], acc_d = 0.f, acc_o = 0.f;
    float last_alpha = 0.f, last_depth = 0.f, last_color[3] = {0.f, 0.f, 0.f}, last_f[SMAX > 0 ? SMAX : 1];
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
        acc_f[c] = 0.f;
        last_f[c] = 0.f;
    }
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max_int(last));
    const int max_last = block_max_last(wmax, &s_max_last);
    const int RS = a.RS;
    (void)ddelx_dx;
    (void)ddely_dy;

    for (int hi = max_last; hi > 0; hi -= kBlock) {
        const int cnt = min(kBlock, hi);
        __syncthreads();  // previous batch fully consumed before the staging arrays are reused
        if (t < cnt) {
            const uint32_t gid = a.point_list[range.x + (uint32_t)(hi - 1 - t)];
            const float4* rec = a.records + (size_t)gid * RF4;
            const float4 co = rec[0], r1 = rec[1];
            s_xy[t] = make_float2(r1.x, r1.y);
            s_co[t] = co;
            s_slot[t] = record_slot(r1, gid == 0 ? 0u : a.offsets[gid - 1], tx, ty, a.grid_x, a.grid_y);
            s_mask[t] = a.contrib[range.x + (uint32_t)(hi - 1 - t)];  // the forward's contribution bits
#pragma unroll
            for (int q = 0; q < NA4; ++q) s_attr[t * NA4 + q] = rec[2 + q];
        }
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const int p = hi - 1 - j;  // position in the tile range (reference `contributor`)
            if (p >= wmax) continue;   // no pixel of this wave reaches this far back
            const uint32_t m = __builtin_amdgcn_readfirstlane(s_mask[j]);
            if (!((m >> (2 * w)) & 3u)) continue;  // either half of quadrant w (render_fwd.hip)
            bool contrib = inside && p < last;
            float G = 0.f, alpha = 0.f;
            float4 co = make_float4(0.f, 0.f, 0.f, 0.f);
            if (contrib) {
                const float2 xy = s_xy[j];
                co = s_co[j];
                const float power = gauss_power(co, xy.x - pfx, xy.y - pfy);
                if (power > 0.0f) {
                    contrib = false;
                } else {
                    G = settle_threshold(power, co.w, fast_expf(power));
                    alpha = fminf(0.99f, co.w * G);
                    if (alpha < 1.0f / 255.0f) contrib = false;
                }
            }
            if (__ballot(contrib) == 0ull) continue;
            float wv = 0.f, qv = 0.f;
            if (contrib) {
                T = T / (1.f - alpha);
                const float dchannel_dcolor = alpha * T;
                float v[NA4 * 4];
#pragma unroll
                for (int q = 0; q < NA4; ++q) {
                    const float4 r = s_attr[j * NA4 + q];
                    v[4 * q] = r.x; v[4 * q + 1] = r.y; v[4 * q + 2] = r.z; v[4 * q + 3] = r.w;
                }
                float dL_dalpha = 0.0f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    acc[c] = last_alpha * last_color[c] + (1.f - last_alpha) * acc[c];
                    last_color[c] = v[c];
                    dL_dalpha += (v[c] - acc[c]) * g[c];
                }
#pragma unroll
                for (int c = 0; c < SMAX; ++c) {
                    acc_f[c] = last_alpha * last_f[c] + (1.f - last_alpha) * acc_f[c];
                    last_f[c] = v[4 + c];
                    if (a.backward_geometry) dL_dalpha += (v[4 + c] - acc_f[c]) * gf[c];
                }
                acc_d = last_alpha * last_depth + (1.f - last_alpha) * acc_d;
                last_depth = v[3];
                dL_dalpha += (v[3] - acc_d) * gd;
                acc_o = last_alpha + (1.f - last_alpha) * acc_o;
                dL_dalpha += (1.0f - acc_o) * go;
                dL_dalpha *= T;
                last_alpha = alpha;
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                wv = dchannel_dcolor;
                qv = G * dL_dalpha;
            }
            // wave totals (full exec mask here: the j loop is wave-uniform); lane 63 writes the row
            float* row = a.rows + ((size_t)s_slot[j] * 4 + w) * RS;
#pragma unroll
            for (int c = 0; c < 4 + SMAX; ++c) {
                if (c < 4 + S) {
                    const float gc = c < 3 ? g[c] : (c < 3 + S ? gf[c - 3 < SMAX ? c - 3 : 0] : gd);
                    const float sum = wave_sum_to_lane63(wv * gc);
                    if (l == 63) row[c] = sum;
                }
            }
            const float mv[6] = {qv, qv * xr, qv * yr, qv * xr * xr, qv * xr * yr, qv * yr * yr};
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const float sum = wave_sum_to_lane63(mv[k]);
                if (l == 63) row[XW + k] = sum;
            }
            if (l == 63) {
                row[XW + 6] = qcx;
                row[XW + 7] = qcy;
            }
            if (l == 63) a.flags[(size_t)s_slot[j] * 4 + w] = 1;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// MFMA variant of the backward blend (default).
//
// Every per-pixel contribution of one instance is linear in two per-pixel scalars:
//   w = alpha*T          -> colour (w*g_c), feature (w*gf_c) and depth (w*gd) gradients;
//   q = G*dL_dalpha      -> opacity (q), and mean2D / conic gradients through the moments
//                           sum q * {1, x, y, x^2, xy, y^2} of quadrant-centred pixel offsets
//                           (expanded about the Gaussian's mean by the gather kernel).
// So a wave's reduction over its 64 pixels for 16 instances is two matrix products,
// W[16 inst x 64 px] @ X[64 px x 16 ch] and Q[16 inst x 64 px] @ Y[64 px x 16 (6 used)], each 16
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains). w and q rows go through a per-wave LDS image,
// XOR-swizzled so the row-wise writes and the column-wise A-operand reads are conflict-free.
//
// Waves are independent between staging barriers: each writes its own partial row per
// (instance, quadrant) straight from the MFMA accumulators -- no cross-wave reduction, no
// per-chunk barriers -- and an MFMA group fills across the whole staged batch.
// ---------------------------------------------------------------------------------------------

// Order this wave's LDS traffic for cross-lane exchange through LDS: wait for the wave's DS
// operations and stop the compiler from moving memory accesses across (it cannot see lanes).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Tuning knobs (experiment builds override them through R3DG_EXTRA_HIPFLAGS). Occupancy is set
// by LDS and VGPRs together; the LDS allocation is rounded up in 2 KiB steps.
typedef float f32x2 __attribute__((ext_vector_type(2)));
#ifndef R3DG_BWD_WAVES
#define R3DG_BWD_WAVES 3  // waves per SIMD the register allocation targets (SMAX <= 12). The kernel
                          // takes 125 VGPRs either way and runs 4 waves per SIMD (LDS: 4 blocks per
                          // CU); the target of 3 only changes the scheduler's latency / pressure
                          // trade-off: render_bwd -0.4 % at M1 (4 pairs), -0.8 % at C3, round 5
#endif

// w|q image: row r (0..15 w, 16..31 q) of 64 pixels, padded stride WQS = 66 floats; pixel c of
// row r at r*WQS + c. ds_read_b32 / ds_write_b32 bank by dword address mod 32 within each 32-lane
// half (MI355X_MICROARCH.md §LDS): a row write is 32 consecutive dwords per half, and an
// A-operand read (lane l: row l&15, pixel 4*s + (l>>4)) hits bank 2*(l&15) + (l>>4) + 4s (mod 32),
// 32 distinct banks per half -- both conflict-free (stride 64 or 68 would be 16- / 2-way) -- and a
// write address is the lane base plus a wave-uniform row offset.
constexpr int WQS = 66;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Exact bf16 splits by truncation: h = the top 8 significant bits of x (its upper 16 bits), r = x - h
// exact in f32 (<= 16 significant bits), m = the top 8 significant bits of r, o = r - m exact and
// <= 8 significant bits, so x = h + m + o EXACTLY and h*y + m*y + o*y with y exact in bf16 (the
// pixel moments 1, x, y, x^2, xy, y^2 of half-integer offsets are) gives the f32 product. Per value
// two v_and + two v_sub, and per value pair one v_perm_b32 per term packing the two upper halves
// (round-to-nearest conversions cost 3.5 v_cvt_pk_bf16_f32 + 2 shifts + 2 subs per value).
union bf16x8_u {
    bf16x8 v;
    uint32_t u[4];
};
__device__ __forceinline__ uint32_t hi16_pair(uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_perm(hi, lo, 0x07060302u);  // [lo.upper16 | hi.upper16]
}
__device__ __forceinline__ void split_bf16x3(const float (&x)[8], bf16x8& h, bf16x8& m, bf16x8& o) {
    uint32_t ux[8], ur[8], uo[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        ux[i] = __float_as_uint(x[i]);
        const float r = x[i] - __uint_as_float(ux[i] & 0xffff0000u);
        ur[i] = __float_as_uint(r);
        uo[i] = __float_as_uint(r - __uint_as_float(ur[i] & 0xffff0000u));
    }
    bf16x8_u H, M, O;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        H.u[k] = hi16_pair(ux[2 * k], ux[2 * k + 1]);
        M.u[k] = hi16_pair(ur[2 * k], ur[2 * k + 1]);
        O.u[k] = hi16_pair(uo[2 * k], uo[2 * k + 1]);
    }
    h = H.v;
    m = M.v;
    o = O.v;
}

#ifndef R3DG_BWD_SPLIT
#define R3DG_BWD_SPLIT 2  // bf16 terms per f32 value of w (= alpha T: colour / feature / depth grads)
                          // in the flush's MFMA products: 2 = h + m, |x - h - m| <= 2^-16 |x|
                          // unbiased; 3 = exact f32 products
#endif
#ifndef R3DG_BWD_SPLIT_Q
#define R3DG_BWD_SPLIT_Q 3  // the same for q = G dL/dalpha (the moments behind the mean2D / conic /
                            // opacity grads): exact, as the conic inverse amplifies their errors by up
                            // to ~1e6 on needle-shaped splats (test_cull_exact_needles: with 2 terms
                            // one needle's dL/dmeans3D left the fp32 sensitivity bound 88x)
#endif

// x = h + m to within 2^-16 |x|: h the truncated top 8 significant bits (v_and + v_perm per pair),
// m = x - h (exact) rounded to nearest bf16 (one v_cvt_pk_bf16_f32 per pair), so the residual is
// unbiased (a truncated m would shrink every |w| and |q| by up to 2^-14)
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_bf16x2(const float (&x)[8], bf16x8& h, bf16x8& m) {
    uint32_t ux[8];
    float r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        ux[i] = __float_as_uint(x[i]);
        r[i] = x[i] - __uint_as_float(ux[i] & 0xffff0000u);
    }
    bf16x8_u H, M;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        H.u[k] = hi16_pair(ux[2 * k], ux[2 * k + 1]);
        M.u[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v{r[2 * k], r[2 * k + 1]}), bf16x2v));
    }
    h = H.v;
    m = M.v;
}

// the atomic flush's add (timing-only builds swap it: tools/exp_build.sh)
#ifdef R3DG_EXP_ATOMSTORE  // timing experiment only (results invalid): plain stores for the atomics
#define R3DG_FLUSH_ADD(p, v) (*(p) = (v))
#elif defined(R3DG_EXP_NOSTORE)  // timing experiment only (results invalid): the epilogue without its stores
#define R3DG_FLUSH_ADD(p, v) do { if ((v) == 1.2345e-30f) *(p) = 0.f; } while (0)
#else
#define R3DG_FLUSH_ADD(p, v) atomicAdd((p), (v))
#endif
#ifndef R3DG_BWD_SWALK
#define R3DG_BWD_SWALK 1  // the pair loop's live-mask walk by s_ff1 + s_bitset0 (inline asm), as the forward's
#endif
#ifndef R3DG_BWD_ORIGIN_MOMENTS
#define R3DG_BWD_ORIGIN_MOMENTS 1  // atomic flush: moments re-centred on the image origin in the D lanes
                                   // (gather_bwd_kernel expands them about the mean); 0: expanded about
                                   // the mean in the flush through LDS tiles (round 5)
#endif
#ifndef R3DG_BWDG_NB
#define R3DG_BWDG_NB 64  // instances per staged batch of the DMA-staged kernel
#endif
#ifndef R3DG_BWDG_GRP
#define R3DG_BWDG_GRP 13  // instances per MFMA group of the DMA-staged kernel (64 / 13 measured best of
                          // 32 / 16, 64 / 12, 64 / 13, 32 / 12: the smaller w|q image buys the larger batch)
#endif

// ---------------------------------------------------------------------------------------------
// The backward blend (default). One 256-thread workgroup per tile (longest tiles first), wave w =
// quadrant w. The render records of batch b+1 are copied HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPRs) while the waves blend batch b, so the record round trip is
// off the critical path and a batch costs one block barrier. A wave visits exactly the staged
// instances that at least one of its pixels blended in the forward: the forward's contribution
// bits (render_fwd.hip, one byte per sorted position, bits 2q, 2q + 1 = the halves of quadrant q), loaded one batch ahead --
// no footprint cull here and no instance without a partial row. The instance's slot comes from
// the lane that loaded its bits (record_slot), so nothing but the records goes through LDS.
// Staging buffer layout: column q (float4 q of the record) of instance t at [q * NB + t].
// ---------------------------------------------------------------------------------------------
// ATOM: the reduction's second stage in the flush itself -- each (instance, wave) row is expanded
// about the Gaussian's mean and added with no-return f32 atomics into the per-Gaussian sums
// [P, SRS] (the reference's own accumulation, backward.cu:552-611, at one atomic per channel per
// (instance, wave) instead of per pixel): no partial rows, no row flags, no row_sum_kernel; sums
// depend on the atomics' arrival order. !ATOM: the deterministic partial rows + row_sum_kernel.
// WS: bf16 terms of w in the X products (R3DG_BWD_SPLIT, default 2); WS = 1 is the one-term
// reduction the gradient parity bar must reject (R3DG_BWD_WTERMS=1, tests/test_gpu_parity.py
// test_one_term_reduction_fails_bar).
template <int SMAX, bool ATOM, int WS = R3DG_BWD_SPLIT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SMAX <= 12 ? R3DG_BWD_WAVES : 1)))
render_bwd_glds_kernel(RenderBwdArgs a) {
    constexpr int NB = R3DG_BWDG_NB;              // instances per batch (two batches staged)
    constexpr int NW = 4;                         // waves per workgroup
    constexpr int NA4 = (4 + SMAX + 3) / 4;
    constexpr int NXB = (4 + SMAX + 15) / 16;
    constexpr int XW = 16 * NXB;
    constexpr int GRP = R3DG_BWDG_GRP;            // instances per MFMA group (<= 16 A rows)
    constexpr int RF4 = 2 + NA4;                  // float4s per render record
    constexpr int NCP = (RF4 * NB + 63) / 64;     // DMA wave-instructions per batch
    constexpr int SBUF = RF4 * NB;                // float4s per staging buffer
    constexpr int WQF4 = 2 * GRP * WQS / 4;       // float4s per wave's w|q image
    static_assert((2 * GRP * WQS) % 4 == 0, "w|q image must be float4-sized");
    static_assert(64 % NB == 0 || NB % 64 == 0, "a DMA wave-instruction covers whole columns");
    static_assert(NB <= 64 && GRP <= 16, "live masks are one ballot; MFMA groups are 16 rows");
    using mask_t = typename std::conditional<(NB > 32), unsigned long long, uint32_t>::type;
    // one LDS array (a second __shared__ object can make the compiler wait for the DMA before
    // unrelated LDS reads): [w|q images | 2 staging buffers | max_last]. With GRP < 16 the MFMA's
    // A reads of rows GRP..15 run past a wave's image into the next image or the staging buffer
    // (valid LDS, values ignored: those D rows are never stored).
    __shared__ float4 s_lds[NW * WQF4 + 2 * SBUF + 1];
    float4* const stage = s_lds + NW * WQF4;

    const int tile = block_tile(a.tile_order, a.num_tiles);
    const int w = threadIdx.x >> 6;
    if (tile >= a.num_tiles) return;
    const int t = threadIdx.x, l = t & 63;
    R3DG_BWD_PIXELS()
    float T = T_final;
    float* wq = reinterpret_cast<float*>(s_lds + w * WQF4);
    int* s_max_last = reinterpret_cast<int*>(stage + 2 * SBUF);

    // B operand of the X products (16x16x32 layout: lane l holds X[pixel 32b + 8(l >> 4) + i][channel
    // l & 15]) as two bf16 terms, X = hi + lo to within 2^-17 |X|
    bf16x8 bXh[NXB][2], bXl[NXB][2];
    {
#pragma unroll
        for (int xb = 0; xb < NXB; ++xb) {
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const int ch = xb * 16 + c;
                float v = 0.f;
                if (ch < 3) v = g[ch];
                else if (ch - 3 < SMAX && ch - 3 < S) v = gf[(ch - 3) < SMAX ? (ch - 3) : 0];
                else if (ch == 3 + S) v = gd;
                wq[c * WQS + l] = v;
            }
            wave_lds_sync();
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float x = wq[(l & 15) * WQS + 32 * b + 8 * (l >> 4) + i];
                    const __bf16 hb = (__bf16)x;
                    bXh[xb][b][i] = hb;
                    bXl[xb][b][i] = (__bf16)(x - (float)hb);
                }
            wave_lds_sync();
        }
    }
    if (!a.backward_geometry) {
#pragma unroll
        for (int c = 0; c < SMAX; ++c) gf[c] = 0.f;
    }
    f32x2 gp[2 * NA4];
#pragma unroll
    for (int c2 = 0; c2 < 2 * NA4; ++c2) {
        float e[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ch = 2 * c2 + h;
            e[h] = ch < 3 ? g[ch] : (ch == 3 ? gd : (ch - 4 < SMAX ? gf[(ch - 4) < SMAX ? ch - 4 : 0] : 0.f));
        }
        gp[c2] = f32x2{e[0], e[1]};
    }
    float u = 0.f;
    const float TFB = T_final * bg_dot;
    const float qcx = (float)(tx * kTileX + (w & 1) * 8) + 3.5f, qcy = (float)(ty * kTileY + (w >> 1) * 8) + 3.5f;
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max_int(last));
    const int max_last = block_max_last(wmax, s_max_last);
    const int RS = a.RS;
    const int nch = l & 15;
    const bool lane0 = l == 0;
    const float4* st = stage;  // staging buffer of the current batch

    auto step = [&](int j, int p, bool live, float opacity, float power, float G, float& wv, float& qv,
                    bool& okv) {
#pragma clang fp contract(off)
        const int ju = __builtin_amdgcn_readfirstlane(j);
        float v[NA4 * 4];
#pragma unroll
        for (int q = 0; q < NA4; ++q) {
            const float4 rr = st[(2 + q) * NB + ju];
            v[4 * q] = rr.x; v[4 * q + 1] = rr.y; v[4 * q + 2] = rr.z; v[4 * q + 3] = rr.w;
        }
        // (the last row stays a ds_read_b96 at S = 11: the forward's whole-float4 read, R3DG_ATTR_B128,
        // measured +0.4 % here, profiles/r06/b128_prio_ab)
        const float alpha = fminf(0.99f, opacity * G);
        const bool ok = live && p < last && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
        okv = ok;
        const float ae = ok ? alpha : 0.f;
        const float Ge = ok ? G : 0.f;
        const float rinv = __builtin_amdgcn_rcpf(1.f - ae);
        const float Tn = T * rinv;
        // the 16-channel dot as two scalar FMA chains (even / odd channels; the packed
        // v_pk_fma_f32 pair computes the same bits but its dependent issue needs s_nop hazards:
        // render_bwd 0.819 -> 0.800 ms with the scalar chains)
        float dx0 = go, dx1 = 0.f;
#pragma unroll
        for (int c2 = 0; c2 < 2 * NA4; ++c2) {
            // (the row's 4 + SMAX real values only: SMAX = 11 skips the pad channel's FMA)
            if (2 * c2 < 4 + SMAX) dx0 = __builtin_fmaf(v[2 * c2], gp[c2].x, dx0);
            if (2 * c2 + 1 < 4 + SMAX) dx1 = __builtin_fmaf(v[2 * c2 + 1], gp[c2].y, dx1);
        }
        const float d = dx0 + dx1;
        const float diff = d - u;
        const float dL_dalpha = rinv * __builtin_fmaf(T, diff, -TFB);
        wv = ae * Tn;
        qv = Ge * dL_dalpha;
        T = Tn;
        u = __builtin_fmaf(ae, diff, u);
    };

    // B operand of the moment products, constant: lane l holds Y[pixel 32b + 8(l >> 4) + i][l & 15]
    // for K-block b (16x16x32 layout), pixel p = (p >> 3) * 8 + (p & 7) about the quadrant centre;
    // exact in bf16 (at most 6 significant bits)
    bf16x8 yb[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = 32 * b + 8 * (l >> 4) + i;
            const float x = (float)(p & 7) - 3.5f, y = (float)(p >> 3) - 3.5f;
            const float v = nch == 0 ? 1.f : nch == 1 ? x : nch == 2 ? y : nch == 3 ? x * x : nch == 4 ? x * y
                          : nch == 5 ? y * y : 0.f;
            yb[b][i] = (__bf16)v;
        }
    // pad lanes of the moment stores: the quadrant centre (row_sum expands the moments about the mean)
    const float cpad = nch == 6 ? qcx : qcy;
    // atomic flush, origin moments: lane column c's re-centring constants (the moment about the image
    // origin G_c = s_c + oka s0 + okb s1 + okc s2; products of half-integers < 2^14: exact in double)
    const double dcx = (double)qcx, dcy = (double)qcy;
    const double oka = nch == 1 ? dcx : nch == 2 ? dcy : nch == 3 ? dcx * dcx : nch == 4 ? dcx * dcy
                     : nch == 5 ? dcy * dcy : 0.0;
    const double okb = nch == 3 ? 2.0 * dcx : nch == 4 ? dcy : 0.0;
    const double okc = nch == 4 ? dcx : nch == 5 ? 2.0 * dcy : 0.0;
    // atomic flush: this lane's column of the per-Gaussian sums, and the row stride in bytes
    float* const lane_sums = a.sums + nch;
    const uint32_t srs = (uint32_t)a.SRS;
    auto flush = [&](int r) {
        if (l == 0) R3DG_EXP_ADD(1, 1);
#ifdef R3DG_EXP_NOFLUSH  // timing experiment only (results invalid): no reduction, no rows
        (void)r;
        return;
#endif
        wave_lds_sync();
        floatx4 accX[NXB], accY = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int xb = 0; xb < NXB; ++xb) accX[xb] = floatx4{0.f, 0.f, 0.f, 0.f};
        // w rows times the upstream gradients on the bf16 MFMA: X = X1 + X2 (two terms), w = h + m
        // (R3DG_BWD_SPLIT = 2, default: m rounded to nearest, three products m X1, h X2, h X1) or
        // w = h + m + o exactly (3: the five products above 2^-24, smallest first)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const float* src = wq + (l & 15) * WQS + 32 * b + 8 * (l >> 4);
            float wv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = src[i];
            bf16x8 h, m, o;
            if constexpr (WS == 1) {  // one term, one product (inexact: the negative parity test)
                split_bf16x2(wv, h, m);
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb)
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bXh[xb][b], accX[xb], 0, 0, 0);
            } else if constexpr (WS == 2) {
                split_bf16x2(wv, h, m);
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb) {
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, bXh[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bXl[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bXh[xb][b], accX[xb], 0, 0, 0);
                }
            } else {
                split_bf16x3(wv, h, m, o);
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb) {
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o, bXh[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, bXl[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, bXh[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bXl[xb][b], accX[xb], 0, 0, 0);
                    accX[xb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, bXh[xb][b], accX[xb], 0, 0, 0);
                }
            }
            (void)o;
        }
        // q rows times the moments on the bf16 MFMA (16 cycles per K = 32, against 32 per K = 4 in
        // f32): three exact-sum bf16 terms of q per K-block
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const float* src = wq + (GRP + (l & 15)) * WQS + 32 * b + 8 * (l >> 4);
            float qv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) qv[i] = src[i];
            bf16x8 h, m, o;
#if R3DG_BWD_SPLIT_Q == 1  // timing experiment only (results inexact)
            split_bf16x2(qv, h, m);
            (void)o;
            (void)m;
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, yb[b], accY, 0, 0, 0);
#elif R3DG_BWD_SPLIT_Q == 2
            split_bf16x2(qv, h, m);
            (void)o;
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, yb[b], accY, 0, 0, 0);
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, yb[b], accY, 0, 0, 0);
#else
            split_bf16x3(qv, h, m, o);
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, yb[b], accY, 0, 0, 0);
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, yb[b], accY, 0, 0, 0);
            accY = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o, yb[b], accY, 0, 0, 0);
#endif
        }
        // Group row r's bookkeeping sits in the pad columns of its w|q image rows (written by lane 0
        // at the visit): the instance's mean (x, y) at w row r, columns 64-65, and its Gaussian
        // (ATOM) or partial row (4 * slot + quadrant) at q row r, column 64. Lane group g handles
        // D rows 4g + i of accumulator element i: one broadcast LDS read per row and value.
        uint32_t rid[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            rid[i] = reinterpret_cast<const uint32_t*>(wq)[(GRP + (l >> 4) * 4 + i) * WQS + 64];
#ifdef R3DG_EXP_NOEPI  // timing experiment only (results invalid): no expansion, no stores
        if (accX[0][0] == 1.2345e-30f && accY[0] == 1.2345e-30f) a.sums[l] = accX[0][1] + accY[1] + rid[0];
        wave_lds_sync();
        return;
#endif
        if constexpr (ATOM && R3DG_BWD_ORIGIN_MOMENTS) {
            // The moments about the quadrant centre re-centred on the image origin in double, in the
            // D registers' own lanes: lane c < 6 of each 16-lane row holds moment c of its rows
            // 4g + i, and G_c = s_c + ka s0 + kb s1 + kc s2 (the wave's constants for column c,
            // X = qcx + x, Y = qcy + y) takes s0, s1, s2 from lanes 0-2 of its row by DPP
            // row_newbcast: no LDS round trip and no per-row mean. gather_bwd_kernel expands the
            // summed origin moments about the Gaussian's mean in double (|X| <= ~8e3 px: the terms
            // are <= ~6e7 times the moments they cancel to, far inside double's 2^-53).
            double ev[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float sv = accY[i];
                const float s0 = __builtin_amdgcn_mov_dpp(sv, 0x150, 0xf, 0xf, true);
                const float s1 = __builtin_amdgcn_mov_dpp(sv, 0x151, 0xf, 0xf, true);
                const float s2 = __builtin_amdgcn_mov_dpp(sv, 0x152, 0xf, 0xf, true);
                ev[i] = __builtin_fma(okc, (double)s2, __builtin_fma(okb, (double)s1, __builtin_fma(oka, (double)s0, (double)sv)));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = (l >> 4) * 4 + i;
                // (only the atomics under lane masks; adding 0 from the masked lanes instead
                // measured 23x slower: rows past the group all name one Gaussian and contend)
                const bool ok = row < r;
                float* dst = lane_sums + (uint64_t)rid[i] * srs;
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb)
                    if (ok && xb * 16 + nch < 4 + S) R3DG_FLUSH_ADD(dst + xb * 16, accX[xb][i]);
                double* mom = reinterpret_cast<double*>(a.sums + (uint64_t)rid[i] * srs + XW);
                if (ok && nch < 6) R3DG_FLUSH_ADD(mom + nch, ev[i]);
            }
            wave_lds_sync();
            return;
        } else if constexpr (ATOM) {
            // The moments about the quadrant centre, expanded about the Gaussian's mean once per row
            // and summed in double: D rows go through a 16 x 8 float tile in w rows 0-1 (free once
            // the MFMA operands were read); lane rr = l & 15 expands row rr in double (expand_moments'
            // formula) into a 16 x 6 double tile in w rows 2-5, and every lane adds its (row, moment)
            // element with an f64 atomic into the per-Gaussian moment sums. A needle's expanded terms
            // (|mean - pixel| ~ 1e3 px) are ~1e3-1e6 times the sums they cancel to: summed in f32 in
            // arrival order, one Gaussian's dL/dmean2D came out 2370x past its conditioning bound
            // (test_cull_exact_needles; profiles/r05/README.md).
            float* const yt = wq;
            auto yoff = [](int row) { return (row >> 3) * WQS + (row & 7) * 8; };
            auto doff = [](int row) { return (2 + (row >> 2)) * WQS + (row & 3) * 16; };  // 8-B aligned
            if (nch < 6) {
#pragma unroll
                for (int i = 0; i < 4; ++i) yt[yoff((l >> 4) * 4 + i) + nch] = accY[i];
            }
            wave_lds_sync();
            if (l < 16) {
                const float2* yr = reinterpret_cast<const float2*>(yt + yoff(l));
                const float2 m01 = yr[0], m23 = yr[1], m45 = yr[2];
                const float2 mxy = *reinterpret_cast<const float2*>(wq + l * WQS + 64);
                const double s0 = m01.x, s1 = m01.y, s2 = m23.x, s3 = m23.y, s4 = m45.x, s5 = m45.y;
                const double dx0 = (double)mxy.x - (double)qcx, dy0 = (double)mxy.y - (double)qcy;
                double* yw = reinterpret_cast<double*>(wq + doff(l));
                yw[0] = s0;
                yw[1] = dx0 * s0 - s1;
                yw[2] = dy0 * s0 - s2;
                yw[3] = dx0 * (dx0 * s0 - 2.0 * s1) + s3;
                yw[4] = dx0 * (dy0 * s0 - s2) - dy0 * s1 + s4;
                yw[5] = dy0 * (dy0 * s0 - 2.0 * s2) + s5;
            }
            wave_lds_sync();
            // the four expanded elements of this lane, read together (the compiler would otherwise
            // sink each read into its atomic's masked branch: four dependent LDS round trips)
            double ev[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                ev[i] = reinterpret_cast<const double*>(wq + doff((l >> 4) * 4 + i))[nch < 6 ? nch : 0];
            asm volatile("" ::"v"(ev[0]), "v"(ev[1]), "v"(ev[2]), "v"(ev[3]));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = (l >> 4) * 4 + i;
                // (only the atomics under lane masks; adding 0 from the masked lanes instead
                // measured 23x slower: rows past the group all name one Gaussian and contend)
                const bool ok = row < r;
                float* dst = lane_sums + (uint64_t)rid[i] * srs;
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb)
                    if (ok && xb * 16 + nch < 4 + S) R3DG_FLUSH_ADD(dst + xb * 16, accX[xb][i]);
                double* mom = reinterpret_cast<double*>(a.sums + (uint64_t)rid[i] * srs + XW);
                if (ok && nch < 6) R3DG_FLUSH_ADD(mom + nch, ev[i]);
            }
            wave_lds_sync();
            return;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (l >> 4) * 4 + i;
            const uint32_t base = rid[i];
            if (row < r) {
                // 32-bit offset in float4 units (RS is a multiple of 8 floats): 4L rows x RS / 4
                // stay below 2^32 (checked on the host: L * RS < 2^32, L < 178M at S <= 12)
                float* dst = reinterpret_cast<float*>(reinterpret_cast<float4*>(a.rows) + base * (uint32_t)(RS >> 2));
#pragma unroll
                for (int xb = 0; xb < NXB; ++xb) dst[xb * 16 + nch] = accX[xb][i];
                const float mv = nch < 6 ? accY[i] : cpad;
                if (nch < 8) dst[XW + nch] = mv;
            }
        }
        wave_lds_sync();
    };

    // Gaussian of instance (l & 31) of the batch ending at tile position hi_b (tail lanes clamp
    // to the batch's last instance, so every DMA lane reads a valid record)
    auto batch_gid = [&](int hi_b) -> uint32_t {
        const int tt = min(l & (NB - 1), min(NB, hi_b) - 1);
        return a.point_list[range.x + (uint32_t)(hi_b - 1 - tt)];
    };
    // The DMA is issued by inline asm: the compiler does not track it, so it does not wait for it
    // before every LDS read of the current buffer (it cannot tell the two buffers apart); the
    // batch loop waits for it explicitly (vmcnt(0) before the batch barrier).
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)s_lds;
    auto issue = [&](uint32_t gid, int buf) {
#pragma unroll
        for (int k = 0; k < NCP; ++k) {
            if ((k & 3) != w) continue;  // wave-uniform
            // lane l of instruction k: entry k * 64 + l = column q, instance l % NB
            const int q = (k * 64 + l) / NB;
            const float4* src = a.records + (size_t)gid * RF4 + min(q, RF4 - 1);
            const uint32_t dst =
                __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)((NW * WQF4 + buf * SBUF + k * 64) * 16));
            if (q < RF4) {  // lanes past the last column are masked off (they would write past the buffer)
                int keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
            }
        }
    };

    // contribution byte of instance l of the batch ending at tile position hi_b (0 past the batch)
    auto batch_bits = [&](int hi_b) -> uint32_t {
        return l < min(NB, hi_b) ? (uint32_t)a.contrib[range.x + (uint32_t)(hi_b - 1 - l)] : 0u;
    };
    int r = 0;
    uint32_t gid_cur = max_last > 0 ? batch_gid(max_last) : 0u;  // Gaussian of instance l of the current batch
    if (max_last > 0) issue(gid_cur, 0);
    uint32_t gid_next = max_last > NB ? batch_gid(max_last - NB) : 0u;
    uint32_t cb_next = max_last > 0 ? batch_bits(max_last) : 0u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int buf = 0;
#ifdef R3DG_EXP_COUNT
    const long long t_begin = wall_clock64();
    long long t_wait = 0, t_mask = 0, t_flush = 0;
#endif
    for (int hi = max_last; hi > 0; hi -= NB) {
        const int cnt = min(NB, hi);
        const int hn = hi - NB;
#ifdef R3DG_EXP_COUNT
        const long long tm0 = wall_clock64();
#endif
        const uint32_t cbits = cb_next;
        const uint32_t gid_staged = gid_next;
        if (hn > 0) {  // block-uniform: stage the next batch while this one blends
            issue(gid_next, buf ^ 1);
            gid_next = hn > NB ? batch_gid(hn - NB) : 0u;
            cb_next = batch_bits(hn);
        }
        st = stage + buf * SBUF;
        // this wave's live instances: the forward's contribution bits for its quadrant (lanes
        // 0..cnt-1; zero past the batch)
        // this wave's partial row of instance l (4 * slot + quadrant), flagged here, once per
        // visited instance (rather than by the flush's row stores)
        uint32_t row_l = 0u;
        const bool mine = (cbits >> (2 * w)) & 3u;  // bit 2w + h: half h of quadrant w blended it
        mask_t bits = (mask_t)__ballot(mine);
        const int lo = hi - wmax;  // instances j < lo lie beyond every pixel of this wave
        if (lo >= NB) bits = 0u;
        else if (lo > 0) bits &= ~(mask_t)0 << lo;
        if constexpr (ATOM) {
            row_l = gid_cur;
        } else if ((bits >> l) & 1u) {
            const uint32_t slot =
                record_slot(st[NB + l], gid_cur == 0 ? 0u : a.offsets[gid_cur - 1], tx, ty, a.grid_x, a.grid_y);
            row_l = 4 * slot + w;
            a.flags[row_l] = 1;
        }
#ifdef R3DG_EXP_COUNT
        if (l == 0) R3DG_EXP_ADD(0, __builtin_popcountll(bits));
        t_mask += wall_clock64() - tm0;
#endif
        auto rec0 = [&](int j) { return st[__builtin_amdgcn_readfirstlane(j)]; };
        auto pos = [&](int j) {
            return *reinterpret_cast<const float2*>(st + NB + __builtin_amdgcn_readfirstlane(j));
        };
        while (bits) {
#if R3DG_BWD_SWALK
            int j0, j1;
            if constexpr (NB > 32) {
                unsigned long long b = bits;
                asm("s_ff1_i32_b64 %0, %2\n\ts_bitset0_b64 %2, %0\n\ts_ff1_i32_b64 %1, %2\n\ts_bitset0_b64 %2, %1"
                    : "=&s"(j0), "=&s"(j1), "+s"(b));
                bits = b;
            } else {
                uint32_t b = bits;
                asm("s_ff1_i32_b32 %0, %2\n\ts_bitset0_b32 %2, %0\n\ts_ff1_i32_b32 %1, %2\n\ts_bitset0_b32 %2, %1"
                    : "=&s"(j0), "=&s"(j1), "+s"(b));
                bits = b;
            }
            const bool has1 = j1 >= 0;
            j1 = has1 ? j1 : j0;
#else
            const int j0 = (int)__builtin_ctzll(bits);
            bits &= bits - 1;
            const bool has1 = bits != 0u;
            const int j1 = has1 ? (int)__builtin_ctzll(bits) : j0;
            bits &= bits - 1;
#endif
            const float4 co0 = rec0(j0), co1 = rec0(j1);
            const float2 xy0 = pos(j0), xy1 = pos(j1);
            const float pw0 = gauss_power(co0, xy0.x - pfx, xy0.y - pfy);
            const float pw1 = gauss_power(co1, xy1.x - pfx, xy1.y - pfy);
            float G0 = fast_expf(pw0), G1 = fast_expf(pw1);
            settle_threshold2(pw0, co0.w, G0, pw1, co1.w, G1);
            float wv0, qv0, wv1, qv1;
            bool ok0, ok1;
            step(j0, hi - 1 - j0, true, co0.w, pw0, G0, wv0, qv0, ok0);
            step(j1, hi - 1 - j1, has1, co1.w, pw1, G1, wv1, qv1, ok1);
#ifdef R3DG_EXP_COUNT
            {
                const unsigned long long b0 = __ballot(ok0), b1 = __ballot(ok1);
                if (l == 0) {
                    R3DG_EXP_ADD(5, (b0 != 0ull ? 1 : 0) + (b1 != 0ull ? 1 : 0));
                    R3DG_EXP_ADD(6, __builtin_popcountll(b0) + __builtin_popcountll(b1));
                }
            }
#else
            (void)ok0;
            (void)ok1;
#endif
            // every visited instance was blended by a pixel of this wave: one group row each; lane 0
            // also writes the row's bookkeeping into the image rows' pad columns (the flush reads it)
            {
                float* wr = wq + r * WQS + l;
                wr[0] = wv0;
                wr[GRP * WQS] = qv0;
                const uint32_t id0 = __builtin_amdgcn_readlane(row_l, j0);
                if (lane0) {
                    if constexpr (!R3DG_BWD_ORIGIN_MOMENTS) *reinterpret_cast<float2*>(wq + r * WQS + 64) = xy0;
                    reinterpret_cast<uint32_t*>(wq)[(GRP + r) * WQS + 64] = id0;
                }
            }
            if (has1) {
                float* wr = wq + (r + 1) * WQS + l;
                wr[0] = wv1;
                wr[GRP * WQS] = qv1;
                const uint32_t id1 = __builtin_amdgcn_readlane(row_l, j1);
                if (lane0) {
                    if constexpr (!R3DG_BWD_ORIGIN_MOMENTS) *reinterpret_cast<float2*>(wq + (r + 1) * WQS + 64) = xy1;
                    reinterpret_cast<uint32_t*>(wq)[(GRP + r + 1) * WQS + 64] = id1;
                }
            }
            r += has1 ? 2 : 1;
            if (r > GRP - 2) {
#ifdef R3DG_EXP_COUNT
                const long long tf0 = wall_clock64();
#endif
                flush(r);
#ifdef R3DG_EXP_COUNT
                t_flush += wall_clock64() - tf0;
#endif
                r = 0;
            }
        }
        // the next batch's records have landed (this wave's DMA) and every wave is done with
        // this buffer before the next iteration's DMA overwrites it
#ifdef R3DG_EXP_COUNT
        const long long tw0 = wall_clock64();
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifndef R3DG_EXP_NOBARRIER  // timing experiment only (results invalid): no cross-wave batch sync
        __syncthreads();
#endif
#ifdef R3DG_EXP_COUNT
        t_wait += wall_clock64() - tw0;
#endif
        buf ^= 1;
        gid_cur = gid_staged;
    }
    if (r > 0) flush(r);
#ifdef R3DG_EXP_COUNT
    if (l == 0) {
        R3DG_EXP_ADD(2, t_wait);                    // batch-end DMA wait + barrier, per wave
        R3DG_EXP_ADD(3, wall_clock64() - t_begin);  // batch loop total, per wave
        R3DG_EXP_ADD(4, t_mask);                    // DMA issue + live masks, per wave
        R3DG_EXP_ADD(7, t_flush);                   // in-loop flushes, per wave
    }
#endif
}

template <int SMAX>
static hipError_t launch_bwd_s(const RenderBwdArgs& a, hipStream_t stream) {
    // variant_dpp (r3dg_options.test_bwd_dpp): the DPP-reduction cross-check (tests/test_gpu_parity.py);
    // default: the DMA-staged MFMA kernel. Both write the same partial rows (the forward's contribution set).
    const bool dpp = a.variant_dpp != 0;
    // wterms 1 / 3 (test_bwd_wterms; S in 9..11, atomic sums only; refused otherwise): w in one bf16
    // term, the inexact reduction the gradient parity bar must reject, or in three (exact products),
    // the reference point of the default two-term split's error (tests/test_gpu_parity.py)
    const int wterms = a.wterms;
    const int grid = padded_tile_grid(a.num_tiles);
    if (wterms) {
        if constexpr (SMAX == 11) {
            if (!a.sums_atomic || dpp || (wterms != 1 && wterms != 3)) return hipErrorInvalidValue;
            if (wterms == 1)
                launch_kernel(render_bwd_glds_kernel<SMAX, true, 1>, dim3(grid), dim3(kBlock), stream, a);
            else
                launch_kernel(render_bwd_glds_kernel<SMAX, true, 3>, dim3(grid), dim3(kBlock), stream, a);
        } else {
            return hipErrorInvalidValue;
        }
    } else if (dpp)
        launch_kernel(render_bwd_dpp_kernel<SMAX>, dim3(grid), dim3(kBlock), stream, a);
    else if (a.sums_atomic)
        launch_kernel(render_bwd_glds_kernel<SMAX, true>, dim3(grid), dim3(kBlock), stream, a);
    else
        launch_kernel(render_bwd_glds_kernel<SMAX, false>, dim3(grid), dim3(kBlock), stream, a);
    return hipGetLastError();
}

hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t stream) {
    if (a.num_tiles == 0) return hipSuccess;
    if (a.S == 0) return launch_bwd_s<0>(a, stream);
    if (a.S <= 4) return launch_bwd_s<4>(a, stream);
    if (a.S <= 8) return launch_bwd_s<8>(a, stream);
    if (a.S <= 11) return launch_bwd_s<11>(a, stream);  // M1 / C3 (S = 11): no pad-channel FMA
    if (a.S <= 12) return launch_bwd_s<12>(a, stream);
    if (a.S <= 16) return launch_bwd_s<16>(a, stream);
    if (a.S <= 24) return launch_bwd_s<24>(a, stream);
    return launch_bwd_s<32>(a, stream);
}

// ---------------------------------------------------------------------------------------------
// per-Gaussian: sum of gradient rows + preprocessing backward
// ---------------------------------------------------------------------------------------------

// The view direction of a Gaussian and its SH basis (backward.cu:27-57): shared by sh_backward
// and the view-parallel SH rebuild, so both evaluate the same expressions to the same bits.
__device__ __forceinline__ void sh_dir_basis(float3 pos, const float* campos, float& dox, float& doy, float& doz,
                                             float& x, float& y, float& z, float* b) {
#pragma clang fp contract(off)
    dox = pos.x - campos[0]; doy = pos.y - campos[1]; doz = pos.z - campos[2];
    const float len = sqrtf(dox * dox + doy * doy + doz * doz);
    x = dox / len; y = doy / len; z = doz / len;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    b[0] = SH_C0;
    b[1] = -SH_C1 * y; b[2] = SH_C1 * z; b[3] = -SH_C1 * x;
    b[4] = SH_C2_0 * xy; b[5] = SH_C2_1 * yz; b[6] = SH_C2_2 * (2.f * zz - xx - yy); b[7] = SH_C2_3 * xz;
    b[8] = SH_C2_4 * (xx - yy);
    b[9] = SH_C3_0 * y * (3.f * xx - yy); b[10] = SH_C3_1 * xy * z; b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
    b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy); b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
    b[14] = SH_C3_5 * z * (xx - yy); b[15] = SH_C3_6 * x * (xx - 3.f * yy);
}

// backward.cu:20-139 (computeColorFromSH backward). dL_dRGB already clamp-masked.
__device__ static void sh_backward(int deg, int M, float3 pos, const float* campos, const float* sh,
                                   const float* dRGB, float* dL_dmean, float* dsh) {
    float dox, doy, doz, x, y, z, b[16];
    sh_dir_basis(pos, campos, dox, doy, doz, x, y, z, b);
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    float ddx[3] = {0.f, 0.f, 0.f}, ddy[3] = {0.f, 0.f, 0.f}, ddz[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (deg > 0) {
            ddx[c] = -SH_C1 * sh[3 * 3 + c];
            ddy[c] = -SH_C1 * sh[1 * 3 + c];
            ddz[c] = SH_C1 * sh[2 * 3 + c];
            if (deg > 1) {
                ddx[c] += SH_C2_0 * y * sh[4 * 3 + c] + SH_C2_2 * 2.f * -x * sh[6 * 3 + c] +
                          SH_C2_3 * z * sh[7 * 3 + c] + SH_C2_4 * 2.f * x * sh[8 * 3 + c];
                ddy[c] += SH_C2_0 * x * sh[4 * 3 + c] + SH_C2_1 * z * sh[5 * 3 + c] +
                          SH_C2_2 * 2.f * -y * sh[6 * 3 + c] + SH_C2_4 * 2.f * -y * sh[8 * 3 + c];
                ddz[c] += SH_C2_1 * y * sh[5 * 3 + c] + SH_C2_2 * 2.f * 2.f * z * sh[6 * 3 + c] +
                          SH_C2_3 * x * sh[7 * 3 + c];
                if (deg > 2) {
                    ddx[c] += (SH_C3_0 * sh[9 * 3 + c] * 3.f * 2.f * xy + SH_C3_1 * sh[10 * 3 + c] * yz +
                               SH_C3_2 * sh[11 * 3 + c] * -2.f * xy + SH_C3_3 * sh[12 * 3 + c] * -3.f * 2.f * xz +
                               SH_C3_4 * sh[13 * 3 + c] * (-3.f * xx + 4.f * zz - yy) +
                               SH_C3_5 * sh[14 * 3 + c] * 2.f * xz + SH_C3_6 * sh[15 * 3 + c] * 3.f * (xx - yy));
                    ddy[c] += (SH_C3_0 * sh[9 * 3 + c] * 3.f * (xx - yy) + SH_C3_1 * sh[10 * 3 + c] * xz +
                               SH_C3_2 * sh[11 * 3 + c] * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3_3 * sh[12 * 3 + c] * -3.f * 2.f * yz + SH_C3_4 * sh[13 * 3 + c] * -2.f * xy +
                               SH_C3_5 * sh[14 * 3 + c] * -2.f * yz + SH_C3_6 * sh[15 * 3 + c] * -3.f * 2.f * xy);
                    ddz[c] += (SH_C3_1 * sh[10 * 3 + c] * xy + SH_C3_2 * sh[11 * 3 + c] * 4.f * 2.f * yz +
                               SH_C3_3 * sh[12 * 3 + c] * 3.f * (2.f * zz - xx - yy) +
                               SH_C3_4 * sh[13 * 3 + c] * 4.f * 2.f * xz + SH_C3_5 * sh[14 * 3 + c] * (xx - yy));
                }
            }
        }
    }
    // dsh may alias sh (the gather kernel updates its LDS copy in place): written after the reads
    const int ncoef = deg > 2 ? 16 : (deg > 1 ? 9 : (deg > 0 ? 4 : 1));
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) dsh[3 * i + c] = i < ncoef ? b[i] * dRGB[c] : 0.f;  // one rounding
    const float dvx = ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2];
    const float dvy = ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2];
    const float dvz = ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2];
    // dnormvdv (auxiliary.h:107-117)
    const float sum2 = dox * dox + doy * doy + doz * doz;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    dL_dmean[0] += ((+sum2 - dox * dox) * dvx - doy * dox * dvy - doz * dox * dvz) * invsum32;
    dL_dmean[1] += (-dox * doy * dvx + (sum2 - doy * doy) * dvy - doz * doy * dvz) * invsum32;
    dL_dmean[2] += (-dox * doz * dvx - doy * doz * dvy + (sum2 - doz * doz) * dvz) * invsum32;
}

// backward.cu:280-343 (gradient w.r.t. the un-normalised quaternion, as the reference)
__device__ static void cov3d_backward(float3 sc, float mod, float4 q, const float* d, float* dscale, float* drot) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    float R[3][3];
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y + r * z); R[0][2] = 2.f * (x * z - r * y);
    R[1][0] = 2.f * (x * y - r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z + r * x);
    R[2][0] = 2.f * (x * z + r * y); R[2][1] = 2.f * (y * z - r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
    const float s[3] = {mod * sc.x, mod * sc.y, mod * sc.z};
    float M[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) M[i][j] = s[i] * R[i][j];
    const float Dm[3][3] = {{d[0], 0.5f * d[1], 0.5f * d[2]}, {0.5f * d[1], d[3], 0.5f * d[4]},
                            {0.5f * d[2], 0.5f * d[4], d[5]}};
    float dM[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) dM[i][j] = 2.0f * (M[i][0] * Dm[0][j] + M[i][1] * Dm[1][j] + M[i][2] * Dm[2][j]);
#pragma unroll
    for (int i = 0; i < 3; ++i) dscale[i] = R[i][0] * dM[i][0] + R[i][1] * dM[i][1] + R[i][2] * dM[i][2];
    float E[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) E[i][j] = dM[i][j] * s[i];
    drot[0] = 2 * z * (E[0][1] - E[1][0]) + 2 * y * (E[2][0] - E[0][2]) + 2 * x * (E[1][2] - E[2][1]);
    drot[1] = 2 * y * (E[1][0] + E[0][1]) + 2 * z * (E[2][0] + E[0][2]) + 2 * r * (E[1][2] - E[2][1]) -
              4 * x * (E[2][2] + E[1][1]);
    drot[2] = 2 * x * (E[1][0] + E[0][1]) + 2 * r * (E[2][0] - E[0][2]) + 2 * z * (E[1][2] + E[2][1]) -
              4 * y * (E[2][2] + E[0][0]);
    drot[3] = 2 * r * (E[0][1] - E[1][0]) + 2 * x * (E[2][0] + E[0][2]) + 2 * y * (E[1][2] + E[2][1]) -
              4 * z * (E[1][1] + E[0][0]);
}

// Per-Gaussian part of the gather: writes the summed instance gradients, then computeCov2DCUDA,
// the projection and SH backward (preprocessCUDA bwd) and computeCov3D backward. `s` holds the
// summed row, `shl` this Gaussian's SH coefficients in LDS, replaced by dL/dsh on return.
template <int SMAX>
__device__ __forceinline__ void gather_gaussian(const GatherBwdArgs& a, int g, const float* s, float* shl) {
#pragma clang fp contract(off)  // the oracle's operation sequence (cov2D backward is ill-conditioned)
    a.dL_dmeans2D[3 * g + 0] = s[kRowMean + 0];
    a.dL_dmeans2D[3 * g + 1] = s[kRowMean + 1];
    a.dL_dmeans2D[3 * g + 2] = s[kRowMean + 2];
    a.dL_dopacity[(size_t)g * a.ld_op] = s[kRowOpacity];
    a.dL_dcolors[3 * g + 0] = s[kRowColor + 0];
    a.dL_dcolors[3 * g + 1] = s[kRowColor + 1];
    a.dL_dcolors[3 * g + 2] = s[kRowColor + 2];
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
        if (c < a.S) a.dL_dfeatures[(size_t)g * a.ld_f + c] = s[kRowFeat + c];

    float* dmean3 = a.dL_dmeans3D + (size_t)g * a.ld_m3;
    float* dcov = a.dL_dcov3D + 6 * g;
    if (!(a.radii[g] > 0)) {
        dmean3[0] = dmean3[1] = dmean3[2] = 0.f;
        for (int i = 0; i < 6; ++i) dcov[i] = 0.f;
        for (int i = 0; i < 3 * a.M; ++i) shl[i] = 0.f;
        for (int i = 0; i < 3; ++i) a.dL_dscales[(size_t)g * a.ld_sc + i] = 0.f;
        for (int i = 0; i < 4; ++i) a.dL_drotations[(size_t)g * a.ld_rot + i] = 0.f;
        return;
    }

    // ---- computeCov2DCUDA (backward.cu:144-276) ----
    const float h_x = a.focal_x, h_y = a.focal_y;
    const float* view = a.view;
    const float3 mean = make_float3(a.means3D[3 * g], a.means3D[3 * g + 1], a.means3D[3 * g + 2]);
    const float* c3 = a.cov3D + 6 * g;
    const float dcx = s[kRowConic + 0], dcy = s[kRowConic + 1], dcz = s[kRowConic + 2];
    float3 t = xform_point4x3(mean, view);
    const float limx = 1.3f * a.tan_fovx, limy = 1.3f * a.tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
    const float j00 = h_x / t.z, j11 = h_y / t.z;
    const float j20 = -(h_x * t.x) / (t.z * t.z), j21 = -(h_y * t.y) / (t.z * t.z);
    float g0[3], g1[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        g0[r] = view[4 * r + 0] * j00 + view[4 * r + 2] * j20;
        g1[r] = view[4 * r + 1] * j11 + view[4 * r + 2] * j21;
    }
    const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float u[3], vv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        u[k] = V[k][0] * g0[0] + V[k][1] * g0[1] + V[k][2] * g0[2];
        vv[k] = V[k][0] * g1[0] + V[k][1] * g1[1] + V[k][2] * g1[2];
    }
    const float ca = g0[0] * u[0] + g0[1] * u[1] + g0[2] * u[2] + 0.3f;
    const float cb = g1[0] * u[0] + g1[1] * u[1] + g1[2] * u[2];
    const float cc = g1[0] * vv[0] + g1[1] * vv[1] + g1[2] * vv[2] + 0.3f;
    const float denom = ca * cc - cb * cb;
    float da = 0.f, db = 0.f, dc = 0.f;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    if (denom2inv != 0.f) {
        da = denom2inv * (-cc * cc * dcx + 2 * cb * cc * dcy + (denom - ca * cc) * dcz);
        dc = denom2inv * (-ca * ca * dcz + 2 * ca * cb * dcy + (denom - ca * cc) * dcx);
        db = denom2inv * 2 * (cb * cc * dcx - (denom + 2 * cb * cb) * dcy + ca * cb * dcz);
        dcov[0] = g0[0] * g0[0] * da + g0[0] * g1[0] * db + g1[0] * g1[0] * dc;
        dcov[3] = g0[1] * g0[1] * da + g0[1] * g1[1] * db + g1[1] * g1[1] * dc;
        dcov[5] = g0[2] * g0[2] * da + g0[2] * g1[2] * db + g1[2] * g1[2] * dc;
        dcov[1] = 2 * g0[0] * g0[1] * da + (g0[0] * g1[1] + g0[1] * g1[0]) * db + 2 * g1[0] * g1[1] * dc;
        dcov[2] = 2 * g0[0] * g0[2] * da + (g0[0] * g1[2] + g0[2] * g1[0]) * db + 2 * g1[0] * g1[2] * dc;
        dcov[4] = 2 * g0[2] * g0[1] * da + (g0[1] * g1[2] + g0[2] * g1[1]) * db + 2 * g1[1] * g1[2] * dc;
    } else {
        for (int i = 0; i < 6; ++i) dcov[i] = 0.f;
    }
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float p0 = g0[0] * V[k][0] + g0[1] * V[k][1] + g0[2] * V[k][2];
        const float p1 = g1[0] * V[k][0] + g1[1] * V[k][1] + g1[2] * V[k][2];
        dT0[k] = 2 * p0 * da + p1 * db;
        dT1[k] = 2 * p1 * dc + p0 * db;
    }
    const float dJ00 = view[0] * dT0[0] + view[4] * dT0[1] + view[8] * dT0[2];
    const float dJ02 = view[2] * dT0[0] + view[6] * dT0[1] + view[10] * dT0[2];
    const float dJ11 = view[1] * dT1[0] + view[5] * dT1[1] + view[9] * dT1[2];
    const float dJ12 = view[2] * dT1[0] + view[6] * dT1[1] + view[10] * dT1[2];
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = x_grad_mul * -h_x * tz2 * dJ02;
    const float dty = y_grad_mul * -h_y * tz2 * dJ12;
    const float dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t.x) * tz3 * dJ02 + (2 * h_y * t.y) * tz3 * dJ12;
    const float vz = dtz + s[kRowMean + 2];
    float dm[3] = {view[0] * dtx + view[1] * dty + view[2] * vz, view[4] * dtx + view[5] * dty + view[6] * vz,
                   view[8] * dtx + view[9] * dty + view[10] * vz};

    // ---- preprocessCUDA backward (backward.cu:372-397) ----
    const float* proj = a.proj;
    const float4 mh = xform_point4x4(mean, proj);
    const float m_w = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
    const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
    const float gx2 = s[kRowMean + 0], gy2 = s[kRowMean + 1];
    dm[0] += (proj[0] * m_w - proj[3] * mul1) * gx2 + (proj[1] * m_w - proj[3] * mul2) * gy2;
    dm[1] += (proj[4] * m_w - proj[7] * mul1) * gx2 + (proj[5] * m_w - proj[7] * mul2) * gy2;
    dm[2] += (proj[8] * m_w - proj[11] * mul1) * gx2 + (proj[9] * m_w - proj[11] * mul2) * gy2;
    if (a.sh) {
        const uint8_t cl = a.clamped[g];
        const float dRGB[3] = {s[kRowColor + 0] * ((cl & 1) ? 0.f : 1.f), s[kRowColor + 1] * ((cl & 2) ? 0.f : 1.f),
                               s[kRowColor + 2] * ((cl & 4) ? 0.f : 1.f)};
        sh_backward(a.D, a.M, mean, a.campos, shl, dRGB, dm, shl);
    } else {
        for (int i = 0; i < 3 * a.M; ++i) shl[i] = 0.f;
    }
    dmean3[0] = dm[0];
    dmean3[1] = dm[1];
    dmean3[2] = dm[2];
    if (a.use_scales) {
        const float3 sc = make_float3(a.scales[3 * g], a.scales[3 * g + 1], a.scales[3 * g + 2]);
        const float4 q = make_float4(a.rotations[4 * g], a.rotations[4 * g + 1], a.rotations[4 * g + 2],
                                     a.rotations[4 * g + 3]);
        cov3d_backward(sc, a.scale_modifier, q, dcov, a.dL_dscales + (size_t)g * a.ld_sc,
                       a.dL_drotations + (size_t)g * a.ld_rot);
    } else {
        for (int i = 0; i < 3; ++i) a.dL_dscales[(size_t)g * a.ld_sc + i] = 0.f;
        for (int i = 0; i < 4; ++i) a.dL_drotations[(size_t)g * a.ld_rot + i] = 0.f;
    }
}

// ---------------------------------------------------------------------------------------------
// View-parallel SH-gradient exchange (include/r3dg_hip.h r3dg_sh_color_grads / _from_views)
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sh_color_grads_kernel(int n, const uint8_t* __restrict__ clamped,
                                                             const float* __restrict__ dcol, float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * n) return;
    const int g = i / 3, c = i - 3 * g;
    out[i] = ((clamped[g] >> c) & 1) ? 0.f : dcol[i];
}

// One thread per Gaussian: the SH basis of each view's direction exactly as sh_backward computes
// it (backward.cu:20-139), summed over the views in order.
// One thread per Gaussian, 128 per workgroup; the block's [128, M, 3] output is assembled in LDS
// and written as one contiguous span (a thread's own 192-byte row would be 64 lines per store).
constexpr int kShViewsBlock = 128;
__global__ void __launch_bounds__(kShViewsBlock) sh_grad_views_kernel(int g0, int n, int deg, int M, int N,
                                                                     const float* __restrict__ means3D,
                                                                     const float* __restrict__ campos,
                                                                     const float* __restrict__ drgb,
                                                                     float* __restrict__ dsh) {
#pragma clang fp contract(off)  // the products and sums round separately, as sh_backward's (no FMA)
    constexpr int SHS = 49;     // LDS stride of one Gaussian's row (odd: conflict-free)
    __shared__ float s_out[kShViewsBlock * SHS];
    const int t = threadIdx.x;
    const int ib = blockIdx.x * kShViewsBlock;
    const int i = ib + t;
    if (i < n) {
        const int g = g0 + i;
        const float3 pos = make_float3(means3D[3 * g], means3D[3 * g + 1], means3D[3 * g + 2]);
        const int ncoef = deg > 2 ? 16 : (deg > 1 ? 9 : (deg > 0 ? 4 : 1));
        float acc[16][3];
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[k][0] = acc[k][1] = acc[k][2] = 0.f;
        for (int v = 0; v < N; ++v) {
            const float* d = drgb + ((size_t)v * n + i) * 3;
            const float d0 = d[0], d1 = d[1], d2 = d[2];
            // a view without colour gradient adds nothing (the reference skips radii == 0,
            // backward.cu:348-398); skipping also keeps a mean at that view's camera centre (0/0
            // direction) from adding NaN * 0. Bitwise the same sums otherwise: acc + (+-0) == acc.
            if (d0 == 0.f && d1 == 0.f && d2 == 0.f) continue;
            float dox, doy, doz, x, y, z, b[16];
            sh_dir_basis(pos, campos + 3 * v, dox, doy, doz, x, y, z, b);
            // each view's product rounded as sh_backward rounds it, then summed in view order
            // (plain operators under this function's contract(off): the __fadd_rn / __fmul_rn
            // helpers are header functions compiled with contraction on, so they would fuse)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                acc[k][0] = acc[k][0] + b[k] * d0;
                acc[k][1] = acc[k][1] + b[k] * d1;
                acc[k][2] = acc[k][2] + b[k] * d2;
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k < M) {
                const bool on = k < ncoef;
                s_out[t * SHS + 3 * k] = on ? acc[k][0] : 0.f;
                s_out[t * SHS + 3 * k + 1] = on ? acc[k][1] : 0.f;
                s_out[t * SHS + 3 * k + 2] = on ? acc[k][2] : 0.f;
            }
    }
    __syncthreads();
    const int M3 = 3 * M, ng = min(kShViewsBlock, n - ib);
    float* o = dsh + (size_t)(g0 + ib) * M3;
    const uint32_t m3 = fastdiv_magic((uint32_t)M3);
    for (int f = t; f < ng * M3; f += kShViewsBlock) {
        const int gg = fastdiv(f, m3);
        o[f] = s_out[gg * SHS + (f - gg * M3)];
    }
}

hipError_t launch_sh_color_grads(int n, const uint8_t* clamped, const float* dcol, float* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sh_color_grads_kernel, dim3((3 * n + 255) / 256), dim3(256), 0, st, n, clamped, dcol, out);
    return hipGetLastError();
}
hipError_t launch_sh_grad_views(int g0, int n, int deg, int M, int N, const float* means3D, const float* campos,
                                const float* drgb, float* dsh, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sh_grad_views_kernel, dim3((n + kShViewsBlock - 1) / kShViewsBlock), dim3(kShViewsBlock), 0, st,
                       g0, n, deg, M, N, means3D,
                       campos, drgb, dsh);
    return hipGetLastError();
}

// Gather phase 1: per-Gaussian sums of its partial rows, in slot order then quadrant order (the
// same fixed order every run). One group of LPG lanes per Gaussian. The Gaussian's rows are the
// contiguous range 4 * [k0, k1) (row 4 * slot + quadrant); per chunk of 8 slots, lanes 0..7 load
// one flag word each and the group ORs them into a 32-bit (slot, quadrant) presence mask, then
// walks the present rows four at a time with independent loads (absent tail rows load nothing).
// Lane c sums float4 column c of every row (c < NXC: the X part); the two moment lanes NXC and
// NXC + 1 swap their columns [S0, Sx, Sy, Sxx], [Sxy, Syy, cx, cy] (DPP) and expand each row's
// moments about the Gaussian's mean with d0 = mean - (cx, cy) (expand_moments): lane NXC sums
// [S0, Sdx, Sdy, Sdxdx], lane NXC + 1 [Sdxdy, Sdydy]. Writes sums + g * RS = [X part (XW) |
// dL/dmean2D x, y | dL/dconic x, y, z | dL/dopacity | 0, 0] (backward.cu:552-611 summed over the
// pixels).
#ifndef R3DG_ROWSUM_RPI
#define R3DG_ROWSUM_RPI 4  // present rows loaded per iteration (independent float4 loads per lane;
                           // measured at M1: 2 -> 0.230, 4 -> 0.206, 8 -> 0.215 ms)
#endif
#ifndef R3DG_ROWSUM_PF
#define R3DG_ROWSUM_PF 1  // row-sum: next chunk's flag word prefetched
#endif

template <int SMAX>
__global__ void __launch_bounds__(256) row_sum_kernel(GatherBwdArgs a) {
    constexpr int NXB = (4 + SMAX + 15) / 16;
    constexpr int NXC = 4 * NXB;                  // float4 columns of a partial row's X part
    constexpr int LPG = NXC + 2 <= 8 ? 8 : 16;    // lanes per Gaussian
    constexpr int CH = 8;                         // slots per chunk (one flag word per lane)
    constexpr int GPB = 256 / LPG;                // Gaussians per workgroup
    const int RS = a.RS;
    const int gb = a.g_begin + blockIdx.x * GPB;  // the workgroup's first Gaussian
    const int g = gb + (int)threadIdx.x / LPG, c = (int)threadIdx.x % LPG;
    const bool active = g < a.g_end && c < NXC + 2;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    double dacc[4] = {0.0, 0.0, 0.0, 0.0};  // moment lanes: the expanded moments, in double as the
                                            // atomic flush's (needle means ~1e3 px off: DESIGN §5)
    uint32_t k0 = 0, n = 0;
    float2 xy = make_float2(0.f, 0.f);
    if (g < a.g_end && a.rows && a.radii[g] > 0) {  // uniform within the group
        k0 = g == 0 ? 0u : a.offsets[g - 1];
        n = a.offsets[g] - k0;
        xy = a.means2D[g];
    }
    const bool mom = c >= NXC;                    // a moment lane (NXC, NXC + 1) or idle
#if R3DG_ROWSUM_PF
    // the next chunk's flag word is loaded before this chunk's rows: one dependent round trip per
    // chunk instead of two
    uint32_t fw_next = (c < CH && c < n) ? a.flags[k0 + c] : 0u;
#endif
    for (uint32_t kb = 0; kb < n; kb += CH) {
#if R3DG_ROWSUM_PF
        const uint32_t fw = fw_next;
        fw_next = (c < CH && kb + CH + c < n) ? a.flags[k0 + kb + CH + c] : 0u;
#else
        const uint32_t fw = (c < CH && kb + c < n) ? a.flags[k0 + kb + c] : 0u;
#endif
        uint32_t mask = ((fw & 0xffu) ? 1u : 0u) | ((fw & 0xff00u) ? 2u : 0u) | ((fw & 0xff0000u) ? 4u : 0u) |
                        ((fw & 0xff000000u) ? 8u : 0u);
        mask <<= 4 * (c & (CH - 1));
#pragma unroll
        for (int o = 1; o < LPG; o <<= 1) mask |= __shfl_xor(mask, o);
        const float* base = a.rows + (size_t)(k0 + kb) * 4 * RS;
        while (mask) {
            float4 v[R3DG_ROWSUM_RPI];
#pragma unroll
            for (int i = 0; i < R3DG_ROWSUM_RPI; ++i) {
                const int bit = mask ? __builtin_ctz(mask) : 0;
                const bool has = mask != 0u;
                const float4* row = reinterpret_cast<const float4*>(base + (size_t)bit * RS);
                mask &= mask - 1u;
                v[i] = active && has ? row[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            if (!mom) {
#pragma unroll
                for (int i = 0; i < R3DG_ROWSUM_RPI; ++i) {
                    acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < R3DG_ROWSUM_RPI; ++i) {
                    // the other moment column from the neighbouring lane (DPP quad_perm [1, 0, 3, 2])
                    const float4 vo = make_float4(dpp_mov<0xB1>(v[i].x), dpp_mov<0xB1>(v[i].y), dpp_mov<0xB1>(v[i].z),
                                                  dpp_mov<0xB1>(v[i].w));
                    const float4 m0 = c == NXC ? v[i] : vo, m1 = c == NXC ? vo : v[i];
                    // expand_moments' formula in double; an absent row is all zero: its centre
                    // (0, 0) multiplies zero moments
                    const double s0 = m0.x, s1 = m0.y, s2 = m0.z, s3 = m0.w, s4 = m1.x, s5 = m1.y;
                    const double dx0 = (double)xy.x - (double)m1.z, dy0 = (double)xy.y - (double)m1.w;
                    if (c == NXC) {
                        dacc[0] += s0;
                        dacc[1] += dx0 * s0 - s1;
                        dacc[2] += dy0 * s0 - s2;
                        dacc[3] += dx0 * (dx0 * s0 - 2.0 * s1) + s3;
                    } else {
                        dacc[0] += dx0 * (dy0 * s0 - s2) - dy0 * s1 + s4;
                        dacc[1] += dy0 * (dy0 * s0 - 2.0 * s2) + s5;
                    }
                }
            }
        }
    }
    // lane NXC takes the [Sdxdy, Sdydy] sums of lane NXC + 1 (all lanes take part in the shuffle)
    const double sxy = __shfl_down(dacc[0], 1), syy = __shfl_down(dacc[1], 1);
    if (!active) return;
    float4* dst = reinterpret_cast<float4*>(a.sums + (size_t)g * RS);
    if (c < NXC) {
        dst[c] = acc;
    } else if (c == NXC) {
        const double S0 = dacc[0], Sdx = dacc[1], Sdy = dacc[2], Sdxdx = dacc[3], Sdxdy = sxy, Sdydy = syy;
        const float4 co = a.conic_opacity[g];
        // dL/dmean2D = -0.5 (W, H) o (o * conic . (Sdx, Sdy)), dL/dconic = -0.5 o (Sdxdx, Sdxdy,
        // Sdydy), dL/dopacity = S0 (backward.cu:583-611), in double and rounded once (as the gather
        // does from the atomic sums)
        const double o = -0.5 * (double)co.w;
        dst[NXC] = make_float4((float)(o * a.W * ((double)co.x * Sdx + (double)co.y * Sdy)),
                               (float)(o * a.H * ((double)co.z * Sdy + (double)co.y * Sdx)), (float)(o * Sdxdx),
                               (float)(o * Sdxdy));
        dst[NXC + 1] = make_float4((float)(o * Sdydy), (float)S0, 0.f, 0.f);
    }
}

// Gather phase 2: one thread per Gaussian reads its sum row, then runs the cov2D / projection /
// SH / cov3D backward (gather_gaussian); SH coefficients staged through LDS by coalesced copies.
template <int SMAX>
__global__ void __launch_bounds__(256) gather_bwd_kernel(GatherBwdArgs a) {
    constexpr int NR = kRowFeat + SMAX;
    constexpr int NXB = (4 + SMAX + 15) / 16;
    constexpr int XW = 16 * NXB;
    constexpr int SHS = 49;                // LDS stride of one Gaussian's SH block (<= 48 used, odd)
    __shared__ float s_buf[256 * SHS];
    const int t = threadIdx.x;
    const int g0 = a.g_begin + blockIdx.x * 256;
    const int g = g0 + t;
    const int S = a.S;

    // sum row -> the kRow layout gather_gaussian reads
    float s[NR];
    if (g < a.g_end) {
        const float* row = a.sums + (size_t)g * (a.sums_moments ? a.SRS : a.RS);
        const float4* src = reinterpret_cast<const float4*>(row);
        float x[XW + 8];
#pragma unroll
        for (int q = 0; q < XW / 4; ++q) {
            const float4 v = src[q];
            x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
        }
        if (a.sums_moments) {
            // the atomic flush summed the moments in double (render_bwd_glds_kernel): about the image
            // origin (R3DG_BWD_ORIGIN_MOMENTS), expanded here about the mean (dx = mean - pixel), or
            // about the mean already; dL/dmean2D, dL/dconic and dL/dopacity from them in double,
            // rounded once
            const double2* md = reinterpret_cast<const double2*>(row + XW);
#if R3DG_BWD_ORIGIN_MOMENTS
            double2 m0 = md[0], m1 = md[1], m2 = md[2];  // [G0, GX], [GY, GXX], [GXY, GYY]
            {
                const float2 mu = a.means2D[g];
                const double mx = mu.x, my = mu.y, G0 = m0.x, GX = m0.y, GY = m1.x;
                const double sdx = mx * G0 - GX, sdy = my * G0 - GY;
                const double sxx = mx * (sdx - GX) + m1.y;              // mx^2 G0 - 2 mx GX + GXX
                const double sxy = mx * sdy - my * GX + m2.x;           // mx my G0 - mx GY - my GX + GXY
                const double syy = my * (sdy - GY) + m2.y;              // my^2 G0 - 2 my GY + GYY
                m0 = make_double2(G0, sdx);
                m1 = make_double2(sdy, sxx);
                m2 = make_double2(sxy, syy);
            }
#else
            const double2 m0 = md[0], m1 = md[1], m2 = md[2];
#endif
            const float4 co = a.conic_opacity[g];
            const double o = -0.5 * (double)co.w;
            x[XW + 0] = (float)(o * a.W * ((double)co.x * m0.y + (double)co.y * m1.x));
            x[XW + 1] = (float)(o * a.H * ((double)co.z * m1.x + (double)co.y * m0.y));
            x[XW + 2] = (float)(o * m1.y);
            x[XW + 3] = (float)(o * m2.x);
            x[XW + 4] = (float)(o * m2.y);
            x[XW + 5] = (float)m0.x;
        } else {
#pragma unroll
            for (int q = XW / 4; q < XW / 4 + 2; ++q) {
                const float4 v = src[q];
                x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
            }
        }
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) s[kRowColor + ch] = x[ch];
#pragma unroll
        for (int ch = 0; ch < SMAX; ++ch) s[kRowFeat + ch] = ch < S ? x[3 + ch] : 0.f;
        float dz = 0.f;
#pragma unroll
        for (int ch = 3; ch < 4 + SMAX; ++ch)
            if (ch == 3 + S) dz = x[ch];
        s[kRowMean + 0] = x[XW + 0];
        s[kRowMean + 1] = x[XW + 1];
        s[kRowMean + 2] = dz;
        s[kRowConic + 0] = x[XW + 2];
        s[kRowConic + 1] = x[XW + 3];
        s[kRowConic + 2] = x[XW + 4];
        s[kRowOpacity] = x[XW + 5];
    }
    // ---- SH coefficients of the block's Gaussians: one coalesced copy into LDS ----
    const int M3 = 3 * a.M;
    const int ng = min(256, a.g_end - g0);
    float* shl = s_buf + t * SHS;
    const uint32_t m3 = fastdiv_magic((uint32_t)M3);
    if (a.sh && a.dL_dsh) {
        const float* src = a.sh + (size_t)g0 * M3;
        block_load4<256>(src, ng * M3, t, [&](int f, float v) {
            const int gg = fastdiv(f, m3);
            s_buf[gg * SHS + (f - gg * M3)] = v;
        });
    }
    __syncthreads();
    if (g < a.g_end) gather_gaussian<SMAX>(a, g, s, shl);
    __syncthreads();
    if (a.dL_dsh) {
        float* dst = a.dL_dsh + (size_t)g0 * M3;
        block_store4<256>(dst, ng * M3, t, [&](int f) {
            const int gg = fastdiv(f, m3);
            return s_buf[gg * SHS + (f - gg * M3)];
        });
    }
}

template <int SMAX>
static hipError_t launch_gather_s(const GatherBwdArgs& a, bool row_sum, hipStream_t stream) {
    constexpr int NXC = 4 * ((4 + SMAX + 15) / 16);
    constexpr int LPG = NXC + 2 <= 8 ? 8 : 16;
    const int n = a.g_end - a.g_begin;
    if (n <= 0) return hipSuccess;
    if (row_sum) {
        const long long threads = (long long)n * LPG;
        launch_kernel(row_sum_kernel<SMAX>, dim3((unsigned)((threads + 255) / 256)), dim3(256), stream, a);
    } else {
        launch_kernel(gather_bwd_kernel<SMAX>, dim3((n + 255) / 256), dim3(256), stream, a);
    }
    return hipGetLastError();
}

static hipError_t launch_per_gaussian(const GatherBwdArgs& a, bool row_sum, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    if (a.S == 0) return launch_gather_s<0>(a, row_sum, stream);
    if (a.S <= 4) return launch_gather_s<4>(a, row_sum, stream);
    if (a.S <= 8) return launch_gather_s<8>(a, row_sum, stream);
    if (a.S <= 12) return launch_gather_s<12>(a, row_sum, stream);
    if (a.S <= 16) return launch_gather_s<16>(a, row_sum, stream);
    if (a.S <= 24) return launch_gather_s<24>(a, row_sum, stream);
    return launch_gather_s<32>(a, row_sum, stream);
}

// the per-instance gradient reduction of renderCUDA's backward (row_sum_kernel)
hipError_t launch_row_sum(const GatherBwdArgs& a, hipStream_t stream) { return launch_per_gaussian(a, true, stream); }
// computeCov2DCUDA + preprocessCUDA backward (gather_bwd_kernel), after launch_row_sum
hipError_t launch_gather_backward(const GatherBwdArgs& a, hipStream_t stream) {
    return launch_per_gaussian(a, false, stream);
}

}  // namespace r3dg
