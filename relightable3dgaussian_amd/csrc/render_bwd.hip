// render_bwd.hip -- backward of the tile blend and of the per-Gaussian preprocessing (gfx950).
//
// Restates reference backward.cu:401-614 (renderCUDA backward), :144-276 (computeCov2DCUDA),
// :20-139 (SH backward), :280-343 (cov3D backward), :348-398 (preprocessCUDA backward).
//
// MI355X design (replaces the reference's per-pixel float atomicAdd scatter, ~(10+S) atomics
// per contributing pixel, backward.cu:552-611):
//   1. render_bwd_kernel: one workgroup per tile replays the tile's list back to front. For each
//      instance every wave reduces its 64 pixels' contributions with DPP (6 VALU ops per value,
//      no LDS traffic) and lane 63 stores the wave total in the wave's own LDS partial row; per
//      chunk of 64 instances the block sums the four wave partials in a fixed order and writes
//      ONE gradient row per (tile, Gaussian) instance with plain vector stores -- at the
//      instance's unsorted slot, which the sort permutation gives us. Slots are
//      Gaussian-contiguous (duplicateWithKeys order).
//   2. gather_bwd_kernel: one thread per Gaussian sums its contiguous rows in a fixed order,
//      then runs the cov2D / projection / SH / cov3D backward for that Gaussian. No global
//      atomics anywhere; the result is bitwise reproducible run to run (the reference's is not).
#include "r3dg_common.h"
#include "r3dg_kernels.h"

namespace r3dg {

__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

template <int SMAX>
__global__ void __launch_bounds__(kBlock) render_bwd_dpp_kernel(RenderBwdArgs a) {
    constexpr int NA4 = (4 + SMAX + 3) / 4;      // attribute row: colour, depth, features
    constexpr int NR = kRowFeat + SMAX;          // reduced values per instance
    constexpr int RSL = (NR + 3) & ~3;           // LDS partial row stride (floats)
    constexpr int CH = 64;                       // instances per flush chunk
    __shared__ float2 s_xy[kBlock];
    __shared__ float4 s_co[kBlock];
    __shared__ uint32_t s_mask[kBlock];
    __shared__ uint32_t s_slot[kBlock];
    __shared__ float4 s_attr[kBlock * NA4];
    __shared__ float4 s_part4[4 * CH * RSL / 4];  // [wave][chunk instance][RSL]
    __shared__ int s_max_last;
    float* s_part = reinterpret_cast<float*>(s_part4);

    const int tile = block_tile(a.tile_order, a.num_tiles);
    if (tile >= a.num_tiles) return;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int px = tx * kTileX + (w & 1) * 8 + (l & 7);
    const int py = ty * kTileY + (w >> 1) * 8 + (l >> 3);
    const bool inside = px < a.W && py < a.H;
    const int pix = inside ? py * a.W + px : 0;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);

    const float T_final = inside ? a.final_T[pix] : 0.f;
    float T = T_final;
    const int last = inside ? (int)a.n_contrib[pix] : 0;
    float g[3], gf[SMAX > 0 ? SMAX : 1], gd = 0.f, go = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) g[c] = inside ? a.dL_dpix[a.ca[c] + pix * a.cm[c]] : 0.f;
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
        gf[c] = (inside && c < a.S) ? a.dL_dpix_f[a.gflay.a[c] + pix * a.gflay.m[c]] : 0.f;
    if (inside) {
        gd = a.dL_dpix_d[pix];
        go = a.dL_dpix_o[pix];
    }
    const float bg_dot = a.bg[0] * g[0] + a.bg[1] * g[1] + a.bg[2] * g[2];
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;

    float acc[3] = {0.f, 0.f, 0.f}, acc_f[SMAX > 0 ? SMAX : 1], acc_d = 0.f, acc_o = 0.f;
    float last_alpha = 0.f, last_depth = 0.f, last_color[3] = {0.f, 0.f, 0.f}, last_f[SMAX > 0 ? SMAX : 1];
#pragma unroll
    for (int c = 0; c < SMAX; ++c) {
        acc_f[c] = 0.f;
        last_f[c] = 0.f;
    }

    // Positions >= max(n_contrib) over the tile are never blended: their rows are zero.
    const int wmax = __builtin_amdgcn_readfirstlane(wave_max_int(last));
    if (t == 0) s_max_last = 0;
    for (int i = t; i < 4 * CH * RSL / 4; i += kBlock) s_part4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (l == 0) atomicMax(&s_max_last, wmax);
    __syncthreads();
    const int max_last = s_max_last;
    const int RS = a.RS;
    for (int p = max_last + t; p < n; p += kBlock) {
        const uint32_t gid = a.point_list[range.x + p];
        const uint32_t slot = instance_slot(a.offsets, a.means2D[gid], a.radii[gid], gid, tx, ty, a.grid_x, a.grid_y);
        float4* row = reinterpret_cast<float4*>(a.rows + (size_t)slot * RS);
        for (int q = 0; q < RS / 4; ++q) row[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    for (int hi = max_last; hi > 0; hi -= kBlock) {
        const int cnt = min(kBlock, hi);
        __syncthreads();  // previous batch fully consumed before the staging arrays are reused
        if (t < cnt) {
            const uint32_t k = range.x + (uint32_t)(hi - 1 - t);
            const uint32_t gid = a.point_list[k];
            const float2 xy = a.means2D[gid];
            s_slot[t] = instance_slot(a.offsets, xy, a.radii[gid], gid, tx, ty, a.grid_x, a.grid_y);
            const float4 co = a.conic_opacity[gid];
            s_xy[t] = xy;
            s_co[t] = co;
            s_mask[t] = quadrant_mask(xy, co, tx * kTileX, ty * kTileY, a.cull);
            float v[NA4 * 4];
#pragma unroll
            for (int i = 0; i < NA4 * 4; ++i) v[i] = 0.f;
            v[0] = a.colors[3 * gid + 0];
            v[1] = a.colors[3 * gid + 1];
            v[2] = a.colors[3 * gid + 2];
            v[3] = a.depths[gid];
            const float* f = a.features + (size_t)gid * a.S;
#pragma unroll
            for (int c = 0; c < SMAX; ++c)
                if (c < a.S) v[4 + c] = f[c];
#pragma unroll
            for (int q = 0; q < NA4; ++q)
                s_attr[t * NA4 + q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
        __syncthreads();
        for (int j0 = 0; j0 < cnt; j0 += CH) {
            const int jn = min(CH, cnt - j0);
            for (int jj = 0; jj < jn; ++jj) {
                const int j = j0 + jj;
                const int p = hi - 1 - j;  // position in the tile range (reference `contributor`)
                if (p >= wmax) continue;   // no pixel of this wave reaches this far back
                const uint32_t m = __builtin_amdgcn_readfirstlane(s_mask[j]);
                if (!((m >> w) & 1u)) continue;
                bool contrib = inside && p < last;
                float G = 0.f, alpha = 0.f, dx = 0.f, dy = 0.f;
                float4 co = make_float4(0.f, 0.f, 0.f, 0.f);
                if (contrib) {
                    const float2 xy = s_xy[j];
                    co = s_co[j];
                    dx = xy.x - pfx;
                    dy = xy.y - pfy;
                    const float power = gauss_power(co, dx, dy);
                    if (power > 0.0f) {
                        contrib = false;
                    } else {
                        G = __expf(power);
                        alpha = fminf(0.99f, co.w * G);
                        if (alpha < 1.0f / 255.0f) contrib = false;
                    }
                }
                if (__ballot(contrib) == 0ull) continue;
                float vals[NR];
#pragma unroll
                for (int r = 0; r < NR; ++r) vals[r] = 0.f;
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
                        vals[kRowColor + c] = dchannel_dcolor * g[c];
                    }
#pragma unroll
                    for (int c = 0; c < SMAX; ++c) {
                        acc_f[c] = last_alpha * last_f[c] + (1.f - last_alpha) * acc_f[c];
                        last_f[c] = v[4 + c];
                        if (a.backward_geometry) dL_dalpha += (v[4 + c] - acc_f[c]) * gf[c];
                        vals[kRowFeat + c] = dchannel_dcolor * gf[c];
                    }
                    acc_d = last_alpha * last_depth + (1.f - last_alpha) * acc_d;
                    last_depth = v[3];
                    dL_dalpha += (v[3] - acc_d) * gd;
                    acc_o = last_alpha + (1.f - last_alpha) * acc_o;
                    dL_dalpha += (1.0f - acc_o) * go;
                    dL_dalpha *= T;
                    last_alpha = alpha;
                    dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                    const float dL_dG = co.w * dL_dalpha;
                    const float gdx = G * dx, gdy = G * dy;
                    const float dG_ddelx = -gdx * co.x - gdy * co.y;
                    const float dG_ddely = -gdy * co.z - gdx * co.y;
                    vals[kRowMean + 0] = dL_dG * dG_ddelx * ddelx_dx;
                    vals[kRowMean + 1] = dL_dG * dG_ddely * ddely_dy;
                    vals[kRowMean + 2] = gd * dchannel_dcolor;
                    vals[kRowConic + 0] = -0.5f * gdx * dx * dL_dG;
                    vals[kRowConic + 1] = -0.5f * gdx * dy * dL_dG;
                    vals[kRowConic + 2] = -0.5f * gdy * dy * dL_dG;
                    vals[kRowOpacity] = G * dL_dalpha;
                }
                // wave totals (full exec mask here: the jj loop is wave-uniform)
                float* dst = s_part + (w * CH + jj) * RSL;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (r < kRowFeat + a.S) {
                        const float sum = wave_sum_to_lane63(vals[r]);
                        if (l == 63) dst[r] = sum;
                    }
                }
            }
            __syncthreads();
            // fixed-order sum of the four wave partials -> one row per instance; re-zero
            for (int i = t; i < jn * (RS / 4); i += kBlock) {
                const int jj = i / (RS / 4), q = i - jj * (RS / 4);
                float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int ww = 0; ww < 4; ++ww) {
                    float4* src = s_part4 + ((ww * CH + jj) * RSL) / 4 + q;
                    const float4 v = *src;
                    acc4.x += v.x; acc4.y += v.y; acc4.z += v.z; acc4.w += v.w;
                    *src = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                reinterpret_cast<float4*>(a.rows + (size_t)s_slot[j0 + jj] * RS)[q] = acc4;
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------------------------
// MFMA variant of the backward blend.
//
// Every per-pixel contribution of one instance is linear in two per-pixel scalars:
//   w = alpha*T          -> colour (w*g_c), feature (w*gf_c) and depth (w*gd) gradients;
//   q = G*dL_dalpha      -> opacity (q), and mean2D / conic gradients through the moments
//                           sum q * {1, x, y, x^2, xy, y^2} of tile-centred pixel coordinates
//                           (dx = d0x - x with d0x the centre offset; expanded at the flush).
// So a wave's reduction over its 64 pixels for 16 instances is two small matrix products,
// [16 inst x 64 px] @ [64 px x 16 ch], done with v_mfma_f32_16x16x4_f32 (exact f32 fma
// chains): per 16 instances 16 MFMAs per 16-channel block instead of (10+S)*6 DPP ops per
// instance. w and q go through a padded LDS image (row stride 66 floats: conflict-free for
// both the row-wise writes and the column-wise A-operand reads).
// ---------------------------------------------------------------------------------------------

// Order this wave's LDS traffic for cross-lane exchange through LDS: wait for the wave's DS
// operations and stop the compiler from moving memory accesses across (it cannot see lanes).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Tuning knobs (experiment builds override them through R3DG_EXTRA_HIPFLAGS). Occupancy is
// set by LDS and VGPRs together; the LDS allocation is rounded up in 2 KiB steps (54,020 B ran
// at two workgroups per CU: 1.63 -> 2.09 ms). The defaults -- 128-instance staging batches and
// a 65-float w|q row stride -- give 40,900 B (four workgroups per CU) and 127 VGPRs (four
// waves per SIMD): 1.63 -> 1.45 ms at M1 against 256 / 66 / three waves.
#ifndef R3DG_BWD_NB
#define R3DG_BWD_NB 128  // instances staged per batch
#endif
#ifndef R3DG_BWD_WQS
#define R3DG_BWD_WQS 65  // padded LDS row stride of the w|q image
#endif
#ifndef R3DG_BWD_WAVES
#define R3DG_BWD_WAVES 4  // waves per SIMD the register allocation targets (SMAX <= 12)
#endif

template <int SMAX>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SMAX <= 12 ? R3DG_BWD_WAVES : 1)))
render_bwd_mfma_kernel(RenderBwdArgs a) {
    constexpr int NB = R3DG_BWD_NB;
    constexpr int NA4 = (4 + SMAX + 3) / 4;       // staged attribute row: colour, depth, features
    constexpr int NR = kRowFeat + SMAX;
    constexpr int RSL = (NR + 3) & ~3;            // LDS partial row stride (floats)
    constexpr int CH = 32;                        // instances per flush chunk (= one compaction mask)
    constexpr int NXB = (4 + SMAX + 15) / 16;     // 16-channel blocks of X = [g0..2, gf0..S-1, gd]
    constexpr int WQS = R3DG_BWD_WQS;             // padded LDS row stride of the w|q image
    constexpr int GRP = 8;                        // instances per MFMA group: rows 0..7 w, 8..15 q
    constexpr int RF4 = 2 + NA4;                  // float4s per render record in HBM
    constexpr int SF4 = 1 + NA4;                  // staged: conic|opacity, attribute row
    __shared__ float4 s_rec[NB * SF4];            // one base address per instance
    __shared__ float2 s_xy[NB];
    __shared__ uint32_t s_slot[NB];
    __shared__ uint32_t s_bits[NB / 32][4];       // [chunk][wave] live-instance masks
    __shared__ float4 s_part4[4 * CH * RSL / 4];  // [wave][chunk instance][RSL]
    __shared__ float s_wq[4][16 * WQS];           // per wave: rows 0..7 w, 8..15 q; [row][pixel]
    __shared__ int s_rowid[4][GRP];
    __shared__ int s_max_last;
    float* s_part = reinterpret_cast<float*>(s_part4);

    const int tile = block_tile(a.tile_order, a.num_tiles);
    if (tile >= a.num_tiles) return;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int px = tx * kTileX + (w & 1) * 8 + (l & 7);
    const int py = ty * kTileY + (w >> 1) * 8 + (l >> 3);
    const bool inside = px < a.W && py < a.H;
    const int pix = inside ? py * a.W + px : 0;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    const int S = a.S;

    const float T_final = inside ? a.final_T[pix] : 0.f;
    float T = T_final;
    const int last = inside ? (int)a.n_contrib[pix] : 0;
    float g[3], gf[SMAX > 0 ? SMAX : 1], gd = 0.f, go = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) g[c] = inside ? a.dL_dpix[a.ca[c] + pix * a.cm[c]] : 0.f;
#pragma unroll
    for (int c = 0; c < SMAX; ++c) gf[c] = (inside && c < S) ? a.dL_dpix_f[a.gflay.a[c] + pix * a.gflay.m[c]] : 0.f;
    if (inside) {
        gd = a.dL_dpix_d[pix];
        go = a.dL_dpix_o[pix];
    }
    const float bg_dot = a.bg[0] * g[0] + a.bg[1] * g[1] + a.bg[2] * g[2];

    // ---- B operands: X[pixel][channel] and Y[pixel][moment] for k-step s (pixel 4s + (l>>4)) ----
    float* wq = s_wq[w];
    float bX[NXB][16];
    // Y[pixel][moment] = [1, x, y, x^2, xy, y^2][nch] at pixel 4*s2 + (l>>4) of this wave: its x
    // offset depends only on s2&1 and its y offset is wave-uniform per s2, so the B operand of k-step
    // s2 is yA[s2&1] + y*(yB[s2&1] + y*yC) (exact: every term but one is a zero product).
    float yA[2], yB[2], yC;
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
            for (int s2 = 0; s2 < 16; ++s2) bX[xb][s2] = wq[(l & 15) * WQS + 4 * s2 + (l >> 4)];
            wave_lds_sync();
        }
        const int nch = l & 15;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float xo = (float)((w & 1) * 8 + 4 * h + (l >> 4)) - 7.5f;
            yA[h] = nch == 0 ? 1.f : (nch == 1 ? xo : (nch == 3 ? xo * xo : 0.f));
            yB[h] = nch == 2 ? 1.f : (nch == 4 ? xo : 0.f);
        }
        yC = nch == 5 ? 1.f : 0.f;
    }

    // The reference keeps one accum_rec per channel (colour, features, depth) and accum_opa; all
    // share the same alpha recurrence and enter dL/dalpha only through their dot with the upstream
    // gradient, so one scalar u = sum_c accum_rec[c] * dL_dchannel[c] + dL_dopacity * accum_opa
    // carries them all. With d = colour.g + dL_dopacity: dL/dalpha = (d - u) * T' - T_final /
    // (1 - alpha) * bg.g, then u += alpha * (d - u) -- the reference's delayed last_alpha /
    // last_color update applied at the end of each contributing step instead. A non-contributing
    // step runs with alpha = 0, which leaves T (1/(1-0) = 1 exactly) and u unchanged.
    if (!a.backward_geometry) {
#pragma unroll
        for (int c = 0; c < SMAX; ++c) gf[c] = 0.f;  // bX already holds the feature grads
    }
    float u = 0.f;
    const float TFB = T_final * bg_dot;

    const int wmax = __builtin_amdgcn_readfirstlane(wave_max_int(last));
    if (t == 0) s_max_last = 0;
    for (int i = t; i < 4 * CH * RSL / 4; i += kBlock) s_part4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    if (l == 0) atomicMax(&s_max_last, wmax);
    __syncthreads();
    const int max_last = s_max_last;
    const int RS = a.RS;
    for (int p = max_last + t; p < n; p += kBlock) {
        const uint32_t gid = a.point_list[range.x + p];
        const uint32_t slot = record_slot(a.records[(size_t)gid * (2 + NA4) + 1], tx, ty, a.grid_x, a.grid_y);
        float4* row = reinterpret_cast<float4*>(a.rows + (size_t)slot * RS);
        for (int q = 0; q < RS / 4; ++q) row[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // partial-row slot of each X channel / Y moment (col l&15 of the MFMA result)
    const int nch = l & 15;
    int xslot[NXB];
#pragma unroll
    for (int xb = 0; xb < NXB; ++xb) {
        const int ch = xb * 16 + nch;
        xslot[xb] = ch < 3 ? kRowColor + ch : (ch - 3 < S ? kRowFeat + (ch - 3) : (ch == 3 + S ? kRowMean + 2 : -1));
    }
    // moments: S0 -> opacity slot, Sx, Sy, Sxx, Sxy, Syy -> mean x, mean y, conic x, y, w slots
    const int yslot = nch == 0 ? kRowOpacity : (nch == 1 ? 0 : (nch == 2 ? 1 : (nch < 6 ? nch : -1)));
    const float ctx = (float)(tx * kTileX) + 7.5f, cty = (float)(ty * kTileY) + 7.5f;
    const bool x_half = (l >> 4) < 2;  // result rows 0..7 (w . X) live in lanes 0..31, 8..15 (q . Y) in 32..63

    for (int hi = max_last; hi > 0; hi -= NB) {
        const int cnt = min(NB, hi);
        __syncthreads();
        uint32_t m = 0;
        if (t < cnt) {
            const uint32_t k = range.x + (uint32_t)(hi - 1 - t);
            const uint32_t gid = a.point_list[k];
            // one contiguous render record per Gaussian (r3dg_kernels.h record_f4), staged verbatim
            const float4* rec = a.records + (size_t)gid * RF4;
            float4 r[RF4];
#pragma unroll
            for (int q = 0; q < RF4; ++q) r[q] = rec[q];
            s_rec[t * SF4] = r[0];
#pragma unroll
            for (int q = 0; q < NA4; ++q) s_rec[t * SF4 + 1 + q] = r[2 + q];
            s_xy[t] = make_float2(r[1].x, r[1].y);
            s_slot[t] = record_slot(r[1], tx, ty, a.grid_x, a.grid_y);
            m = quadrant_mask(make_float2(r[1].x, r[1].y), r[0], tx * kTileX, ty * kTileY, a.cull);
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const unsigned long long bal = __ballot((m >> b) & 1u);
            if (l == 0 && w < NB / 64) {
                s_bits[2 * w][b] = (uint32_t)bal;
                s_bits[2 * w + 1][b] = (uint32_t)(bal >> 32);
            }
        }
        __syncthreads();
        const int jmin = hi - wmax;  // instances j < jmin lie beyond every pixel of this wave
        for (int c = 0; c * CH < cnt; ++c) {
            uint32_t bits = __builtin_amdgcn_readfirstlane(s_bits[c][w]);
            const int lo = jmin - c * CH;
            if (lo >= CH) bits = 0;
            else if (lo > 0) bits &= ~0u << lo;
            int r = 0;  // rows filled in the current MFMA group
            // One blend step of the reference's per-pixel loop (backward.cu:520-611), predicated
            // rather than branched: every LDS read is issued up front and a non-contributing pixel
            // (outside, past n_contrib, power > 0 or alpha < 1/255) leaves its state unchanged.
            auto step = [&](int j, bool live, float& wv, float& qv) {
#pragma clang fp contract(off)  // explicit FMAs only: both unrolled copies round alike
                const int ju = __builtin_amdgcn_readfirstlane(j);  // uniform addresses
                const float4* rj = s_rec + ju * SF4;
                const float4 co = rj[0];
                const float2 xy = s_xy[ju];
                float v[NA4 * 4];
#pragma unroll
                for (int q = 0; q < NA4; ++q) {
                    const float4 rr = rj[1 + q];
                    v[4 * q] = rr.x; v[4 * q + 1] = rr.y; v[4 * q + 2] = rr.z; v[4 * q + 3] = rr.w;
                }
                const int p = hi - 1 - j;  // position in the tile range (reference `contributor`)
                const float power = gauss_power(co, xy.x - pfx, xy.y - pfy);
                const float G = __expf(power);
                const float alpha = fminf(0.99f, co.w * G);
                // p < last is false for pixels outside the image (last = 0 there)
                const bool ok = live && p < last && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
                const float ae = ok ? alpha : 0.f;
                const float Ge = ok ? G : 0.f;
                const float rinv = __builtin_amdgcn_rcpf(1.f - ae);
                const float Tn = T * rinv;
                float d = __builtin_fmaf(v[0], g[0], go);
                d = __builtin_fmaf(v[1], g[1], d);
                d = __builtin_fmaf(v[2], g[2], d);
                d = __builtin_fmaf(v[3], gd, d);
#pragma unroll
                for (int c2 = 0; c2 < SMAX; ++c2) d = __builtin_fmaf(v[4 + c2], gf[c2], d);
                const float diff = d - u;
                const float dL_dalpha = rinv * __builtin_fmaf(T, diff, -TFB);
                wv = ae * Tn;
                qv = Ge * dL_dalpha;
                T = Tn;
                u = __builtin_fmaf(ae, diff, u);
            };
            while (bits) {
                // two compacted instances per iteration: the second one's LDS reads and exp
                // overlap the first one's dependent chain
                const int jj0 = __builtin_ctz(bits);
                bits &= bits - 1;
                const bool has1 = bits != 0u;
                const int jj1 = has1 ? __builtin_ctz(bits) : jj0;
                bits &= bits - 1;
                float wv0, qv0, wv1, qv1;
                step(c * CH + jj0, true, wv0, qv0);
                step(c * CH + jj1, has1, wv1, qv1);
                wq[r * WQS + l] = wv0;
                wq[(GRP + r) * WQS + l] = qv0;
                wq[(r + 1) * WQS + l] = wv1;
                wq[(GRP + r + 1) * WQS + l] = qv1;
                if (l == 0) {
                    s_rowid[w][r] = jj0;
                    s_rowid[w][r + 1] = jj1;
                }
                r += has1 ? 2 : 1;
                if (r == GRP || bits == 0) {
                    // [8 w rows | 8 q rows] x [64 px] against X (16 ch) and Y (moments): rows 0..7
                    // of w.X and rows 8..15 of q.Y are the useful halves
                    wave_lds_sync();
                    floatx4 accX[NXB], accY = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int xb = 0; xb < NXB; ++xb) accX[xb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s2 = 0; s2 < 16; ++s2) {
                        const float av = wq[(l & 15) * WQS + 4 * s2 + (l >> 4)];
#pragma unroll
                        for (int xb = 0; xb < NXB; ++xb)
                            accX[xb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bX[xb][s2], accX[xb], 0, 0, 0);
                        const float yo = (float)((w >> 1) * 8 + (s2 >> 1)) - 7.5f;
                        const float by = yA[s2 & 1] + yo * (yB[s2 & 1] + yo * yC);
                        accY = __builtin_amdgcn_mfma_f32_16x16x4f32(av, by, accY, 0, 0, 0);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = (l >> 4) * 4 + i;        // D row held by this lane
                        const int gi = x_half ? row : row - GRP;  // group instance
                        if (gi < r) {
                            float* dst = s_part + (w * CH + s_rowid[w][gi]) * RSL;
                            if (x_half) {
#pragma unroll
                                for (int xb = 0; xb < NXB; ++xb)
                                    if (xslot[xb] >= 0) dst[xslot[xb]] = accX[xb][i];
                            } else if (yslot >= 0) {
                                dst[yslot] = accY[i];
                            }
                        }
                    }
                    wave_lds_sync();
                    r = 0;
                }
            }
            __syncthreads();
            // fixed-order sum of the four wave partials, moments -> mean2D / conic grads, one row
            // per instance, re-zero the partials
            const int jn = min(CH, cnt - c * CH);
            constexpr int NC4 = RSL / 4;  // float4 columns; column pair 0|1 holds the moments
            for (int it = t; it < jn * (NC4 - 1); it += kBlock) {
                const int jj = it / (NC4 - 1);
                const int col = it - jj * (NC4 - 1) + 1;  // 1 -> columns 0 and 1, else column col
                const int j = c * CH + jj;
                float4* row = reinterpret_cast<float4*>(a.rows + (size_t)s_slot[j] * RS);
                if (col == 1) {
                    float4 u0 = make_float4(0.f, 0.f, 0.f, 0.f), u1 = u0;
#pragma unroll
                    for (int ww = 0; ww < 4; ++ww) {
                        float4* src = s_part4 + (ww * CH + jj) * NC4;
                        const float4 v0 = src[0], v1 = src[1];
                        u0.x += v0.x; u0.y += v0.y; u0.z += v0.z; u0.w += v0.w;
                        u1.x += v1.x; u1.y += v1.y; u1.z += v1.z; u1.w += v1.w;
                        src[0] = make_float4(0.f, 0.f, 0.f, 0.f);
                        src[1] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                    const float2 xy = s_xy[j];
                    const float4 co = s_rec[j * SF4];
                    // slots: 0 Sx, 1 Sy, 2 depth, 3 Sxx, 4 Sxy, 5 Syy, 6 S0 (= opacity grad), 7 colour r
                    const float S0 = u1.z, Sx = u0.x, Sy = u0.y, Sxx = u0.w, Sxy = u1.x, Syy = u1.y;
                    const float d0x = xy.x - ctx, d0y = xy.y - cty;
                    const float Sdx = d0x * S0 - Sx, Sdy = d0y * S0 - Sy;
                    const float Sdxdx = d0x * d0x * S0 - 2.f * d0x * Sx + Sxx;
                    const float Sdxdy = d0x * d0y * S0 - d0x * Sy - d0y * Sx + Sxy;
                    const float Sdydy = d0y * d0y * S0 - 2.f * d0y * Sy + Syy;
                    row[0] = make_float4(-0.5f * a.W * co.w * (co.x * Sdx + co.y * Sdy),
                                         -0.5f * a.H * co.w * (co.z * Sdy + co.y * Sdx), u0.z, -0.5f * co.w * Sdxdx);
                    row[1] = make_float4(-0.5f * co.w * Sdxdy, -0.5f * co.w * Sdydy, S0, u1.w);
                } else {
                    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int ww = 0; ww < 4; ++ww) {
                        float4* src = s_part4 + (ww * CH + jj) * NC4 + col;
                        const float4 v0 = *src;
                        u.x += v0.x; u.y += v0.y; u.z += v0.z; u.w += v0.w;
                        *src = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                    if (4 * col < RS) row[col] = u;
                }
            }
            __syncthreads();
        }
    }
}

template <int SMAX>
static hipError_t launch_bwd_s(const RenderBwdArgs& a, hipStream_t stream) {
    const char* e = getenv("R3DG_BWD");  // "dpp" selects the DPP-reduction variant (A/B and cross-check)
    const bool use_dpp = e && e[0] == 'd';
    if (use_dpp)
        hipLaunchKernelGGL((render_bwd_dpp_kernel<SMAX>), dim3(padded_tile_grid(a.num_tiles)), dim3(kBlock), 0, stream,
                           a);
    else
        hipLaunchKernelGGL((render_bwd_mfma_kernel<SMAX>), dim3(padded_tile_grid(a.num_tiles)), dim3(kBlock), 0,
                           stream, a);
    return hipGetLastError();
}

hipError_t launch_render_backward(const RenderBwdArgs& a, hipStream_t stream) {
    if (a.num_tiles == 0) return hipSuccess;
    if (a.S == 0) return launch_bwd_s<0>(a, stream);
    if (a.S <= 4) return launch_bwd_s<4>(a, stream);
    if (a.S <= 8) return launch_bwd_s<8>(a, stream);
    if (a.S <= 12) return launch_bwd_s<12>(a, stream);
    if (a.S <= 16) return launch_bwd_s<16>(a, stream);
    if (a.S <= 24) return launch_bwd_s<24>(a, stream);
    return launch_bwd_s<32>(a, stream);
}

// ---------------------------------------------------------------------------------------------
// per-Gaussian: sum of gradient rows + preprocessing backward
// ---------------------------------------------------------------------------------------------

// backward.cu:20-139 (computeColorFromSH backward). dL_dRGB already clamp-masked.
__device__ static void sh_backward(int deg, int M, float3 pos, const float* campos, const float* sh,
                                   const float* dRGB, float* dL_dmean, float* dsh) {
    const float dox = pos.x - campos[0], doy = pos.y - campos[1], doz = pos.z - campos[2];
    const float len = sqrtf(dox * dox + doy * doy + doz * doz);
    const float x = dox / len, y = doy / len, z = doz / len;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    float ddx[3] = {0.f, 0.f, 0.f}, ddy[3] = {0.f, 0.f, 0.f}, ddz[3] = {0.f, 0.f, 0.f};
    float b[16];
    b[0] = SH_C0;
    b[1] = -SH_C1 * y; b[2] = SH_C1 * z; b[3] = -SH_C1 * x;
    b[4] = SH_C2_0 * xy; b[5] = SH_C2_1 * yz; b[6] = SH_C2_2 * (2.f * zz - xx - yy); b[7] = SH_C2_3 * xz;
    b[8] = SH_C2_4 * (xx - yy);
    b[9] = SH_C3_0 * y * (3.f * xx - yy); b[10] = SH_C3_1 * xy * z; b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
    b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy); b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
    b[14] = SH_C3_5 * z * (xx - yy); b[15] = SH_C3_6 * x * (xx - 3.f * yy);
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
        for (int c = 0; c < 3; ++c) dsh[3 * i + c] = i < ncoef ? b[i] * dRGB[c] : 0.f;
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
    a.dL_dmeans2D[3 * g + 0] = s[kRowMean + 0];
    a.dL_dmeans2D[3 * g + 1] = s[kRowMean + 1];
    a.dL_dmeans2D[3 * g + 2] = s[kRowMean + 2];
    a.dL_dopacity[g] = s[kRowOpacity];
    a.dL_dcolors[3 * g + 0] = s[kRowColor + 0];
    a.dL_dcolors[3 * g + 1] = s[kRowColor + 1];
    a.dL_dcolors[3 * g + 2] = s[kRowColor + 2];
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
        if (c < a.S) a.dL_dfeatures[(size_t)g * a.S + c] = s[kRowFeat + c];

    float* dmean3 = a.dL_dmeans3D + 3 * g;
    float* dcov = a.dL_dcov3D + 6 * g;
    if (!(a.radii[g] > 0)) {
        dmean3[0] = dmean3[1] = dmean3[2] = 0.f;
        for (int i = 0; i < 6; ++i) dcov[i] = 0.f;
        for (int i = 0; i < 3 * a.M; ++i) shl[i] = 0.f;
        for (int i = 0; i < 3; ++i) a.dL_dscales[3 * g + i] = 0.f;
        for (int i = 0; i < 4; ++i) a.dL_drotations[4 * g + i] = 0.f;
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
        cov3d_backward(sc, a.scale_modifier, q, dcov, a.dL_dscales + 3 * g, a.dL_drotations + 4 * g);
    } else {
        for (int i = 0; i < 3; ++i) a.dL_dscales[3 * g + i] = 0.f;
        for (int i = 0; i < 4; ++i) a.dL_drotations[4 * g + i] = 0.f;
    }
}

template <int SMAX>
__global__ void __launch_bounds__(256) gather_bwd_kernel(GatherBwdArgs a) {
    constexpr int NR = kRowFeat + SMAX;
    constexpr int NQ = (NR + 3) / 4;       // float4 columns of a gradient row (upper bound)
    constexpr int LPG = NQ <= 8 ? 8 : 16;  // lanes per Gaussian in the row-sum phase
    constexpr int SHS = 49;                // LDS stride of one Gaussian's SH block (<= 48 used, odd)
    constexpr int SUMF = 256 * NQ * 4, SHF = 256 * SHS;
    __shared__ float4 s_buf4[((SUMF > SHF ? SUMF : SHF) + 3) / 4];
    float* s_buf = reinterpret_cast<float*>(s_buf4);
    const int t = threadIdx.x;
    const int g0 = blockIdx.x * 256;
    const int nq = a.RS / 4;

    // ---- phase 1: per-Gaussian sums of its contiguous rows. LPG lanes per Gaussian, lane c owns
    // float4 column c, so a row is read as one contiguous 16*nq-byte segment. Rows are added in
    // slot order, the same fixed order for every run.
    {
        const int c = t % LPG, gl0 = t / LPG;
        const float4* col = reinterpret_cast<const float4*>(a.rows) + c;
        for (int r = 0; r < LPG; ++r) {
            const int gl = r * (256 / LPG) + gl0;
            const int g = g0 + gl;
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            if (g < a.P && c < nq && a.radii[g] > 0) {
                uint32_t k = g == 0 ? 0u : a.offsets[g - 1];
                const uint32_t end = a.offsets[g];
                for (; k + 4 <= end; k += 4) {
                    const float4 v0 = col[(size_t)k * nq], v1 = col[(size_t)(k + 1) * nq];
                    const float4 v2 = col[(size_t)(k + 2) * nq], v3 = col[(size_t)(k + 3) * nq];
                    acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
                    acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
                    acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
                    acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
                }
                for (; k < end; ++k) {
                    const float4 v = col[(size_t)k * nq];
                    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
                }
            }
            if (c < NQ) s_buf4[gl * NQ + c] = acc;
        }
    }
    __syncthreads();
    const int g = g0 + t;
    float s[NQ * 4];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float4 v = s_buf4[t * NQ + q];
        s[4 * q] = v.x; s[4 * q + 1] = v.y; s[4 * q + 2] = v.z; s[4 * q + 3] = v.w;
    }
    __syncthreads();
    // ---- SH coefficients of the block's Gaussians: one coalesced copy into LDS ----
    const int M3 = 3 * a.M;
    const int ng = min(256, a.P - g0);
    float* shl = s_buf + t * SHS;
    if (a.sh && a.dL_dsh) {
        const float* src = a.sh + (size_t)g0 * M3;
        for (int f = t; f < ng * M3; f += 256) {
            const int gg = f / M3;
            s_buf[gg * SHS + (f - gg * M3)] = src[f];
        }
    }
    __syncthreads();
    if (g < a.P) gather_gaussian<SMAX>(a, g, s, shl);
    __syncthreads();
    if (a.dL_dsh) {
        float* dst = a.dL_dsh + (size_t)g0 * M3;
        for (int f = t; f < ng * M3; f += 256) {
            const int gg = f / M3;
            dst[f] = s_buf[gg * SHS + (f - gg * M3)];
        }
    }
}

template <int SMAX>
static hipError_t launch_gather_s(const GatherBwdArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL((gather_bwd_kernel<SMAX>), dim3((a.P + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_gather_backward(const GatherBwdArgs& a, hipStream_t stream) {
    if (a.P == 0) return hipSuccess;
    if (a.S == 0) return launch_gather_s<0>(a, stream);
    if (a.S <= 4) return launch_gather_s<4>(a, stream);
    if (a.S <= 8) return launch_gather_s<8>(a, stream);
    if (a.S <= 12) return launch_gather_s<12>(a, stream);
    if (a.S <= 16) return launch_gather_s<16>(a, stream);
    if (a.S <= 24) return launch_gather_s<24>(a, stream);
    return launch_gather_s<32>(a, stream);
}

}  // namespace r3dg
