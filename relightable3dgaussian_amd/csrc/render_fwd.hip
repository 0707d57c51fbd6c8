// render_fwd.hip -- front-to-back alpha blend per 16x16 screen tile (gfx950, wave64).
//
// Restates reference forward.cu:388-561 (renderCUDA) with an MI355X layout:
//   * one 256-thread workgroup per tile; each wave64 owns an 8x8 quadrant (square, so the
//     per-wave footprint test below rejects more Gaussians than 16x4 strips would);
//   * the render records of the next 64-instance batch are copied HBM -> LDS by LDS-DMA while the
//     current batch blends (render_fwd_glds_kernel; one block barrier per batch, 8 waves/SIMD);
//   * a conservative per-quadrant footprint test (minimum of the conic form over the quadrant
//     against the widened alpha >= 1/255 threshold, r3dg_common.h rect_culled) decides which
//     instances a wave visits. Skipping is exact: a skipped instance would have failed the
//     reference's alpha test on every pixel of the quadrant (tests/test_gpu_parity.py checks cull
//     on == cull off bit for bit, also on needle-shaped splats);
//   * every wave records which staged instances at least one of its pixels blended: one byte
//     per sorted position (bit 2q + h = half h of quadrant q), the exact visit list of the backward;
//   * early exit per wave (ballot) and per block (__syncthreads_count), as the reference;
//   * XCD-aware tile order (r3dg_kernels.h).
// render_fwd_glds_kernel<SMAX, true> blends the splat-shader colour as well (non-default splat shaders).
#include "r3dg_common.h"
#include "r3dg_kernels.h"
#include "r3dg_tilesort.h"

namespace r3dg {

#ifdef R3DG_EXP_COUNT
R3DG_EXP_READER(r3dg_exp_counters_fwd)
#endif

#ifndef R3DG_FWD_WAVES
#define R3DG_FWD_WAVES 8  // waves per SIMD the register allocation targets (SMAX <= 12): 64 VGPR
#endif

// ---------------------------------------------------------------------------------------------
// The default-shader blend (render records only): the records of batch b+1 are copied HBM -> LDS
// by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no staging stores) while the waves blend batch b,
// so the record round trip leaves the critical path and a batch costs one block barrier (the
// early-exit count). Every wave evaluates the exact quadrant cull of the staged instances for its
// own quadrant. Staging layout: column q (float4 q of the render record) of instance j at
// [q * NB + j].
// ---------------------------------------------------------------------------------------------
#ifndef R3DG_FWD_TSIGN
#define R3DG_FWD_TSIGN 1  // the pixel's stop kept as T's sign (no done mask); 0: a done mask (rounds 1-5)
#endif
#ifndef R3DG_FWD_SWALK
#define R3DG_FWD_SWALK 1  // the pair loop's live-mask walk by s_ff1 + s_bitset0 (inline asm)
#endif
#ifndef R3DG_FWD_HALF
#define R3DG_FWD_HALF 0  // 1: each 8x4 half of a wave's quadrant walks its own cull list (measured 3.4 % slower: profiles/r06/fwd_half_ab)
#endif
#ifndef R3DG_FWDG_NB
#define R3DG_FWDG_NB 64  // instances per staged batch (two resident: 12.3 KB, 64 VGPRs -> 8 waves/SIMD;
                         // 128: 24.6 KB -> 6 waves/SIMD, measured 0.480 vs 0.447 ms at M1)
#endif

// SHADER (non-default splat shaders, forward.cu:907-971): the splat shaders edit the shader colour
// and the features after the render records were written (the records keep the caller's features:
// the backward reads those, as the reference's does), so the staged columns are the record's conic,
// position and [colour, depth] float4 followed by the shader record [shader colour, 0 | shaded
// features] (RenderFwdArgs::shader_rec, NA4 float4 per Gaussian, the attribute row's layout) -- the
// same DMA staging, cull, step and contribution bits as the default path.
template <int SMAX, bool SHADER>
// (SMAX = 0 keeps the 6-wave target: at 8 the compiler spills 14 SGPRs)
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SMAX == 0 ? 6 : SMAX <= 12 ? R3DG_FWD_WAVES : 1)))
render_fwd_glds_kernel(RenderFwdArgs a) {
    constexpr int NB = R3DG_FWDG_NB;
    constexpr int NH = NB / 64;                // staged instances per lane
    constexpr int NA4 = (4 + SMAX + 3) / 4;    // float4 per attribute row
    constexpr int RF4 = 2 + NA4;               // float4 per render record
    constexpr int NCOL = RF4 + (SHADER ? 1 : 0);  // staged float4 columns per instance (SHADER: 3 + NA4)
    constexpr int SBUF = NCOL * NB;            // float4 per staging buffer
    constexpr int NCP = NCOL * NH;             // DMA wave-instructions per batch
    static_assert(NB == 64, "one 64-bit contribution word per wave and batch");
    // one LDS array: [2 staging buffers | 2 x 64 x 4 contribution flags (batch buffer, instance, wave)
    // | the tile's sorted Gaussian ids (fused sort)]; the fused sort's scratch aliases the staging
    constexpr int SORT4 = (int)((sizeof(TileSortLds<kFusedSortMax / kSortBT>) + 15) / 16);
    constexpr int STG = 2 * SBUF > SORT4 ? 2 * SBUF : SORT4;  // float4 of staging / sort scratch
    __shared__ float4 s_lds[STG + 64 + kFusedSortMax / 4];
    uint8_t* const s_cf = reinterpret_cast<uint8_t*>(s_lds + STG);
    uint32_t* const s_ids = reinterpret_cast<uint32_t*>(s_lds + STG + 64);
    reinterpret_cast<uint32_t*>(s_cf)[threadIdx.x] = 0u;  // 2 x 64 x 8 flag bytes, before the first barrier

    const int tile = block_tile(a.tile_order, a.num_tiles);
    if (tile >= a.num_tiles) return;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int px = tx * kTileX + (w & 1) * 8 + (l & 7);
    const int py = ty * kTileY + (w >> 1) * 8 + (l >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    const float qx0 = (float)(tx * kTileX + (w & 1) * 8), qy0 = (float)(ty * kTileY + (w >> 1) * 8);
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);

    // fused depth sort (block-uniform): the tile's (depth bits, id) pairs sorted in the prologue
    // (r3dg_tilesort.h), ids kept in LDS for the staging and written out for the backward; saves
    // the standalone sort launch, whose time is its barriers' latency, not its work
    const bool fused = a.pairs != nullptr && n <= kFusedSortMax;
    if (fused && n > 0) {
        constexpr int IPT = kFusedSortMax / kSortBT;
        uint32_t keys[IPT], vals[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int i = t * IPT + k;
            const uint2 kv = i < n ? a.pairs[range.x + i] : make_uint2(0xffffffffu, 0xffffffffu);
            keys[k] = kv.x;
            vals[k] = kv.y;
        }
#ifndef R3DG_EXP_NOSORT  // timing experiment only (results invalid): the blend without the fused sort
        if (n > 1) sort_pairs_chunk<IPT>(keys, vals, n, *reinterpret_cast<TileSortLds<IPT>*>(s_lds));
#endif
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int i = t * IPT + k;
            if (i < n) {
                s_ids[i] = vals[k];
                a.point_list_out[range.x + i] = vals[k];
            }
        }
        __syncthreads();
    }

#if R3DG_FWD_TSIGN
    // A pixel's stop is T's sign: the reference sets `done` when a contributing instance would take T
    // below 1e-4 and keeps T; here T becomes -|T| (one v_cndmask with source modifiers), every later
    // test_T = T (1 - alpha) < 0 stops again and leaves it there, and final_T is |T|. No separate
    // done mask, which the compiler moved between SGPR and VGPR form at every step.
    float T = inside ? 1.0f : -1.0f;
#define R3DG_DONE (T < 0.0f)
#else
    bool done = !inside;
    float T = 1.0f;
#define R3DG_DONE done
#endif
    uint32_t last = 0;
    float C[3] = {0.f, 0.f, 0.f}, F[SMAX > 0 ? SMAX : 1];
    float CS[SHADER ? 3 : 1];
#pragma unroll
    for (int c = 0; c < (SHADER ? 3 : 1); ++c) CS[c] = 0.f;
    float Dp = 0.f, Op = 0.f;
#pragma unroll
    for (int c = 0; c < SMAX; ++c) F[c] = 0.f;

    // Gaussian of staged instance h * 64 + l of the batch at tile position b0 (tail lanes clamp to
    // the tile's last instance, so every DMA lane reads a valid record)
    auto load_gids = [&](int b0, uint32_t (&gd)[NH]) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const int i = min(b0 + h * 64 + l, n - 1);
            gd[h] = fused ? s_ids[i] : a.point_list[range.x + (uint32_t)i];
        }
    };
    // the DMA is inline asm: the compiler does not wait for it before the LDS reads of the other
    // buffer; the batch loop waits for it explicitly (vmcnt(0) before the batch barrier)
    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)s_lds;
    auto issue = [&](const uint32_t (&gd)[NH], int buf) {
#pragma unroll
        for (int k = 0; k < NCP; ++k) {
            if ((k & 3) != w) continue;  // wave-uniform
            // lane l of instruction k: column k / NH, instance (k % NH) * 64 + l -> entry k * 64 + l
            const float4* src = (SHADER && k / NH >= 3) ? a.shader_rec + (size_t)gd[k % NH] * NA4 + (k / NH - 3)
                                                       : a.records + (size_t)gd[k % NH] * RF4 + k / NH;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)((buf * SBUF + k * 64) * 16));
            int keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
        }
    };

    uint32_t gnext[NH];
    if (n > 0) {
        uint32_t g0[NH];
        load_gids(0, g0);
        issue(g0, 0);
        if (n > NB) load_gids(NB, gnext);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // Contribution bits for the backward (render_bwd.hip): the byte of sorted position p holds bit
    // 2q + h when a pixel of half h (rows 0-3 / 4-7) of quadrant q blended instance p. Every
    // accumulating lane of wave w sets the LDS flag byte [batch buffer][instance][2w + h] (all write
    // the same 1: no per-step ballot or scalar work); after the next batch barrier wave 0 folds each
    // instance's eight flag bytes into the contribution byte, stores it and clears the flags for
    // their reuse two batches on. Positions past a block's early exit are never written: the
    // backward only visits positions below the tile's largest n_contrib.
    // (wave 0 also counts the backward's visits per quadrant: the tile's backward work, below)
    int vq0 = 0, vq1 = 0, vq2 = 0, vq3 = 0;
    const bool wave0 = __builtin_amdgcn_readfirstlane(w) == 0;  // uniform: the counters stay scalar
    auto write_bits = [&](int b0, int cnt, int bb) {
        if (wave0) {
            uint32_t v = 0u;
            if (l < cnt) {
                uint2* f = reinterpret_cast<uint2*>(s_cf) + 64 * bb + l;
                const uint2 fw = *f;
                *f = make_uint2(0u, 0u);
                v = (fw.x & 1u) | (fw.x >> 7 & 2u) | (fw.x >> 14 & 4u) | (fw.x >> 21 & 8u) |
                    ((fw.y & 1u) | (fw.y >> 7 & 2u) | (fw.y >> 14 & 4u) | (fw.y >> 21 & 8u)) << 4;
                a.contrib[range.x + (uint32_t)(b0 + l)] = (uint8_t)v;
            }
            if (a.bwd_work) {
                vq0 += __builtin_popcountll(__ballot(v & 0x03u));
                vq1 += __builtin_popcountll(__ballot(v & 0x0cu));
                vq2 += __builtin_popcountll(__ballot(v & 0x30u));
                vq3 += __builtin_popcountll(__ballot(v & 0xc0u));
            }
        }
    };
    int buf = 0;
    int base = 0;
    for (; base < n; base += NB) {
        // batch `base` has landed (every wave waited for its own DMA) and nobody reads the other
        // buffer any more
        const bool all_done = __syncthreads_count(R3DG_DONE) == kBlock;
        // the previous batch's flags, before the DMA issue: folding them after wave 0's DMA issue
        // measured 0.556 vs 0.480 ms
        if (base > 0) write_bits(base - NB, NB, buf ^ 1);
        if (all_done) break;
        if (base + NB < n) {  // block-uniform: stage the next batch while this one blends
            issue(gnext, buf ^ 1);
            if (base + 2 * NB < n) load_gids(base + 2 * NB, gnext);
        }
        const float4* st = s_lds + buf * SBUF;
        const int cnt = min(NB, n - base);
#if R3DG_FWD_HALF
        // the exact cull per 8x4 half of the quadrant: one live mask per half
        unsigned long long bt, bb;
        {
            bool mt = false, mb = false;
            if (l < cnt) {
                const float4 co = st[l], r1 = st[NB + l];
                half_live(make_float2(r1.x, r1.y), co, uniform_f(qx0), uniform_f(qx0 + 7.0f), uniform_f(qy0),
                          uniform_f(qy0 + 3.0f), uniform_f(qy0 + 4.0f), uniform_f(qy0 + 7.0f), a.cull, mt, mb);
            }
            bt = __ballot(mt);
            bb = __ballot(mb);
        }
#else
        unsigned long long bits[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const int j = h * 64 + l;
            bool mine = false;
            if (j < cnt) {
                const float4 co = st[j], r1 = st[NB + j];
                mine = quadrant_live(make_float2(r1.x, r1.y), co, qx0, qy0, a.cull);
            }
            bits[h] = __ballot(mine);
        }
#endif
        // j: the staged instance (R3DG_FWD_HALF: per lane, one per half of the wave)
        auto step = [&](int j, bool live, float opacity, float power, float G) {
#pragma clang fp contract(off)  // explicit FMAs only: both unrolled copies round alike
#if R3DG_FWD_HALF
            const int ju = j;
#else
            const int ju = __builtin_amdgcn_readfirstlane(j);
#endif
            float v[NA4 * 4];
#pragma unroll
            for (int q = 0; q < NA4; ++q) {
                // SHADER: [colour, depth] from the record, the shaded features from the shader record
                const float4 r = st[((SHADER && q > 0) ? 3 + q : 2 + q) * NB + ju];
                v[4 * q] = r.x; v[4 * q + 1] = r.y; v[4 * q + 2] = r.z; v[4 * q + 3] = r.w;
            }
            const float alpha = fminf(0.99f, opacity * G);  // bit-identical to the oracle
#if R3DG_FWD_TSIGN
            const bool contrib = live && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            const float test_T = T * (1.0f - alpha);
            const bool stop = test_T < 0.0001f;  // also every step after the pixel's stop (T < 0)
            if (contrib && stop) T = -fabsf(T);
#else
            const bool contrib = live && !done && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            const float test_T = T * (1.0f - alpha);
            const bool stop = test_T < 0.0001f;
            done = done || (contrib && stop);
#endif
#ifdef R3DG_EXP_COUNT
            {
                const unsigned long long acc_b = __ballot(contrib && !stop);
                if (l == 0) {
                    R3DG_EXP_ADD(4, __builtin_popcountll(acc_b));
                    R3DG_EXP_ADD(5, acc_b != 0ull ? 1 : 0);
                }
            }
#endif
            if (contrib && !stop) {
#if R3DG_ATTR_B128
                // the unused pad channel kept live: one ds_read_b128 (4 LDS-array cycles) for the
                // last row instead of a ds_read_b96 (8)
                if constexpr ((4 + SMAX) % 4 != 0) asm volatile("" ::"v"(v[NA4 * 4 - 1]));
#endif
                const float wgt = alpha * T;
                C[0] = __builtin_fmaf(v[0], wgt, C[0]);
                C[1] = __builtin_fmaf(v[1], wgt, C[1]);
                C[2] = __builtin_fmaf(v[2], wgt, C[2]);
                if constexpr (SHADER) {
                    const float4 sc = st[3 * NB + ju];
                    CS[0] = __builtin_fmaf(sc.x, wgt, CS[0]);
                    CS[1] = __builtin_fmaf(sc.y, wgt, CS[1]);
                    CS[2] = __builtin_fmaf(sc.z, wgt, CS[2]);
                }
#pragma unroll
                for (int c2 = 0; c2 < SMAX; ++c2) F[c2] = __builtin_fmaf(v[4 + c2], wgt, F[c2]);
                Dp = __builtin_fmaf(v[3], wgt, Dp);
                Op += wgt;
                T = test_T;
                last = (uint32_t)(base + j + 1);
                s_cf[(buf * 64 + ju) * 8 + 2 * w + (l >> 5)] = 1;  // every accumulating lane of a half: one byte
            }
        };
#if R3DG_FWD_HALF
        // Each half of the wave walks its own live list, two instances per iteration; a half whose
        // 32 pixels are all done, or whose list ran out, idles (live = false) while the other walks on.
        const bool top = l < 32;
        {
            const unsigned long long nd = __ballot(!R3DG_DONE);
            if ((uint32_t)nd == 0u) bt = 0ull;
            if ((uint32_t)(nd >> 32) == 0u) bb = 0ull;
        }
        while (bt | bb) {
            const int t0 = bt ? (int)__builtin_ctzll(bt) : -1;
            bt &= bt - 1;
            const int t1 = bt ? (int)__builtin_ctzll(bt) : -1;
            bt &= bt - 1;
            const int b0 = bb ? (int)__builtin_ctzll(bb) : -1;
            bb &= bb - 1;
            const int b1 = bb ? (int)__builtin_ctzll(bb) : -1;
            bb &= bb - 1;
            const int s0 = top ? t0 : b0, s1 = top ? t1 : b1;
            const bool live0 = s0 >= 0, live1 = s1 >= 0;
            const int j0 = live0 ? s0 : 0, j1 = live1 ? s1 : j0;  // valid staging slots either way
            const float4 co0 = st[j0], co1 = st[j1];
            const float2 xy0 = *reinterpret_cast<const float2*>(st + NB + j0);
            const float2 xy1 = *reinterpret_cast<const float2*>(st + NB + j1);
            const float pw0 = gauss_power(co0, xy0.x - pfx, xy0.y - pfy);
            const float pw1 = gauss_power(co1, xy1.x - pfx, xy1.y - pfy);
            const f32x2 G = {blend_expf(pw0), blend_expf(pw1)};
            step(j0, live0, co0.w, pw0, G.x);
            step(j1, live1, co1.w, pw1, G.y);
            const unsigned long long nd = __ballot(!R3DG_DONE);
            if ((uint32_t)nd == 0u) bt = 0ull;
            if ((uint32_t)(nd >> 32) == 0u) bb = 0ull;
        }
#else
        static_assert(NH == 1, "one 64-bit live mask per batch");
        unsigned long long b = bits[0];
        if (l == 0) R3DG_EXP_ADD(3, __builtin_popcountll(b));
        if (__ballot(!R3DG_DONE) == 0ull) b = 0ull;  // (every pixel of the wave stopped)
        {
            constexpr int h = 0;
            while (b) {
#if R3DG_FWD_SWALK
                // the pair from the live mask by s_ff1 + s_bitset0 (s_ff1 of an empty mask is -1, whose
                // s_bitset0 clears the already clear bit 63): 4 scalar ops for what b &= b - 1 twice,
                // two s_ff1 and their selects took 11
                int j0, j1;
                asm("s_ff1_i32_b64 %0, %2\n\ts_bitset0_b64 %2, %0\n\ts_ff1_i32_b64 %1, %2\n\ts_bitset0_b64 %2, %1"
                    : "=&s"(j0), "=&s"(j1), "+s"(b));
                const bool has1 = j1 >= 0;
                j1 = has1 ? j1 : j0;
#else
                const int j0 = h * 64 + (int)__builtin_ctzll(b);
                b &= b - 1;
                const bool has1 = b != 0ull;
                const int j1 = has1 ? h * 64 + (int)__builtin_ctzll(b) : j0;
                b &= b - 1;
#endif
                const int u0 = __builtin_amdgcn_readfirstlane(j0), u1 = __builtin_amdgcn_readfirstlane(j1);
                const float4 co0 = st[u0], co1 = st[u1];
                const float2 xy0 = *reinterpret_cast<const float2*>(st + NB + u0);
                const float2 xy1 = *reinterpret_cast<const float2*>(st + NB + u1);
                const float pw0 = gauss_power(co0, xy0.x - pfx, xy0.y - pfy);
                const float pw1 = gauss_power(co1, xy1.x - pfx, xy1.y - pfy);
                // two scalar exp chains, interleaved by the scheduler (the packed pair, r3dg_expf2,
                // needs an s_nop between its dependent v_pk_fma_f32: 0.3 % slower at M1)
                const f32x2 G = {blend_expf(pw0), blend_expf(pw1)};
                step(j0, true, co0.w, pw0, G.x);
                step(j1, has1, co1.w, pw1, G.y);
                if (l == 0) R3DG_EXP_ADD(2, has1 ? 2 : 1);
                // converged here: a uniform exit (testing every 2 or 4 iterations instead, which
                // drops ~10 scalar instructions per iteration, measured no faster in round 3)
                if (__ballot(!R3DG_DONE) == 0ull) break;
            }
        }
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        buf ^= 1;
    }
    // a block that stops early has no DMA in flight: every issued batch was waited for above
    if (base >= n && n > 0) {  // ran to the end: the last batch's bits are still in LDS (block-uniform)
        __syncthreads();
        const int b0 = (n - 1) / NB * NB;
        write_bits(b0, n - b0, buf ^ 1);
    }

    // the tile's backward work: the most visits any of its quadrants makes (the backward's batches are
    // barrier-synchronised, so its slowest quadrant paces the workgroup); the backward's launch order
    // sorts by it (xyz_normal_kernel's extra workgroup, tile_order_by_work)
    if (a.bwd_work && wave0 && l == 0) {
        const uint32_t work = (uint32_t)max(max(vq0, vq1), max(vq2, vq3));
        a.bwd_work[tile] = work;
        // the tile's rank in its work bucket (the order's bucket sort needs no atomics then)
        a.bwd_rank[tile] = atomicAdd(a.bwd_hist + work_bucket(work), 1u);
    }
    // the backward's atomic sums (RenderFwdArgs::zero_sums): this tile's share, after its blend
    if (!SHADER && a.zero_sums) {  // (training forwards only: never with splat shaders)
        const uint32_t z0 = (uint32_t)tile * a.zero_chunk, z1 = min(z0 + a.zero_chunk, a.zero_n4);
        for (uint32_t i = z0 + (uint32_t)t; i < z1; i += kBlock) a.zero_sums[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#undef R3DG_DONE
#if R3DG_FWD_TSIGN
    T = fabsf(T);
#endif
    if (inside) {
        const int pix = py * a.W + px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        const float b0 = a.bg[0], b1 = a.bg[1], b2 = a.bg[2];
        const float o0 = C[0] + T * b0, o1 = C[1] + T * b1, o2 = C[2] + T * b2;
        a.out_color[3 * pix + 0] = o0;
        a.out_color[3 * pix + 1] = o1;
        a.out_color[3 * pix + 2] = o2;
        if constexpr (SHADER) {
            a.out_shader_color[3 * pix + 0] = CS[0] + T * b0;
            a.out_shader_color[3 * pix + 1] = CS[1] + T * b1;
            a.out_shader_color[3 * pix + 2] = CS[2] + T * b2;
        } else {
            // default splat shader: shader colour == SH colour (splatShader.cu:67-71)
            a.out_shader_color[3 * pix + 0] = o0;
            a.out_shader_color[3 * pix + 1] = o1;
            a.out_shader_color[3 * pix + 2] = o2;
        }
        a.out_depth[pix] = Dp;
        a.out_opacity[pix] = Op;
        if (a.zero_stencil) a.zero_stencil[pix] = 0.f;
#pragma unroll
        for (int c = 0; c < SMAX; ++c)
            if (c < a.S) a.out_feature[a.flay.a[c] + pix * a.flay.m[c]] = F[c];
    }
}

template <int SMAX>
static hipError_t launch_fwd_s(const RenderFwdArgs& a, bool shader, hipStream_t stream) {
    const int grid = padded_tile_grid(a.num_tiles);
    if (shader)
        launch_kernel(render_fwd_glds_kernel<SMAX, true>, dim3(grid), dim3(kBlock), stream, a);
    else
        launch_kernel(render_fwd_glds_kernel<SMAX, false>, dim3(grid), dim3(kBlock), stream, a);
    return hipGetLastError();
}

hipError_t launch_render_forward(const RenderFwdArgs& a, bool shader, hipStream_t stream) {
    if (a.num_tiles == 0) return hipSuccess;
    if (a.S == 0) return launch_fwd_s<0>(a, shader, stream);
    if (a.S <= 4) return launch_fwd_s<4>(a, shader, stream);
    if (a.S <= 8) return launch_fwd_s<8>(a, shader, stream);
    if (a.S <= 11) return launch_fwd_s<11>(a, shader, stream);  // M1 / C3 (S = 11): no pad-channel FMA
    if (a.S <= 12) return launch_fwd_s<12>(a, shader, stream);
    if (a.S <= 16) return launch_fwd_s<16>(a, shader, stream);
    if (a.S <= 24) return launch_fwd_s<24>(a, shader, stream);
    return launch_fwd_s<32>(a, shader, stream);
}

// forward.cu:271-383 (RenderIntermediateTexturesCUDA) on the default blend's machinery: the
// render record's conic + opacity and position plus one packed float4 [depth, stencil,
// stencil opacity, 0] per Gaussian (IntermediateArgs::inter_rec, packed by the caller right before
// the launch: the splat shaders edit stencils) are copied HBM -> LDS by LDS-DMA one 64-instance batch
// ahead; each wave culls the staged instances for its 8x8 quadrant with the larger of the two
// opacities (an instance it skips fails both alpha tests on every pixel of the quadrant) and
// steps through the survivors two at a time (both exps packed). The arithmetic is the oracle's
// (oracle_render_intermediate: contraction off, plain products), the Stencil accumulator starts
// at 0 (the reference leaves it uninitialised, forward.cu:312). The register-staged 256-instance
// kernel it replaced evaluated every (instance, pixel) pair of the tile list: 0.97 ms per pass at
// M1.
__global__ void __launch_bounds__(kBlock) intermediate_glds_kernel(IntermediateArgs a) {
#pragma clang fp contract(off)
    constexpr int NB = 64, NCOL = 3, SBUF = NCOL * NB;
    __shared__ float4 s_lds[2 * SBUF];
    const int tile = block_tile(a.tile_order, a.num_tiles);
    if (tile >= a.num_tiles) return;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int px = tx * kTileX + (w & 1) * 8 + (l & 7);
    const int py = ty * kTileY + (w >> 1) * 8 + (l >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    const float qx0 = (float)(tx * kTileX + (w & 1) * 8), qy0 = (float)(ty * kTileY + (w >> 1) * 8);
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    bool done = !inside;
    float sT = 1.f, T = 1.f, St = 0.f, Dp = 0.f;

    const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)s_lds;
    auto gid_of = [&](int b0) { return a.point_list[range.x + (uint32_t)min(b0 + l, n - 1)]; };
    auto issue = [&](uint32_t gid, int buf) {
#pragma unroll
        for (int k = 0; k < NCOL; ++k) {
            if ((k & 3) != w) continue;  // wave-uniform
            const float4* src = k < 2 ? a.records + (size_t)gid * a.rec4 + k : a.inter_rec + gid;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)((buf * SBUF + k * NB) * 16));
            int keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
        }
    };
    uint32_t gnext = 0;
    if (n > 0) {
        issue(gid_of(0), 0);
        if (n > NB) gnext = gid_of(NB);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int buf = 0;
    for (int base = 0; base < n; base += NB) {
        if (__syncthreads_count(done) == kBlock) break;
        if (base + NB < n) {  // block-uniform: stage the next batch while this one blends
            issue(gnext, buf ^ 1);
            if (base + 2 * NB < n) gnext = gid_of(base + 2 * NB);
        }
        const float4* st = s_lds + buf * SBUF;
        const int cnt = min(NB, n - base);
        bool mine = false;
        if (l < cnt) {
            float4 co = st[l];
            const float4 r1 = st[NB + l];
            co.w = fmaxf(co.w, st[2 * NB + l].z);  // either alpha may pass
            mine = quadrant_live(make_float2(r1.x, r1.y), co, qx0, qy0, 1);
        }
        unsigned long long bits = __ballot(mine);
        // the tests predicated, only the accumulation a branch (as the blend's step)
        auto step = [&](int j, bool live, float power, float G) {
            const int ju = __builtin_amdgcn_readfirstlane(j);
            const float o = st[ju].w;
            const float4 ds = st[2 * NB + ju];  // depth, stencil, stencil opacity
            const float alpha = fminf(0.99f, o * G), salpha = fminf(0.99f, ds.z * G);
            const bool contrib = live && !done && !(power > 0.0f) &&
                                 !(alpha < 1.0f / 255.0f && salpha < 1.0f / 255.0f);
            const float tT = T * (1 - alpha), tS = sT * (1 - salpha);
            const bool stop = tT < 0.0001f && tS < 0.0001f;
            done = done || (contrib && stop);
            if (contrib && !stop) {
                Dp += ds.x * (alpha * T);
                T = tT;
                St += ds.y * (salpha * sT);
                sT = tS;
            }
        };
        while (bits && __ballot(!done) != 0ull) {
            const int j0 = (int)__builtin_ctzll(bits);
            bits &= bits - 1;
            const bool has1 = bits != 0ull;
            const int j1 = has1 ? (int)__builtin_ctzll(bits) : j0;
            bits &= bits - 1;
            const int u0 = __builtin_amdgcn_readfirstlane(j0), u1 = __builtin_amdgcn_readfirstlane(j1);
            const float4 co0 = st[u0], co1 = st[u1];
            const float2 xy0 = *reinterpret_cast<const float2*>(st + NB + u0);
            const float2 xy1 = *reinterpret_cast<const float2*>(st + NB + u1);
            const float pw0 = gauss_power(co0, xy0.x - pfx, xy0.y - pfy);
            const float pw1 = gauss_power(co1, xy1.x - pfx, xy1.y - pfy);
            const f32x2 G = {blend_expf(pw0), blend_expf(pw1)};  // scalar chains, as the default blend
            step(j0, true, pw0, G.x);
            step(j1, has1, pw1, G.y);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        buf ^= 1;
    }
    // a block that stops early has no DMA in flight: every issued batch was waited for above
    if (inside) {
        const int pix = py * a.W + px;
        a.out_depth[pix] = Dp;
        a.out_stencil[pix] = St;
    }
}

__global__ void __launch_bounds__(256) pack_inter_rec_kernel(int P, const int* __restrict__ radii,
                                                             const float* __restrict__ depths,
                                                             const float* __restrict__ stencils,
                                                             const float* __restrict__ stencil_opacity,
                                                             float4* __restrict__ inter_rec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || radii[i] <= 0) return;
    inter_rec[i] = make_float4(depths[i], stencils[i], stencil_opacity[i], 0.f);
}

hipError_t launch_intermediate(const IntermediateArgs& a, int P, const int* radii, hipStream_t st) {
    if (a.num_tiles == 0) return hipSuccess;
    if (P > 0)
        hipLaunchKernelGGL(pack_inter_rec_kernel, dim3((P + 255) / 256), dim3(256), 0, st, P, radii, a.depths,
                           a.stencils, a.stencil_opacity, a.inter_rec);
    hipLaunchKernelGGL(intermediate_glds_kernel, dim3(padded_tile_grid(a.num_tiles)), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

// forward.cu:564-658 (renderSurfaceXYZCUDA + renderPseudoNormalCUDA) fused: every thread
// recomputes its 3x3 neighbourhood's surface points from depth/opacity (same expression as
// the xyz it stores), so one pass produces both outputs.
__device__ __forceinline__ float3 surface_point(const XyzNormalArgs& a, int x, int y, float depth, float opacity) {
    const float d = depth / fmaxf(opacity, 0.0000001f);
    return make_float3(((float)x - a.cx) / a.focal_x * d, ((float)y - a.cy) / a.focal_y * d, d);
}

// One workgroup per 16 x (16 XYZ_R) pixels (XYZ_R tile rows: the halo and the launch's latency
// amortised over more pixels); thread t handles pixel column t & 15 of rows t >> 4, + 16, ...
#ifndef R3DG_XYZ_R
#define R3DG_XYZ_R 4
#endif
// The backward's launch order from the forward's per-tile work counts (RenderFwdArgs::bwd_work): a
// bucket sort by work / 4 (capped), descending, as the binning's instance-count order
// (preprocess.hip tile_order_block). The forward counted the buckets and gave every tile its rank in
// its bucket (global atomics, one per tile), so one 256-thread workgroup scans the 1024 bucket counts
// and places every tile at its bucket's start + rank, with no atomics. The padded grid's last slots
// name no tile (T).
// Workgroup `slice` of `nslices` places tiles [T slice / nslices, T (slice + 1) / nslices) (every one
// scans the bucket counts itself: 4 KB), so the placement's dependent loads spread over workgroups.
__device__ void tile_order_by_work(int T, const uint32_t* __restrict__ work, const uint32_t* __restrict__ rank,
                                   const uint32_t* __restrict__ hist, uint32_t* __restrict__ order, int slice,
                                   int nslices, uint32_t* lds) {
    constexpr int NT = 256, BPT = kWorkBuckets / NT;
    uint32_t* const cur = lds;                   // [kWorkBuckets] (the caller's LDS)
    uint32_t* const s_wave = lds + kWorkBuckets;  // [NT / 64]
    const int t = threadIdx.x, l = t & 63, wv = t >> 6;
    // exclusive scan in descending bucket order: thread t owns reversed buckets [BPT t, BPT t + BPT)
    uint32_t c[BPT], sum = 0;
#pragma unroll
    for (int k = 0; k < BPT; ++k) {
        c[k] = hist[kWorkBuckets - 1 - (BPT * t + k)];
        sum += c[k];
    }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    if (l == 63) s_wave[wv] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int k = 0; k < wv; ++k) run += s_wave[k];
#pragma unroll
    for (int k = 0; k < BPT; ++k) {
        cur[kWorkBuckets - 1 - (BPT * t + k)] = run;  // the bucket's first slot
        run += c[k];
    }
    __syncthreads();
    const int i0 = (int)((long long)T * slice / nslices), i1 = (int)((long long)T * (slice + 1) / nslices);
    for (int i = i0 + t; i < i1; i += NT) order[cur[work_bucket(work[i])] + rank[i]] = (uint32_t)i;
    if (slice == nslices - 1) {
        const int TP = padded_tile_grid(T);
        for (int i = T + t; i < TP; i += NT) order[i] = (uint32_t)T;
    }
}

// the backward's tile order on its own (forwards that compute no pseudo normal)
__global__ void __launch_bounds__(256) bwd_order_kernel(int T, const uint32_t* __restrict__ work,
                                                        const uint32_t* __restrict__ rank,
                                                        const uint32_t* __restrict__ hist, uint32_t* __restrict__ order) {
    __shared__ uint32_t lds[kWorkBuckets + 4];
    tile_order_by_work(T, work, rank, hist, order, blockIdx.x, gridDim.x, lds);
}

hipError_t launch_bwd_order(int T, const uint32_t* work, const uint32_t* rank, const uint32_t* hist, uint32_t* order,
                            hipStream_t st) {
    hipLaunchKernelGGL(bwd_order_kernel, dim3((T + 1023) / 1024), dim3(256), 0, st, T, work, rank, hist, order);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) xyz_normal_kernel(XyzNormalArgs a) {
    // the extra column of the grid: the backward's tile order, one slice of the tiles per workgroup
    // (off the critical path)
    // (a 1-D grid whose first kOrderSlices workgroups are dispatched first and finish long before
    // the kernel's last pixel blocks; as a last grid column they lengthened it by ~4 us)
    // the block's 18 x (16 R + 2) neighbourhood (edge-clamped) of surface points, each evaluated
    // once into LDS instead of nine times per pixel (the order workgroups use the same array)
    constexpr int R = R3DG_XYZ_R, HW_ = 18, HH = 16 * R + 2;
    static_assert(3 * HW_ * HH >= kWorkBuckets + 4, "the order's LDS fits the halo array");
    __shared__ float sp[3][HW_ * HH];
    const int nord = a.bwd_order ? kOrderSlices : 0;
    if ((int)blockIdx.x < nord) {
        tile_order_by_work(a.num_tiles, a.bwd_work, a.bwd_rank, a.bwd_hist, a.bwd_order, blockIdx.x, nord,
                           reinterpret_cast<uint32_t*>(&sp[0][0]));
        return;
    }
    const int pb = (int)blockIdx.x - nord, pbx = pb % a.blocks_x, pby = pb / a.blocks_x;
    const int bx = pbx * 16, by = pby * 16 * R;
    // every halo point's depth and opacity loaded first (all in flight at once), then evaluated
    constexpr int NIT = (HW_ * HH + 255) / 256;
    float dv[NIT], ov[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int k = (int)threadIdx.x + it * 256;
        dv[it] = 0.f;
        ov[it] = 0.f;
        if (k < HW_ * HH) {
            const int hx = min(max(bx + k % HW_ - 1, 0), a.W - 1), hy = min(max(by + k / HW_ - 1, 0), a.H - 1);
            dv[it] = a.depth[hy * a.W + hx];
            ov[it] = a.opacity[hy * a.W + hx];
        }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int k = (int)threadIdx.x + it * 256;
        if (k < HW_ * HH) {
            const int hx = min(max(bx + k % HW_ - 1, 0), a.W - 1), hy = min(max(by + k / HW_ - 1, 0), a.H - 1);
            const float3 q = surface_point(a, hx, hy, dv[it], ov[it]);
            sp[0][k] = q.x;
            sp[1][k] = q.y;
            sp[2][k] = q.z;
        }
    }
    __syncthreads();
    // the view rotation in registers, once: the xyz / normal stores may alias a.view, so the compiler
    // re-read it per row, each read waited for
    float v[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) v[i] = a.view[i];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
        const int lx = threadIdx.x & 15, ly = (threadIdx.x >> 4) + 16 * rr;
        const int x = bx + lx, y = by + ly;
        if (x >= a.W || y >= a.H) continue;
        const int pix = y * a.W + x;
        // neighbour (dx, dy) of this pixel; edge clamping already happened in the halo load, except
        // that a pixel on the image's last row / column inside the block must clamp to itself
        const int xm = lx, xc = lx + 1, xp = x == a.W - 1 ? lx + 1 : lx + 2;
        const int ym = ly, yc = ly + 1, yp = y == a.H - 1 ? ly + 1 : ly + 2;
        auto P3 = [&](int hx, int hy) {
            const int k = hy * HW_ + hx;
            return make_float3(sp[0][k], sp[1][k], sp[2][k]);
        };
        const float3 c = P3(xc, yc);
        a.xyz[3 * pix + 0] = c.x;
        a.xyz[3 * pix + 1] = c.y;
        a.xyz[3 * pix + 2] = c.z;
        const float3 p00 = P3(xm, ym), p01 = P3(xc, ym), p02 = P3(xp, ym);
        const float3 p10 = P3(xm, yc), p12 = P3(xp, yc);
        const float3 p20 = P3(xm, yp), p21 = P3(xc, yp), p22 = P3(xp, yp);
        float ga[3], gb[3];
        const float* f00 = &p00.x; const float* f01 = &p01.x; const float* f02 = &p02.x; const float* f10 = &p10.x;
        const float* f12 = &p12.x; const float* f20 = &p20.x; const float* f21 = &p21.x; const float* f22 = &p22.x;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            ga[i] = -0.125f * f00[i] + 0.125f * f02[i] - 0.25f * f10[i] + 0.25f * f12[i] - 0.125f * f20[i] +
                    0.125f * f22[i];
            gb[i] = -0.125f * f00[i] - 0.25f * f01[i] - 0.125f * f02[i] + 0.125f * f20[i] + 0.25f * f21[i] +
                    0.125f * f22[i];
        }
        float nx = ga[1] * gb[2] - ga[2] * gb[1];
        float ny = -ga[0] * gb[2] + ga[2] * gb[0];
        float nz = ga[0] * gb[1] - ga[1] * gb[0];
        const float norm = sqrtf(nx * nx + ny * ny + nz * nz);
        if (norm <= 0.0f) {
            a.normal[3 * pix + 0] = 0.f;
            a.normal[3 * pix + 1] = 0.f;
            a.normal[3 * pix + 2] = 0.f;
            continue;
        }
        nx = -nx / norm;
        ny = -ny / norm;
        nz = -nz / norm;
        a.normal[3 * pix + 0] = v[0] * nx + v[1] * ny + v[2] * nz;
        a.normal[3 * pix + 1] = v[4] * nx + v[5] * ny + v[6] * nz;
        a.normal[3 * pix + 2] = v[8] * nx + v[9] * ny + v[10] * nz;
    }
}

}  // namespace r3dg
