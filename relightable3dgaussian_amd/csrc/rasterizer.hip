// rasterizer.hip -- host orchestration of the rasterizer and the C ABI (include/r3dg_hip.h).
//
// Restates CudaRasterizer::Rasterizer::forward / backward / markVisible
// (reference rasterizer_impl.cu:143-639) on one HIP stream (the caller's), with:
//   * no input clones when the SH shaders are the defaults (the reference clones six inputs
//     every call, rasterize_points.cu:117-122, only so shaders may mutate them);
//   * no RenderIntermediateTextures pass and no splat-shader launch when the splat shaders are
//     the defaults (their only outputs are then a stencil of zeros and shader_rgb == rgb);
//   * rocprim inclusive scan, then binning by per-tile counters (counting and range passes
//     overlapped with the num_rendered readback) and a per-tile sort by (depth bits, Gaussian id)
//     instead of a radix sort of L 64-bit keys (preprocess.hip bin_count_kernel);
//   * one blocking D2H read of num_rendered, as the reference (rasterizer_impl.cu:347).
#include <cstring>  // before rocprim on ROCm 7.2
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "r3dg_common.h"
#include "r3dg_kernels.h"
#include "shaders.h"

namespace r3dg {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// ---- options (r3dg_get_options / r3dg_set_options) -------------------------------------------
// Read by the host code of each call as one snapshot. The environment is consulted once, when the
// library is loaded, and only for the supported runtime option R3DG_BWD_REDUCE.
static r3dg_options initial_options() {
    r3dg_options o{};
    o.struct_size = sizeof(r3dg_options);
    const char* e = getenv("R3DG_BWD_REDUCE");
    o.bwd_reduce = (e && e[0] == 'r') ? R3DG_REDUCE_ROWS : R3DG_REDUCE_ATOMIC;
#ifdef R3DG_EXP_BIN_ONE_PASS  // experiment builds (A/B of the binning scatter in bench.py)
    o.test_bin_one_pass = 1;
#endif
    return o;
}
static std::mutex g_opt_mu;
static r3dg_options g_options = initial_options();
r3dg_options options() {
    std::lock_guard<std::mutex> lk(g_opt_mu);
    return g_options;
}

static inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

FeatureLayout make_feature_layout(int S, long long HW, bool native) {
    FeatureLayout f{};
    int groups[kMaxFeatures];
    const int ng = r3dg_feature_groups(S, groups);
    int c = 0;
    for (int gi = 0; gi < ng; ++gi)
        for (int k = 0; k < groups[gi]; ++k, ++c) {
            if (c >= kMaxFeatures) break;
            if (native) {
                f.a[c] = (int)(HW * (c - k) + k);
                f.m[c] = groups[gi];
            } else {  // planar [S, H, W]
                f.a[c] = (int)(HW * c);
                f.m[c] = 1;
            }
        }
    return f;
}

// ---- state buffer layouts --------------------------------------------------------------------
// the single-pass scan's status words (scan_touched_kernel): one per workgroup + the ticket counter
int scan_blocks(size_t P);
static size_t scan_temp_size(size_t P) { return sizeof(uint64_t) * ((size_t)scan_blocks(P) + 1); }

// ---- the backward's atomic sums, prepared by the forward (RenderFwdArgs::zero_sums) -------------
// Row stride (floats) of the per-Gaussian sums of the atomic flush: [X part (f32) | 6 moments (f64) |
// pad], rows of 32 floats (128 B) so each 16-float X segment is one aligned 64-B atomic request and
// the moments are 8-B aligned (at least the X part and the 6 double moments: XW + 12 floats per row);
// test_bwd_srs (A/B) rounds up to 8 floats.
static int atomic_sums_min_stride(int S) { return 16 * bwd_xblocks(S) + 12; }
static int atomic_sums_stride(int S, const r3dg_options& opt) {
    const int srs_min = atomic_sums_min_stride(S);
    if (opt.test_bwd_srs > 0) return (std::max(srs_min, opt.test_bwd_srs) + 7) & ~7;
    return (std::max(part_row_stride(S), srs_min) + 31) & ~31;
}
// A training forward (atomic reduction, no shaders / post passes) appends the sums to its geometry
// state and has its blend zero them (the stores drain under the blend, which waits on latency, not
// on memory), so the backward launches no memset (M1: the 128 MB fill, 17 us per step). The host
// records which geometry states hold such still-zero sums; the first backward on one uses them,
// any other backward (a second one on the same state, other options) zeroes scratch as before.
struct PreparedSums {
    float* sums;
    int P, S, SRS;
    bool fresh;
};
static std::mutex g_sums_mu;
static std::map<uintptr_t, PreparedSums> g_sums;  // key: geometry state base
static void note_prepared_sums(void* geom, const PreparedSums* ps) {
    std::lock_guard<std::mutex> lk(g_sums_mu);
    g_sums.erase((uintptr_t)geom);  // a new forward's state at a reused address replaces the old entry
    if (!ps) return;
    if (g_sums.size() >= 4096) g_sums.clear();  // entries are hints: a missing one costs a memset
    g_sums[(uintptr_t)geom] = *ps;
}
static float* take_prepared_sums(void* geom, int P, int S, int SRS) {
    std::lock_guard<std::mutex> lk(g_sums_mu);
    auto it = g_sums.find((uintptr_t)geom);
    if (it == g_sums.end() || !it->second.fresh || it->second.P != P || it->second.S != S || it->second.SRS != SRS)
        return nullptr;
    it->second.fresh = false;
    return it->second.sums;
}

// the backward's launch order: longest tiles first; test_tile_order_spatial the XCD-aware spatial
// order (per-XCD-band orders measured and dropped)
static const uint32_t* bwd_tile_order(const ImageState& is, const r3dg_options& opt) {
    if (opt.test_tile_order_spatial) return nullptr;
#ifdef R3DG_EXP_BWD_COUNT_ORDER  // experiment builds: the binning's instance-count order
    return is.tile_order;
#else
    return is.bwd_order;  // most backward work first (the forward's visit counts)
#endif
}

// Carving works on an integer cursor so the same code computes sizes (base 0) and pointers.
template <typename T>
static T* carve(uintptr_t& p, size_t count) {
    T* r = reinterpret_cast<T*>(p);
    p += align256(sizeof(T) * count);
    return r;
}

static GeomState carve_geom(uintptr_t p, size_t P, int S, uintptr_t* end) {
    GeomState g{};
    g.depths = carve<float>(p, P);
    g.internal_radii = carve<int>(p, P);
    g.means2D = carve<float2>(p, P);
    g.cov3D = carve<float>(p, 6 * P);
    g.conic_opacity = carve<float4>(p, P);
    g.rgb = carve<float>(p, 3 * P);
    g.shader_rgb = carve<float>(p, 3 * P);
    g.stencils = carve<float>(p, P);
    g.stencil_opacity = carve<float>(p, P);
    g.clamped = carve<uint8_t>(p, P);
    g.tiles_touched = carve<uint32_t>(p, P);
    g.point_offsets = carve<uint32_t>(p, P);
    g.depth_keys = carve<uint32_t>(p, P);
    g.scan_temp_bytes = scan_temp_size(P);
    g.scan_temp = carve<char>(p, g.scan_temp_bytes);
    // render records last: every other offset is independent of S
    g.records = S >= 0 ? carve<float4>(p, P * (size_t)record_f4(S)) : nullptr;
    if (end) *end = p;
    return g;
}
size_t geom_state_bytes(size_t P, int S) {
    uintptr_t end = 0;
    carve_geom(0, P, S, &end);
    return (size_t)end;
}
GeomState geom_state_from(void* base, size_t P, int S) { return carve_geom((uintptr_t)base, P, S, nullptr); }

static BinningState carve_binning(uintptr_t p, size_t L, uintptr_t* end) {
    BinningState b{};
    b.point_list = carve<uint32_t>(p, L);
    b.pairs = carve<uint2>(p, L);
    // sort_k1 | sort_v1 as one block: the two-pass scatter stages its bucketed pairs there (uint2[L])
    // before the long-tile depth sort uses them
    b.sort_k1 = reinterpret_cast<uint32_t*>(carve<uint2>(p, L));
    b.sort_v1 = b.sort_k1 + L;
    b.sort_k2 = carve<uint32_t>(p, L);
    b.flags = carve<uint32_t>(p, L);
    b.contrib = carve<uint8_t>(p, L);
    if (end) *end = p;
    return b;
}
size_t binning_state_bytes(size_t L) {
    uintptr_t end = 0;
    carve_binning(0, L, &end);
    return (size_t)end + 256;
}
BinningState binning_state_from(void* base, size_t L) { return carve_binning((uintptr_t)base, L, nullptr); }

static int num_tiles_of(int H, int W) { return ((W + kTileX - 1) / kTileX) * ((H + kTileY - 1) / kTileY); }
// the binning's per-workgroup tile counts, then (8-B aligned) bin_colscan_kernel's look-back status
// words and ticket
static size_t bin_hist_words(size_t T) { return ((size_t)bin_blocks_max((int)T) * T + 1) & ~(size_t)1; }
static size_t bin_hist_count(size_t T) { return bin_hist_words(T) + 2 * ((T + 63) / 64 + 1); }
static uint64_t* bin_tile_scan(uint32_t* hist, size_t T) { return reinterpret_cast<uint64_t*>(hist + bin_hist_words(T)); }

static ImageState carve_image(uintptr_t p, int H, int W, uintptr_t* end, bool with_hist = true) {
    ImageState s{};
    const size_t N = (size_t)H * W;
    s.final_T = carve<float>(p, N);
    s.n_contrib = carve<uint32_t>(p, N);
    const size_t T = (size_t)num_tiles_of(H, W);
    s.ranges = carve<uint2>(p, T);
    s.tile_order = carve<uint32_t>(p, padded_tile_grid((int)T));
    s.tile_work = carve<uint32_t>(p, T);
    s.bwd_work = carve<uint32_t>(p, T);
    s.bwd_rank = carve<uint32_t>(p, T);
    s.bwd_hist = carve<uint32_t>(p, kWorkBuckets);
    s.bwd_order = carve<uint32_t>(p, padded_tile_grid((int)T));
    // the binning's per-workgroup tile counts: last, so the backward's view of the buffer does
    // not depend on whether they live here (r3dg_rasterize_gaussians) or in transient scratch
    // (r3dg_rasterize_gaussians_ex)
    if (with_hist) s.bin_hist = carve<uint32_t>(p, bin_hist_count(T));
    if (end) *end = p;
    return s;
}
size_t image_state_bytes(int H, int W, bool with_hist) {
    uintptr_t end = 0;
    carve_image(0, H, W, &end, with_hist);
    return (size_t)end;
}
// the backward and the accessors never read the tile counts
ImageState image_state_from(void* base, int H, int W) { return carve_image((uintptr_t)base, H, W, nullptr, false); }

// ---- profiling events (r3dg_profile_*) -----------------------------------------------------------
struct Profiler {
    int max_records = 0;
    std::vector<hipEvent_t> ev[R3DG_PROF_KINDS][2];
    int n[R3DG_PROF_KINDS] = {0};
};
static Profiler g_prof;
static std::mutex g_prof_mu;

static thread_local LaunchEvents t_pending;
LaunchEvents take_launch_events() {
    const LaunchEvents e = t_pending;
    t_pending = LaunchEvents{};
    return e;
}

// A profiled stage. Kernel stages (the default) pass the events to their launch (launch_kernel,
// r3dg_kernels.h): timestamps inside the dispatch packet, no marker packets between kernels.
// Marker stages (library calls such as the rocPRIM sorts) record the events around the calls;
// they are recorded only with the prof_sort_markers option, since marker packets add gaps to the
// stream.
struct ProfScope {
    int k;
    hipStream_t st;
    bool marker;
    int idx = -1;
    ProfScope(int kind, hipStream_t s, bool markers = false, bool sort_markers = false)
        : k(kind), st(s), marker(markers) {
        if (marker && !sort_markers) return;
        if (g_prof.max_records > 0 && g_prof.n[k] < g_prof.max_records) {
            idx = g_prof.n[k]++;
            if (marker) (void)hipEventRecord(g_prof.ev[k][0][idx], st);
            else t_pending = LaunchEvents{g_prof.ev[k][0][idx], g_prof.ev[k][1][idx]};
        }
    }
    ~ProfScope() {
        if (idx < 0) return;
        if (marker) {
            (void)hipEventRecord(g_prof.ev[k][1][idx], st);
        } else if (t_pending.start) {  // no launch took the events (empty stage): zero duration
            (void)hipEventRecord(t_pending.start, st);
            (void)hipEventRecord(t_pending.stop, st);
            t_pending = LaunchEvents{};
        }
    }
};

// Pinned host words for the num_rendered readback, one per (host thread, device): a
// thread's calls on one device are issued in order, so the slot is free again by its next call.
struct Readback {
    uint32_t* host = nullptr;      // pinned, coherent host words (num_rendered, the error flag)
    uint32_t* host_dev = nullptr;  // the same words as the device addresses them
    uint32_t* dev_flag = nullptr;  // preprocess error flag (prefiltered runs only)
};
static hipError_t readback_slot(Readback** out) {
    constexpr int kMaxDevices = 64;
    thread_local Readback slots[kMaxDevices];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    Readback& r = slots[dev];
    if (!r.host) {
        void* p = nullptr;
        if ((e = hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess) return e;
        void* d = nullptr;
        if ((e = hipHostGetDevicePointer(&d, p, 0)) != hipSuccess) {
            (void)hipHostFree(p);
            return e;
        }
        r.host = static_cast<uint32_t*>(p);
        r.host_dev = static_cast<uint32_t*>(d);
    }
    *out = &r;
    return hipSuccess;
}

// Inclusive scan of tiles_touched -> point_offsets (rasterizer_impl.cu:255-257 cub::InclusiveSum) in
// one pass, and num_rendered published by the last workgroup: replaces rocPRIM's scan (an init
// kernel + the scan kernel) and a one-thread publish kernel -- three launches, 18 us at M1 (round 6),
// for 8 MB of traffic. The count goes straight into the pinned host words (a D2H copy cost a blit
// kernel plus the copy engine's hand-back: 4.5 us + a 5.6 us gap before the next kernel). Workgroup b scans its kScanItems contiguous items in registers / LDS and
// publishes its aggregate, then its inclusive prefix, in status[b] (decoupled look-back: flag in
// the top bits of one 64-bit word with the value, so one atomic load reads both). status[] is zeroed
// by preprocess_kernel, which runs before on the same stream. The grid (<= P / 16384 workgroups, 62
// at M1) is co-resident, so the look-back spins only while a predecessor is still summing.
constexpr int kScanThreads = 1024, kScanIPT = 16, kScanItems = kScanThreads * kScanIPT;
constexpr uint64_t kScanAggregate = 1ull << 62, kScanInclusive = 2ull << 62;
int scan_blocks(size_t P) { return (int)std::max<size_t>(1, (P + kScanItems - 1) / kScanItems); }
__global__ void __launch_bounds__(kScanThreads) scan_touched_kernel(const uint32_t* __restrict__ in,
                                                                    uint32_t* __restrict__ out, int P,
                                                                    uint64_t* status,
                                                                    const uint32_t* __restrict__ flag,
                                                                    uint32_t* host) {
    __shared__ uint32_t s_wave[kScanThreads / 64];
    __shared__ uint32_t s_prefix;
    __shared__ int s_b;
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    // the logical workgroup id from a ticket (status[gridDim.x], zeroed with the status words): a
    // workgroup only ever waits for tickets drawn before its own, i.e. for running workgroups
    if (t == 0) s_b = (int)__hip_atomic_fetch_add(status + gridDim.x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int b = s_b;
    const int i0 = b * kScanItems + t * kScanIPT;
    uint32_t v[kScanIPT];
    if (i0 + kScanIPT <= P) {
        const uint4* src = reinterpret_cast<const uint4*>(in + i0);  // in: 256-B aligned, i0 % 16 == 0
#pragma unroll
        for (int k = 0; k < kScanIPT / 4; ++k) {
            const uint4 q = src[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanIPT; ++k) v[k] = i0 + k < P ? in[i0 + k] : 0u;
    }
#pragma unroll
    for (int k = 1; k < kScanIPT; ++k) v[k] += v[k - 1];
    // exclusive scan of the thread totals across the workgroup
    uint32_t x = v[kScanIPT - 1];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    if (l == 63) s_wave[w] = x;
    __syncthreads();
    uint32_t wpre = 0, agg = 0;
#pragma unroll
    for (int k = 0; k < kScanThreads / 64; ++k) {
        const uint32_t s = s_wave[k];
        wpre += k < w ? s : 0u;
        agg += s;
    }
    const uint32_t texcl = wpre + x - v[kScanIPT - 1];
    if (w == 0) {
        if (b > 0 && l == 0)
            __hip_atomic_store(status + b, kScanAggregate | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t prefix = lookback_prefix(status, b);
        if (l == 0) {
            __hip_atomic_store(status + b, kScanInclusive | (prefix + agg), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            s_prefix = prefix;
            if (b == (int)gridDim.x - 1) {  // the total: num_rendered into the pinned host words
                if (flag) host[1] = *flag;
                __threadfence_system();  // the flag before the count the host polls for
                host[0] = prefix + agg;
                __threadfence_system();
            }
        }
    }
    __syncthreads();
    const uint32_t base = s_prefix + texcl;
    if (i0 + kScanIPT <= P) {
        uint4* dst = reinterpret_cast<uint4*>(out + i0);
#pragma unroll
        for (int k = 0; k < kScanIPT / 4; ++k)
            dst[k] = make_uint4(base + v[4 * k], base + v[4 * k + 1], base + v[4 * k + 2], base + v[4 * k + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kScanIPT; ++k)
            if (i0 + k < P) out[i0 + k] = base + v[k];
    }
}

// The host waits for scan_touched_kernel's word itself instead of an event behind the kernel: an
// event record between two kernels of the stream cost a 5.5 us dispatch gap at M1 (round 6). The
// word starts at kUnpublished (num_rendered < 2^31 never is); the stream is queried every few
// thousand spins so a failed launch or a fault surfaces as its error instead of a hang.
constexpr uint32_t kUnpublished = 0xffffffffu;
static hipError_t wait_published(const Readback* rb, hipStream_t st) {
    volatile uint32_t* w = rb->host;
    for (uint64_t spin = 1;; ++spin) {
        if (w[0] != kUnpublished) return hipSuccess;
        if ((spin & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return w[0] != kUnpublished ? hipSuccess : hipErrorUnknown;  // drained, no word
            if (q != hipErrorNotReady) return q;
        }
    }
}

// InitializeStencil (rasterizer_impl.cu:203-209)
__global__ void __launch_bounds__(256) init_stencil_kernel(int P, float* stencil, float* stencil_opacity) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    stencil[i] = 0.0f;
    stencil_opacity[i] = 1.0f;
}

// Splat shaders edit conic_opacity.w after the render records were written: refresh the records'
// opacity (the backward reads records; the reference's backward reads the edited geometry state).
__global__ void __launch_bounds__(256) refresh_record_opacity_kernel(int P, const int* __restrict__ radii,
                                                                     const float4* __restrict__ conic_opacity,
                                                                     float4* __restrict__ records, int rec4) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || radii[i] <= 0) return;
    records[(size_t)i * rec4].w = conic_opacity[i].w;
}

// The shader record of every visible Gaussian (render_fwd_glds_kernel<SMAX, true>): na4 float4 in
// the attribute row's layout, [shader colour, 0 | the splat shaders' features, zero padded] -- the
// blend's staged colour and feature columns after the splat shaders ran. One thread per float4, so
// the stores are coalesced (a thread per Gaussian wrote a 112-byte row each: 0.37 ms at 1 M, S = 21).
__global__ void __launch_bounds__(256) shader_record_kernel(int P, int na4, const int* __restrict__ radii,
                                                            const float* __restrict__ shader_rgb,
                                                            const float* __restrict__ feats, int S,
                                                            float4* __restrict__ shader_rec) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)P * na4) return;
    const int i = (int)(e / na4), q = (int)(e - (long long)i * na4);
    if (radii[i] <= 0) return;
    float v[4];
    if (q == 0) {
        v[0] = shader_rgb[3 * i]; v[1] = shader_rgb[3 * i + 1]; v[2] = shader_rgb[3 * i + 2]; v[3] = 0.f;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = 4 * (q - 1) + k;
            v[k] = c < S ? feats[(size_t)i * S + c] : 0.f;
        }
    }
    shader_rec[e] = make_float4(v[0], v[1], v[2], v[3]);
}

// ---- shader registry (ShShader.cu:196-230, splatShader.cu:283-333, postProcessShader.cu:395-436) ----
// Handles are opaque ids: (kind + 1) << 32 | index into the alphabetically ordered name list
// (the reference's ShaderManager iterates a std::map, i.e. in name order).
static const std::vector<std::string>& shader_names(int kind) {
    static const std::vector<std::string> sh = {"CullHalf", "ExpPos", "GaussDissolve", "Heartbeat", "ShDefault"};
    static const std::vector<std::string> splat = {"Crack",         "CrackNoRecon",  "Dissolve",     "NaiveOutline",
                                                   "QuantizeFlats", "QuantizeLight", "RoughnessOnly", "SplatDefault",
                                                   "Stencil",       "Wireframe"};
    static const std::vector<std::string> post = {"BlurLighting", "CrackReconstriction", "Invert",
                                                  "Outline",      "QuantizeLighting",    "SobelFilter",
                                                  "SplatDefault", "TexturedShadows",     "ToonShader"};
    static const std::vector<std::string> none;
    return kind == R3DG_SHADER_SH ? sh : kind == R3DG_SHADER_SPLAT ? splat : kind == R3DG_SHADER_POST ? post : none;
}
static int64_t make_handle(int kind, int idx) { return ((int64_t)(kind + 1) << 32) | (int64_t)idx; }
static int handle_kind(int64_t h) { return (int)(h >> 32) - 1; }
static int handle_index(int64_t h) { return (int)(h & 0xffffffff); }
static int default_index(int kind) {
    const auto& n = shader_names(kind);
    const char* d = kind == R3DG_SHADER_SH ? "ShDefault" : "SplatDefault";
    return (int)(std::find(n.begin(), n.end(), d) - n.begin());
}

struct ShaderManagerObj {
    int kind;
    std::vector<int> counts;       // per shader (name order)
    std::vector<int*> d_lists;     // device splat-index list per shader
    bool all_default;
};
static std::mutex g_mgr_mu;
static std::map<int64_t, ShaderManagerObj*> g_managers;
static int64_t g_next_mgr = 1;

static ShaderManagerObj* lookup_manager(int64_t h) {
    if (h == 0) return nullptr;
    std::lock_guard<std::mutex> lk(g_mgr_mu);
    auto it = g_managers.find(h);
    return it == g_managers.end() ? nullptr : it->second;
}

static int build_manager(int kind, int P, const std::vector<int>& idx_per_splat, int64_t* out, hipStream_t st) {
    const int n = (int)shader_names(kind).size();
    auto* m = new ShaderManagerObj();
    m->kind = kind;
    m->counts.assign(n, 0);
    std::vector<std::vector<int>> lists(n);
    for (int i = 0; i < P; ++i) {
        const int s = idx_per_splat[i];
        if (s < 0 || s >= n) {
            delete m;
            set_error("shader manager: invalid shader index");
            return R3DG_ERR_ARG;
        }
        lists[s].push_back(i);  // ascending splat order, as SortShadersCUDA (preprocessModel.cu:116-134)
    }
    m->all_default = true;
    for (int s = 0; s < n; ++s) {
        m->counts[s] = (int)lists[s].size();
        int* d = nullptr;
        if (!lists[s].empty()) {
            R3DG_CHECK_HIP(hipMalloc(&d, sizeof(int) * lists[s].size()));
            R3DG_CHECK_HIP(hipMemcpyAsync(d, lists[s].data(), sizeof(int) * lists[s].size(), hipMemcpyHostToDevice, st));
            if (s != default_index(kind)) m->all_default = false;
        }
        m->d_lists.push_back(d);
    }
    R3DG_CHECK_HIP(hipStreamSynchronize(st));
    std::lock_guard<std::mutex> lk(g_mgr_mu);
    const int64_t h = (int64_t)0x5233000000000000ll | g_next_mgr++;
    g_managers[h] = m;
    *out = h;
    return R3DG_OK;
}

// preprocessModel.cu:17-59 (SelectShadersCUDA): shader choice by splat position.
__global__ void select_shaders_kernel(int P, const float* __restrict__ xyz, int8_t* sh_idx, int8_t* splat_idx,
                                      int i_sh_default, int i_heartbeat, int i_gauss_dissolve, int i_splat_default,
                                      int i_wireframe, int i_outline, int i_dissolve) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1];
    sh_idx[i] = (int8_t)(y < -0.3f ? i_sh_default : (y > 0.4f ? i_heartbeat : i_gauss_dissolve));
    int s;
    if (x < -0.6f) s = i_splat_default;
    else if (x > -0.6f && x < 0) s = i_wireframe;
    else if (x > 0 && x < 0.5) s = i_outline;
    else s = i_dissolve;
    splat_idx[i] = (int8_t)s;
}

static int name_index(int kind, const char* name) {
    const auto& n = shader_names(kind);
    auto it = std::find(n.begin(), n.end(), std::string(name));
    return it == n.end() ? -1 : (int)(it - n.begin());
}

}  // namespace r3dg

using namespace r3dg;

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" int r3dg_abi_version(void) { return R3DG_ABI_VERSION; }
extern "C" const char* r3dg_last_error(void) { return g_last_error.c_str(); }

extern "C" int r3dg_get_options(r3dg_options* o) {
    R3DG_REQUIRE(o && o->struct_size == sizeof(r3dg_options), "get_options: struct_size must be sizeof(r3dg_options)");
    *o = options();
    return R3DG_OK;
}

extern "C" int r3dg_set_options(const r3dg_options* o) {
    R3DG_REQUIRE(o && o->struct_size == sizeof(r3dg_options), "set_options: struct_size must be sizeof(r3dg_options)");
    R3DG_REQUIRE(o->bwd_reduce == R3DG_REDUCE_ATOMIC || o->bwd_reduce == R3DG_REDUCE_ROWS,
                 "set_options: bwd_reduce must be R3DG_REDUCE_ATOMIC or R3DG_REDUCE_ROWS");
    R3DG_REQUIRE(o->test_bwd_wterms == 0 || o->test_bwd_wterms == 1 || o->test_bwd_wterms == 3,
                 "set_options: test_bwd_wterms must be 0, 1 or 3");
    R3DG_REQUIRE(o->test_bin_blocks >= 0 && o->test_bwd_srs >= 0 && o->test_bwd_srs <= 4096 &&
                     o->test_bvh_lanes >= 0 && o->test_bvh_lanes <= 64 && o->test_bvh_sort >= 0 &&
                     o->test_bvh_sort <= 2,
                 "set_options: option out of range");
    std::lock_guard<std::mutex> lk(g_opt_mu);
    g_options = *o;
    return R3DG_OK;
}

extern "C" int r3dg_feature_groups(int S, int* groups) {
    int n = 0;
    if (S == 21) {
        const int g[9] = {1, 1, 1, 3, 3, 3, 3, 3, 3};
        for (n = 0; n < 9; ++n) groups[n] = g[n];
    } else if (S == 11) {
        const int g[5] = {1, 1, 3, 3, 3};
        for (n = 0; n < 5; ++n) groups[n] = g[n];
    } else {
        for (n = 0; n < S; ++n) groups[n] = 1;
    }
    return n;
}

extern "C" size_t r3dg_image_state_n_contrib_offset(int H, int W) { return align256(4 * (size_t)H * W); }
extern "C" size_t r3dg_geom_state_bytes(int P, int S) { return geom_state_bytes(P > 0 ? (size_t)P : 0, S); }

extern "C" int r3dg_rasterize_gaussians(const r3dg_raster_settings* s, const r3dg_gaussians* g,
                                        const r3dg_forward_outputs* out, r3dg_alloc_fn geom_alloc, void* geom_ctx,
                                        r3dg_alloc_fn binning_alloc, void* binning_ctx, r3dg_alloc_fn image_alloc,
                                        void* image_ctx, int* num_rendered, r3dg_stream_t stream) {
    return r3dg_rasterize_gaussians_ex(s, g, out, geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc,
                                       image_ctx, nullptr, nullptr, num_rendered, stream);
}

extern "C" int r3dg_rasterize_gaussians_ex(const r3dg_raster_settings* s, const r3dg_gaussians* g,
                                           const r3dg_forward_outputs* out, r3dg_alloc_fn geom_alloc, void* geom_ctx,
                                           r3dg_alloc_fn binning_alloc, void* binning_ctx, r3dg_alloc_fn image_alloc,
                                           void* image_ctx, r3dg_alloc_fn scratch_alloc, void* scratch_ctx,
                                           int* num_rendered, r3dg_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    R3DG_REQUIRE(s && g && out && num_rendered, "rasterize_gaussians: null argument");
    R3DG_REQUIRE(s->struct_size == sizeof(r3dg_raster_settings),
                 "rasterize_gaussians: settings->struct_size must be sizeof(r3dg_raster_settings) (ABI 2)");
    const r3dg_options opt = options();
    const int P = s->P, S = s->S, H = s->H, W = s->W;
    R3DG_REQUIRE(P >= 0 && H > 0 && W > 0, "rasterize_gaussians: invalid sizes");
    R3DG_REQUIRE(S >= 0 && S <= kMaxFeatures, "rasterize_gaussians: at most 32 feature channels are supported");
    R3DG_REQUIRE((g->colors_precomp != nullptr) != (g->sh != nullptr) || P == 0,
                 "Please provide excatly one of either SHs or precomputed colors!");
    R3DG_REQUIRE(((g->scales && g->rotations) != (g->cov3D_precomp != nullptr)) || P == 0,
                 "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    R3DG_REQUIRE(S == 0 || P == 0 || g->features, "rasterize_gaussians: features missing");
    R3DG_REQUIRE(!g->sh || P == 0 || (s->D >= 0 && s->D <= 3 && (s->D + 1) * (s->D + 1) <= s->M && s->M <= 16),
                 "rasterize_gaussians: SH degree must be 0..3 with (degree+1)^2 <= M <= 16 coefficients");
    R3DG_REQUIRE((long long)H * W * (S > 3 ? S : 3) < (1ll << 31), "rasterize_gaussians: image too large");
    *num_rendered = 0;

    // shaders (forward.cu:805-971): SH shaders shade working copies of the inputs before
    // preprocessing, splat shaders run after the intermediate depth/stencil pass
    ShaderManagerObj* shm = lookup_manager(s->sh_shader_manager);
    ShaderManagerObj* spm = lookup_manager(s->splat_shader_manager);
    R3DG_REQUIRE(s->sh_shader_manager == 0 || shm, "rasterize_gaussians: unknown SH shader manager handle");
    R3DG_REQUIRE(s->splat_shader_manager == 0 || spm, "rasterize_gaussians: unknown splat shader manager handle");
    R3DG_REQUIRE(!shm || shm->kind == R3DG_SHADER_SH, "rasterize_gaussians: h_shShaderManager is not an SH manager");
    R3DG_REQUIRE(!spm || spm->kind == R3DG_SHADER_SPLAT,
                 "rasterize_gaussians: h_splatShaderManager is not a splat manager");
    R3DG_REQUIRE(s->n_post_passes >= 0 && (s->n_post_passes == 0 || s->post_passes),
                 "rasterize_gaussians: invalid post-process pass list");
    const bool sh_active = P > 0 && shm && !shm->all_default;
    const bool splat_active = P > 0 && spm && !spm->all_default;
    const std::map<std::string, TexDesc>* tex_names = nullptr;
    TexDesc tex_error{};
    if (s->texture_manager)
        R3DG_REQUIRE(lookup_texture_manager(s->texture_manager, &tex_names, &tex_error),
                     "rasterize_gaussians: unknown texture manager handle");
    // TextureManager::GetTexture (texture.cu:298-314): the error texture for a missing name
    auto resolve = [&](const char* name, TexDesc* d) {
        if (!name) return true;
        if (!tex_names) return false;
        auto it = tex_names->find(name);
        *d = it == tex_names->end() ? tex_error : it->second;
        return true;
    };
    auto check_shader = [&](int kind, int id) -> bool {
        const bool feats = kind == R3DG_SHADER_SH ? sh_shader_needs_features(id) : splat_shader_needs_features(id);
        if (feats && S < 21) {
            set_error("rasterize_gaussians: shader " + shader_names(kind)[id] +
                      " addresses the reference's 21-channel feature layout (ShShader.h/splatShader.h); S < 21");
            return false;
        }
        TexDesc d{};
        const char* t0 = kind == R3DG_SHADER_SH ? sh_shader_texture(id, 0) : splat_shader_texture(id);
        const char* t1 = kind == R3DG_SHADER_SH ? sh_shader_texture(id, 1) : nullptr;
        if (!resolve(t0, &d) || !resolve(t1, &d)) {
            set_error("rasterize_gaussians: shader " + shader_names(kind)[id] + " samples textures; pass a "
                      "texture manager (UploadTexturesToDevice)");
            return false;
        }
        return true;
    };
    if (sh_active) {
        R3DG_REQUIRE(g->scales && g->rotations && g->sh,
                     "rasterize_gaussians: SH shaders need scales, rotations and SH coefficients");
        for (int id = 0; id < (int)shm->counts.size(); ++id)
            if (shm->counts[id] > 0 && id != kShDefault && !check_shader(R3DG_SHADER_SH, id)) return R3DG_ERR_ARG;
    }
    if (splat_active)
        for (int id = 0; id < (int)spm->counts.size(); ++id)
            if (spm->counts[id] > 0 && !check_shader(R3DG_SHADER_SPLAT, id)) return R3DG_ERR_ARG;
    const bool work_copies = sh_active || splat_active;
    // post-process passes (rasterizer_impl.cu:485-529): registry ids in list order
    std::vector<int> post_ids;
    bool post_blur = false;
    TexDesc shadow_tex{};
    for (int i = 0; i < s->n_post_passes; ++i) {
        const int64_t h = s->post_passes[i];
        const int id = handle_index(h);
        R3DG_REQUIRE(handle_kind(h) == R3DG_SHADER_POST && id >= 0 && id < (int)shader_names(R3DG_SHADER_POST).size(),
                     "rasterize_gaussians: unknown post-process pass handle (GetPostProcessShaderAddressMap)");
        const std::string& name = shader_names(R3DG_SHADER_POST)[id];
        if (post_pass_needs_features(id) && S != 21) {
            set_error("rasterize_gaussians: post-process pass " + name +
                      " reads the reference's 21-channel feature image (postProcessShader.cu:17-28); S != 21");
            return R3DG_ERR_ARG;
        }
        if (post_pass_needs_shadow(id) && !resolve("shadow", &shadow_tex)) {
            set_error("rasterize_gaussians: post-process pass " + name +
                      " samples the \"shadow\" texture; pass a texture manager (UploadTexturesToDevice)");
            return R3DG_ERR_ARG;
        }
        post_blur = post_blur || id == kPpBlurLighting;
        post_ids.push_back(id);
    }
    R3DG_REQUIRE(post_ids.empty() || (out->color && out->opacity && out->depth && out->stencil && out->shader_color &&
                                      out->normal && out->surface_xyz && (S == 0 || out->feature)),
                 "rasterize_gaussians: post-process passes need every image output");

    const int gx = (W + kTileX - 1) / kTileX, gy = (H + kTileY - 1) / kTileY;
    const int T = gx * gy;
    // working copies of the six inputs the shaders may edit (rasterize_points.cu:117-122), after
    // the geometry state proper (the backward never reads them)
    const size_t geom_bytes = geom_state_bytes((size_t)P, S);
    const size_t M3 = (size_t)3 * (g->sh ? s->M : 0);
    // Only the inputs an active shader writes get a working copy (the others are read in place;
    // shaders.hip): positions (SH ExpPos / Heartbeat / GaussDissolve), scales (ExpPos / Heartbeat /
    // CullHalf), opacity (CullHalf / GaussDissolve), the SH block (GaussDissolve: sh0), features
    // (splat CrackNoRecon / RoughnessOnly / QuantizeLight); rotations never. The reference copies all
    // six (rasterize_points.cu:117-122): results are the same, the copies were 0.11 ms per frame at
    // M1 with S = 21.
    auto sh_on = [&](int id) { return sh_active && id < (int)shm->counts.size() && shm->counts[id] > 0; };
    auto sp_on = [&](int id) { return splat_active && id < (int)spm->counts.size() && spm->counts[id] > 0; };
    const bool w_pos = sh_on(kShExpPos) || sh_on(kShHeartbeat) || sh_on(kShGaussDissolve);
    const bool w_scale = sh_on(kShExpPos) || sh_on(kShHeartbeat) || sh_on(kShCullHalf);
    const bool w_opac = sh_on(kShCullHalf) || sh_on(kShGaussDissolve);
    const bool w_sh = sh_on(kShGaussDissolve);
    const bool w_feat = sp_on(kSpCrackNoRecon) || sp_on(kSpRoughnessOnly) || sp_on(kSpQuantizeLight);
    const size_t work_floats = work_copies ? (size_t)P * ((w_pos ? 3 : 0) + (w_scale ? 3 : 0) + (w_opac ? 1 : 0) +
                                                         (w_sh ? M3 : 0) + (w_feat ? S : 0))
                                           : 0;
    // the splat shaders that read the intermediate depth image (Crack, CrackNoRecon: the depth at the
    // mean pixel); without them the pre-shader intermediate pass only yields a stencil of zeros (every
    // stencil opacity is still InitializeStencil's 0 there, so every stencil alpha is 0) and the
    // blend overwrites its depth, so it is replaced by a memset
    const bool inter_pre = sp_on(kSpCrack) || sp_on(kSpCrackNoRecon);
    const size_t post_floats = post_blur ? (size_t)3 * H * W : 0;  // BlurLighting's incident-light snapshot
    // the splat shaders' colour as one float4 per Gaussian (16-B aligned, after the other extras)
    const size_t shrec_off = (work_floats + post_floats + 3) & ~(size_t)3;
    const size_t shrec_floats = splat_active ? 4 * (size_t)P * (record_f4(S) - 2) : 0;
    // the intermediate depth / stencil pass's packed per-Gaussian record (launch_intermediate)
    const size_t inter_floats = (splat_active || !post_ids.empty()) ? 4 * (size_t)P : 0;
    // With a scratch allocator (one call, stream-ordered memory freed when the call returns) the
    // forward-only transients live there instead of in the state autograd keeps until the
    // backward: the binning's per-workgroup tile counts (needed until the scatter) and the splat
    // shaders' / intermediate pass's per-Gaussian records (112 MB at 1M Gaussians with S = 21).
    const bool use_scratch = scratch_alloc != nullptr && P > 0;
    const size_t rec_bytes = sizeof(float) * (shrec_floats + inter_floats);
    // a training forward prepares the backward's zeroed atomic sums at the end of its geometry state
    const bool prep_sums = P > 0 && opt.bwd_reduce == R3DG_REDUCE_ATOMIC && !opt.test_bwd_dpp && !work_copies &&
                           post_ids.empty() && !splat_active;
    const int sums_srs = atomic_sums_stride(S, opt);
    const size_t extra_bytes = align256(sizeof(float) * shrec_off + (use_scratch ? 0 : rec_bytes));
    const size_t sums_bytes = prep_sums ? sizeof(float) * (size_t)sums_srs * (size_t)P : 0;
    void* geom_base = geom_alloc(geom_ctx, geom_bytes + extra_bytes + sums_bytes);
    void* img_base = image_alloc(image_ctx, image_state_bytes(H, W, !use_scratch));
    const size_t hist_bytes = (4 * bin_hist_count((size_t)T) + 255) & ~(size_t)255;
    char* scratch_base = use_scratch ? (char*)scratch_alloc(scratch_ctx, hist_bytes + rec_bytes) : nullptr;
    if (!geom_base || !img_base || (use_scratch && !scratch_base)) {
        set_error("rasterize_gaussians: state allocation failed");
        return R3DG_ERR_ALLOC;
    }
    uint32_t* hist_base = use_scratch ? reinterpret_cast<uint32_t*>(scratch_base) : nullptr;
    char* rec_base = use_scratch ? scratch_base + hist_bytes
                                 : static_cast<char*>(geom_base) + geom_bytes + sizeof(float) * shrec_off;
    GeomState geom = geom_state_from(geom_base, (size_t)P, S);
    float* prepared_sums = prep_sums ? reinterpret_cast<float*>(static_cast<char*>(geom_base) + geom_bytes + extra_bytes)
                                     : nullptr;
    float4* shader_rec = splat_active ? reinterpret_cast<float4*>(rec_base) : nullptr;
    float4* inter_rec = inter_floats ? reinterpret_cast<float4*>(rec_base + sizeof(float) * shrec_floats) : nullptr;
    const bool hist_scratch = use_scratch;
    ImageState img = carve_image((uintptr_t)img_base, H, W, nullptr, !hist_scratch);
    if (hist_scratch) img.bin_hist = hist_base;
    int* radii = out->radii ? out->radii : geom.internal_radii;
    const float focal_y = H / (2.0f * s->tan_fovy);
    const float focal_x = W / (2.0f * s->tan_fovx);

    const float* means3D = g->means3D;
    const float* scales = g->scales;
    const float* rotations = g->rotations;
    const float* opacity = g->opacity;
    const float* shs = g->sh;
    float* feats = const_cast<float*>(g->features);
    if (work_copies) {
        float* w = reinterpret_cast<float*>(static_cast<char*>(geom_base) + geom_bytes);
        hipError_t ce = hipSuccess;
        auto copy = [&](const float* src, size_t n, bool written) -> float* {
            if (!written) return const_cast<float*>(src);  // read in place: no active shader writes it
            float* d = w;
            w += n;
            if (src && n && ce == hipSuccess) ce = hipMemcpyAsync(d, src, sizeof(float) * n, hipMemcpyDeviceToDevice, st);
            return src ? d : nullptr;
        };
        means3D = copy(g->means3D, 3 * (size_t)P, w_pos);
        scales = copy(g->scales, 3 * (size_t)P, w_scale);
        opacity = copy(g->opacity, (size_t)P, w_opac);
        shs = copy(g->sh, M3 * P, w_sh);
        feats = copy(g->features, (size_t)S * P, w_feat);
        R3DG_CHECK_HIP(ce);
    }
    // InitializeStencil (rasterizer_impl.cu:203-209): only the shaders and the intermediate
    // depth / stencil pass read the per-Gaussian stencils; the all-default path skips the launch
    if (P > 0 && (sh_active || splat_active || !post_ids.empty())) {
        hipLaunchKernelGGL(init_stencil_kernel, dim3((P + 255) / 256), dim3(256), 0, st, P, geom.stencils,
                           geom.stencil_opacity);
        R3DG_CHECK_LAUNCH(s->debug, st);
    }
    if (sh_active) {  // RunSHShaders (forward.cu:805-877): one launch per non-empty bucket
        for (int id = 0; id < (int)shm->counts.size(); ++id) {
            if (shm->counts[id] == 0 || id == kShDefault) continue;
            ShShaderArgs sa{};
            sa.idx = shm->d_lists[id]; sa.n = shm->counts[id]; sa.time = s->time; sa.dt = s->dt;
            sa.pos = const_cast<float*>(means3D); sa.scale = const_cast<float*>(scales);
            sa.rot = const_cast<float*>(rotations); sa.opacity = const_cast<float*>(opacity);
            sa.sh = const_cast<float*>(shs); sa.M = s->M; sa.features = feats; sa.S = S;
            resolve(sh_shader_texture(id, 0), &sa.tex0);
            resolve(sh_shader_texture(id, 1), &sa.tex1);
            R3DG_CHECK_HIP(launch_sh_shader(id, sa, st));
            R3DG_CHECK_LAUNCH(s->debug, st);
        }
    }

    // the default-shader blend sorts its tiles itself (fused, tiles of up to kFusedSortMax instances)
    // only for S <= 12: with more feature channels its registers leave fewer waves to hide the
    // sort's barriers (M1 with S = 21: fused blend 0.78 ms vs 0.49 + 0.10 ms for the separate sort)
    // With depth-reading splat shaders the intermediate depth / stencil pass is the first consumer of
    // the sorted order: every tile is sorted by tile_depth_sort_kernel first (sorting in that pass's
    // prologue, as the blend does, measured slower: its larger LDS costs the pass more occupancy
    // than the separate sort, 0.43 + 0.10 -> 0.52 + 0.03 ms per frame at M1 / S = 21, round 5).
    // Otherwise the blend is the first consumer and sorts tiles of up to kFusedSortMax itself.
    const bool inter_first = splat_active && inter_pre;
    const bool fuse_sort = !inter_first && S <= 12;
    const bool sort_fused = fuse_sort;
    int L = 0;
    BinArgs binning{};
    binning.P = P; binning.grid_x = gx; binning.grid_y = gy; binning.rec4 = record_f4(S); binning.T = T;
    binning.offsets = geom.point_offsets; binning.means2D = geom.means2D; binning.radii = radii;
    binning.depth_keys = geom.depth_keys;
    binning.tile_work = img.tile_work;
    {
        const bool lds = bin_blocks_max(T) > 0 && !opt.test_bin_atomic;  // test_bin_atomic: the fallback (tests)
        int nb = bin_blocks_max(T);
        if (opt.test_bin_blocks > 0) nb = std::min(nb, opt.test_bin_blocks);  // experiments
        binning.nblk = lds ? std::min(nb, (P + kBinSub - 1) / kBinSub) : 0;
        binning.hist = lds && P > 0 ? img.bin_hist : nullptr;
        binning.tile_scan = binning.hist ? bin_tile_scan(img.bin_hist, (size_t)T) : nullptr;
    }
    if (P > 0) {
        PreprocessArgs pa{};
        pa.P = P; pa.D = s->D; pa.M = s->M; pa.W = W; pa.H = H; pa.grid_x = gx; pa.grid_y = gy;
        pa.prefiltered = s->prefiltered;
        pa.focal_x = focal_x; pa.focal_y = focal_y; pa.tan_fovx = s->tan_fovx; pa.tan_fovy = s->tan_fovy;
        pa.scale_modifier = s->scale_modifier;
        pa.means3D = means3D; pa.scales = scales; pa.rotations = rotations; pa.opacity = opacity;
        pa.sh = shs; pa.cov3D_precomp = g->cov3D_precomp; pa.colors_precomp = g->colors_precomp;
        pa.view = s->viewmatrix; pa.proj = s->projmatrix; pa.campos = s->campos;
        pa.radii = radii; pa.tiles_touched = geom.tiles_touched; pa.depth_keys = geom.depth_keys;
        pa.records = geom.records; pa.rec4 = record_f4(S); pa.S = S; pa.features = g->features;
        pa.depths = geom.depths;
        pa.means2D = geom.means2D; pa.cov3D = geom.cov3D; pa.conic_opacity = geom.conic_opacity;
        pa.rgb = geom.rgb; pa.clamped = geom.clamped; pa.error_flag = nullptr;
        pa.tile_count = binning.hist ? nullptr : img.tile_work;  // the atomic binning's counters
        pa.num_tiles = T;
        pa.scan_status = reinterpret_cast<uint64_t*>(geom.scan_temp);  // zeroed for scan_touched_kernel
        pa.scan_words = scan_blocks((size_t)P) + 1;
        pa.work_hist = img.bwd_hist;  // the forward's work buckets start at zero
        Readback* rb = nullptr;
        R3DG_CHECK_HIP(readback_slot(&rb));
        if (s->prefiltered) {
            // the reference __trap()s on a point the frustum test drops although the caller
            // promised a prefiltered set (auxiliary.h:154-160); here the kernel raises a flag and
            // the call fails with R3DG_ERR_ARG
            if (!rb->dev_flag) R3DG_CHECK_HIP(hipMalloc(&rb->dev_flag, sizeof(uint32_t)));
            R3DG_CHECK_HIP(hipMemsetAsync(rb->dev_flag, 0, sizeof(uint32_t), st));
            pa.error_flag = rb->dev_flag;
        }
        {
            ProfScope ps(R3DG_PROF_PREPROCESS, st);
            launch_kernel(preprocess_kernel, dim3((P + 255) / 256), dim3(256), st, pa);
        }
        R3DG_CHECK_LAUNCH(s->debug, st);

        // offsets = inclusive scan of tiles_touched; num_rendered (rasterizer_impl.cu:259-263 reads it
        // with a blocking cudaMemcpy) written by the scan's last workgroup into pinned coherent host
        // memory, which the host polls (wait_published)
        reinterpret_cast<volatile uint32_t*>(rb->host)[0] = kUnpublished;
        hipLaunchKernelGGL(scan_touched_kernel, dim3(scan_blocks((size_t)P)), dim3(kScanThreads), 0, st,
                           geom.tiles_touched, geom.point_offsets, P, reinterpret_cast<uint64_t*>(geom.scan_temp),
                           s->prefiltered ? rb->dev_flag : nullptr, rb->host_dev);
        R3DG_CHECK_HIP(hipGetLastError());
        // binning passes that need only the scan: per-tile counts, ranges, the tile order and the
        // scatter positions run on the device while the host waits for num_rendered and allocates
        {
            ProfScope ps(R3DG_PROF_SORT, st, true, opt.prof_sort_markers);
            R3DG_CHECK_HIP(launch_bin_prepare(binning, img.ranges, img.tile_order, st));
            R3DG_CHECK_LAUNCH(s->debug, st);
        }
        R3DG_CHECK_HIP(wait_published(rb, st));
        const uint32_t Lh = *reinterpret_cast<volatile uint32_t*>(rb->host);
        R3DG_REQUIRE(!s->prefiltered || reinterpret_cast<volatile uint32_t*>(rb->host)[1] == 0,
                     "rasterize_gaussians: point is filtered although prefiltered is set (the reference traps, "
                     "auxiliary.h:156-160)");
        R3DG_REQUIRE(Lh < (1u << 31), "rasterize_gaussians: too many tile instances");
        L = (int)Lh;
    } else if (T > 0) {  // no Gaussians: every tile range empty
        R3DG_CHECK_HIP(hipMemsetAsync(img.tile_work, 0, sizeof(uint32_t) * (size_t)T, st));
        R3DG_CHECK_HIP(hipMemsetAsync(img.bwd_hist, 0, sizeof(uint32_t) * kWorkBuckets, st));  // (no preprocess)
        R3DG_CHECK_HIP(launch_bin_prepare(binning, img.ranges, img.tile_order, st));
        R3DG_CHECK_LAUNCH(s->debug, st);
    }

    void* bin_base = binning_alloc(binning_ctx, binning_state_bytes((size_t)L));
    if (!bin_base) {
        set_error("rasterize_gaussians: binning allocation failed");
        return R3DG_ERR_ALLOC;
    }
    BinningState bin = binning_state_from(bin_base, (size_t)L);
    if (L == 0) R3DG_CHECK_HIP(launch_bin_order(binning, img.ranges, img.tile_order, st));  // (no scatter)
    if (L > 0) {
        // every instance to its tile's next position (also records each Gaussian's first slot),
        // then every tile by (depth bits, Gaussian id): the
        // reference's 45-bit stable sort of (tile << 32 | depth bits) (rasterizer_impl.cu:366-374)
        ProfScope ps(R3DG_PROF_SORT, st, true, opt.prof_sort_markers);
        binning.pairs = bin.pairs;
        binning.flags = nullptr;  // the rows reduction zeroes its flags itself (backward)
        binning.L = (uint32_t)L;
        // two-pass scatter through tile buckets (the staged ids carry the tile's index in its bucket
        // in their top bits); test_bin_one_pass: straight to the tiles
        binning.stage = (!opt.test_bin_one_pass && P < (1 << kBinBucketShift)) ? reinterpret_cast<uint2*>(bin.sort_k1)
                                                                                : nullptr;
        R3DG_CHECK_HIP(launch_bin_scatter(binning, img.ranges, img.tile_order, st));
        R3DG_CHECK_LAUNCH(s->debug, st);
        // the default-shader blend sorts the tiles of up to kFusedSortMax instances itself
        R3DG_CHECK_HIP(launch_tile_depth_sort(T, img.ranges, img.tile_order, bin.pairs, bin.point_list,
                                              bin.sort_k1, bin.sort_v1, bin.sort_k2,
                                              sort_fused ? kFusedSortMax : 0, st));
        R3DG_CHECK_LAUNCH(s->debug, st);
    }

    // RenderIntermediateTextures (forward.cu:271-383): depth + stencil images
    IntermediateArgs ia{};
    ia.ranges = img.ranges; ia.point_list = bin.point_list; ia.means2D = geom.means2D;
    ia.conic_opacity = geom.conic_opacity; ia.depths = geom.depths; ia.stencils = geom.stencils;
    ia.stencil_opacity = geom.stencil_opacity; ia.W = W; ia.H = H; ia.grid_x = gx; ia.num_tiles = T;
    ia.out_depth = out->depth; ia.out_stencil = out->stencil;
    ia.records = geom.records; ia.rec4 = record_f4(S); ia.inter_rec = inter_rec;
    ia.tile_order = img.tile_order;  // longest tiles first, as the blends
    if (splat_active) {
        // the splat shaders read the intermediate depth / stencil images
        R3DG_REQUIRE(out->depth && out->stencil, "rasterize_gaussians: splat shaders need depth and stencil outputs");
        if (inter_pre) {
            R3DG_CHECK_HIP(launch_intermediate(ia, P, radii, st));
        } else {
            R3DG_CHECK_HIP(hipMemsetAsync(out->stencil, 0, sizeof(float) * (size_t)H * W, st));
        }
        R3DG_CHECK_LAUNCH(s->debug, st);
        for (int id = 0; id < (int)spm->counts.size(); ++id) {  // RunSplatShaders (forward.cu:907-971)
            if (spm->counts[id] == 0) continue;
            SplatShaderArgs sp{};
            sp.idx = spm->d_lists[id]; sp.n = spm->counts[id]; sp.W = W; sp.H = H; sp.time = s->time;
            sp.dt = s->dt; sp.pos = means3D; sp.means2D = geom.means2D; sp.depth_tex = out->depth;
            sp.stencil_tex = out->stencil; sp.viewmatrix_inv = s->viewmatrix_inv; sp.depths = geom.depths;
            // the reference passes geomState.rgb even with precomputed colours (then uninitialised)
            sp.rgb = g->colors_precomp ? g->colors_precomp : geom.rgb;
            sp.conic_opacity = geom.conic_opacity; sp.features = feats; sp.S = S; sp.stencils = geom.stencils;
            sp.stencil_opacity = geom.stencil_opacity; sp.out_rgb = geom.shader_rgb;
            resolve(splat_shader_texture(id), &sp.tex0);
            R3DG_CHECK_HIP(launch_splat_shader(id, sp, st));
            R3DG_CHECK_LAUNCH(s->debug, st);
        }
        hipLaunchKernelGGL(refresh_record_opacity_kernel, dim3((P + 255) / 256), dim3(256), 0, st, P, radii,
                           geom.conic_opacity, geom.records, record_f4(S));
        const int na4 = record_f4(S) - 2;
        hipLaunchKernelGGL(shader_record_kernel, dim3((unsigned)(((long long)P * na4 + 255) / 256)), dim3(256), 0, st,
                           P, na4, radii, geom.shader_rgb, feats, S, shader_rec);
        R3DG_CHECK_LAUNCH(s->debug, st);
    }

    RenderFwdArgs ra{};
    ra.records = geom.records;
    ra.ranges = img.ranges;
    ra.point_list = bin.point_list;
    ra.means2D = geom.means2D;
    ra.conic_opacity = geom.conic_opacity;
    ra.depths = geom.depths;
    ra.colors = g->colors_precomp ? g->colors_precomp : geom.rgb;
    ra.shader_colors = splat_active ? geom.shader_rgb : ra.colors;
    ra.features = feats;
    ra.bg = s->bg;
    ra.S = S; ra.W = W; ra.H = H; ra.grid_x = gx; ra.num_tiles = T; ra.cull = 1;
#ifdef R3DG_EXP_FWD_SPATIAL  // experiment builds: the forward in the XCD-aware spatial order
    ra.tile_order = nullptr;
#else
    // forward: longest tiles first, as the backward (round 6: render_fwd 0.507 -> 0.495 ms at M1,
    // profiles/r06/fwd_order_ab; rounds 2-4 measured the spatial order faster, before the fused sort)
    ra.tile_order = img.tile_order;
#endif
    ra.final_T = img.final_T;
    ra.n_contrib = img.n_contrib;
    ra.out_color = out->color;
    ra.out_opacity = out->opacity;
    ra.out_depth = out->depth;
    ra.out_feature = out->feature;
    ra.out_shader_color = out->shader_color;
    ra.flay = make_feature_layout(S, (long long)H * W, true);
    // default splat shaders leave every stencil value 0 (InitializeStencil, rasterizer_impl.cu:203-209):
    // the blend writes those zeros with its other outputs (no separate memset launch)
    ra.zero_stencil = splat_active ? nullptr : out->stencil;
    ra.contrib = bin.contrib;
    ra.pairs = fuse_sort ? bin.pairs : nullptr;  // fused depth sort (render_fwd_glds_kernel)
    ra.point_list_out = bin.point_list;
    ra.shader_rec = shader_rec;
    ra.cull = opt.test_no_cull ? 0 : 1;
    ra.bwd_work = T > 0 ? img.bwd_work : nullptr;
    ra.bwd_rank = img.bwd_rank;
    ra.bwd_hist = img.bwd_hist;
    if (prepared_sums && T > 0) {
        ra.zero_sums = reinterpret_cast<float4*>(prepared_sums);
        ra.zero_n4 = (uint32_t)((size_t)sums_srs * (size_t)P / 4);
        ra.zero_chunk = (ra.zero_n4 + (uint32_t)T - 1) / (uint32_t)T;
    }
    {
        ProfScope ps(R3DG_PROF_RENDER_FWD, st);
        R3DG_CHECK_HIP(launch_render_forward(ra, splat_active, st));
    }
    R3DG_CHECK_LAUNCH(s->debug, st);

    if (s->compute_pseudo_normal) {
        XyzNormalArgs xa{};
        xa.W = W; xa.H = H; xa.view = s->viewmatrix; xa.focal_x = focal_x; xa.focal_y = focal_y;
        xa.cx = s->cx; xa.cy = s->cy; xa.opacity = out->opacity; xa.depth = out->depth;
        xa.normal = out->normal; xa.xyz = out->surface_xyz;
        // kOrderSlices leading workgroups sort the backward's tile order (tile_order_by_work) meanwhile
        xa.num_tiles = T; xa.bwd_work = img.bwd_work; xa.bwd_rank = img.bwd_rank; xa.bwd_hist = img.bwd_hist;
        xa.bwd_order = T > 0 ? img.bwd_order : nullptr;
        xa.blocks_x = gx;
        hipLaunchKernelGGL(xyz_normal_kernel, dim3((T > 0 ? kOrderSlices : 0) + gx * ((gy + R3DG_XYZ_R - 1) / R3DG_XYZ_R)),
                           dim3(256), 0, st, xa);
        R3DG_CHECK_LAUNCH(s->debug, st);
    } else {
        if (T > 0) R3DG_CHECK_HIP(launch_bwd_order(T, img.bwd_work, img.bwd_rank, img.bwd_hist, img.bwd_order, st));
        if (out->normal) R3DG_CHECK_HIP(hipMemsetAsync(out->normal, 0, sizeof(float) * 3 * (size_t)H * W, st));
        if (out->surface_xyz)
            R3DG_CHECK_HIP(hipMemsetAsync(out->surface_xyz, 0, sizeof(float) * 3 * (size_t)H * W, st));
    }
    if (!post_ids.empty()) {
        // rasterizer_impl.cu:485-529: depth and stencil are rendered again (now with the splat
        // shaders' stencils) and replace the blended depth, then the passes run in list order
        R3DG_CHECK_HIP(launch_intermediate(ia, P, radii, st));
        R3DG_CHECK_LAUNCH(s->debug, st);
        PostArgs pp{};
        pp.W = W; pp.H = H; pp.sh_color = out->color; pp.opacity = out->opacity; pp.depth = out->depth;
        pp.stencil = out->stencil; pp.surface_xyz = out->surface_xyz; pp.pseudonormal = out->normal;
        pp.shader_color = out->shader_color; pp.features = S == 21 ? out->feature : nullptr;
        pp.shadow = shadow_tex;
        float* scratch = post_blur ? reinterpret_cast<float*>(static_cast<char*>(geom_base) + geom_bytes) + work_floats
                                   : nullptr;
        R3DG_CHECK_HIP(launch_post_passes(post_ids.data(), (int)post_ids.size(), pp, scratch, st));
        R3DG_CHECK_LAUNCH(s->debug, st);
    }
    if (prepared_sums && T > 0) {
        const PreparedSums ps{prepared_sums, P, S, sums_srs, true};
        note_prepared_sums(geom_base, &ps);
    } else {
        note_prepared_sums(geom_base, nullptr);
    }
    *num_rendered = L;
    return R3DG_OK;
}

extern "C" int r3dg_state_view(int P, int H, int W, int L, void* geom, void* binning, void* image,
                               r3dg_binning_view* v) {
    R3DG_REQUIRE(v, "state_view: null");
    GeomState gs = geom_state_from(geom, (size_t)P);
    BinningState bs = binning_state_from(binning, (size_t)L);
    ImageState is = image_state_from(image, H, W);
    v->point_list = bs.point_list;
    v->ranges = reinterpret_cast<const uint32_t*>(is.ranges);
    v->point_offsets = gs.point_offsets;
    v->depths = gs.depths;
    v->means2D = reinterpret_cast<const float*>(gs.means2D);
    v->conic_opacity = reinterpret_cast<const float*>(gs.conic_opacity);
    v->rgb = gs.rgb;
    v->cov3D = gs.cov3D;
    v->clamped = gs.clamped;
    return R3DG_OK;
}

extern "C" int r3dg_rasterize_gaussians_backward(const r3dg_raster_settings* s, const r3dg_gaussians* g,
                                                 const int* radii_in, const r3dg_backward_grads* gr, void* geom,
                                                 void* binning, void* image, int num_rendered,
                                                 int backward_geometry, r3dg_alloc_fn scratch_alloc,
                                                 void* scratch_ctx, const r3dg_backward_outputs* out,
                                                 r3dg_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    R3DG_REQUIRE(s && g && gr && out, "rasterize_gaussians_backward: null argument");
    R3DG_REQUIRE(s->struct_size == sizeof(r3dg_raster_settings),
                 "rasterize_gaussians_backward: settings->struct_size must be sizeof(r3dg_raster_settings) (ABI 2)");
    R3DG_REQUIRE(out->struct_size == sizeof(r3dg_backward_outputs),
                 "rasterize_gaussians_backward: out->struct_size must be sizeof(r3dg_backward_outputs) (ABI 2)");
    const r3dg_options opt = options();
    const int P = s->P, S = s->S, H = s->H, W = s->W, L = num_rendered;
    R3DG_REQUIRE(P >= 0 && L >= 0 && S >= 0 && S <= kMaxFeatures, "rasterize_gaussians_backward: invalid sizes");
    R3DG_REQUIRE(out->dense_stride == 0 || out->dense_stride == 11 + S,
                 "rasterize_gaussians_backward: dense_stride must be 0 or 11 + S");
    R3DG_REQUIRE(!g->sh || P == 0 || (s->D >= 0 && s->D <= 3 && (s->D + 1) * (s->D + 1) <= s->M && s->M <= 16),
                 "rasterize_gaussians_backward: SH degree must be 0..3 with (degree+1)^2 <= M <= 16 coefficients");
    if (P == 0) return R3DG_OK;
    const int gx = (W + kTileX - 1) / kTileX, gy = (H + kTileY - 1) / kTileY;
    const int T = gx * gy;
    GeomState gs = geom_state_from(geom, (size_t)P, S);
    BinningState bs = binning_state_from(binning, (size_t)L);
    ImageState is = image_state_from(image, H, W);
    const int* radii = radii_in ? radii_in : gs.internal_radii;
    const int RS = part_row_stride(S);
    // scratch: partial rows [4L, RS] (one per instance and quadrant, written sparsely) and the
    // per-Gaussian sums [P, RS]; the rows' presence flags live in the binning state, zeroed here
    // (rows reduction only: the default atomic flush has no flags, so the forward's scatter no
    // longer writes the 4L bytes)
    // the backward blend addresses partial rows with 32-bit offsets in float4 units
    R3DG_REQUIRE((size_t)RS * (size_t)L < (1ull << 32), "rasterize_gaussians_backward: too many tile instances");
    // The second stage of the per-instance reduction (backward.cu:552-611 accumulates per pixel with
    // atomics). Default: the backward blend adds each (instance, wave) row into the per-Gaussian sums
    // with f32 atomics (no partial rows, flags or row_sum_kernel; last bits depend on arrival order,
    // as the reference's do; M1: step 2.00 -> 1.94 ms). bwd_reduce = R3DG_REDUCE_ROWS: partial rows
    // summed in a fixed order by row_sum_kernel, bitwise reproducible run to run. The DPP
    // cross-check kernel writes partial rows.
    const bool atomic_sums = opt.bwd_reduce != R3DG_REDUCE_ROWS && !opt.test_bwd_dpp;
    // atomic sums: [X part (f32) | 6 moments (f64) | pad] per Gaussian (atomic_sums_stride), zeroed
    // by the forward's blend when it prepared them (take_prepared_sums), else here
    const int srs_min = atomic_sums_min_stride(S);
    const int SRS = atomic_sums_stride(S, opt);
    R3DG_REQUIRE(SRS >= srs_min && SRS % 8 == 0, "rasterize_gaussians_backward: sums row stride too small");
    float* prepared = atomic_sums ? take_prepared_sums(geom, P, S, SRS) : nullptr;
    const size_t row_bytes = atomic_sums ? 0 : sizeof(float) * (size_t)RS * 4 * L;
    const size_t sum_bytes = sizeof(float) * (size_t)(atomic_sums ? SRS : RS) * P;
    char* scratch = (char*)scratch_alloc(scratch_ctx, row_bytes + (prepared ? 0 : sum_bytes));
    if (!scratch) {
        set_error("rasterize_gaussians_backward: scratch allocation failed");
        return R3DG_ERR_ALLOC;
    }
    float* rows = L > 0 && !atomic_sums ? reinterpret_cast<float*>(scratch) : nullptr;
    float* sums = prepared ? prepared : reinterpret_cast<float*>(scratch + row_bytes);
    if (atomic_sums && !prepared) {
        ProfScope ps(R3DG_PROF_ROW_SUM, st);
        R3DG_CHECK_HIP(hipMemsetAsync(sums, 0, sum_bytes, st));
    }
    uint8_t* flags = reinterpret_cast<uint8_t*>(bs.flags);
    if (!atomic_sums && L > 0) R3DG_CHECK_HIP(hipMemsetAsync(flags, 0, sizeof(uint32_t) * (size_t)L, st));
    if (L > 0) {
        RenderBwdArgs ba{};
        ba.records = gs.records;
        ba.ranges = is.ranges;
        ba.point_list = bs.point_list;
        ba.offsets = gs.point_offsets;
        ba.radii = radii;
        ba.means2D = gs.means2D;
        ba.conic_opacity = gs.conic_opacity;
        ba.depths = gs.depths;
        ba.colors = g->colors_precomp ? g->colors_precomp : gs.rgb;
        ba.features = g->features;
        ba.bg = s->bg;
        ba.final_T = is.final_T;
        ba.n_contrib = is.n_contrib;
        ba.dL_dpix = gr->dL_dout_color;
        const long long HW = (long long)H * W;
        for (int c = 0; c < 3; ++c) {
            ba.ca[c] = gr->color_hwc ? c : (int)(c * HW);
            ba.cm[c] = gr->color_hwc ? 3 : 1;
        }
        ba.dL_dpix_o = gr->dL_dout_opacity;
        ba.dL_dpix_d = gr->dL_dout_depth;
        ba.dL_dpix_f = gr->dL_dout_feature;
        ba.gflay = make_feature_layout(S, HW, gr->feature_native != 0);
        ba.S = S; ba.W = W; ba.H = H; ba.grid_x = gx; ba.grid_y = gy; ba.num_tiles = T; ba.cull = 1;
        ba.tile_order = bwd_tile_order(is, opt);
        ba.cull = opt.test_no_cull ? 0 : 1;
        ba.variant_dpp = opt.test_bwd_dpp;
        ba.wterms = opt.test_bwd_wterms;
        ba.backward_geometry = backward_geometry;
        ba.RS = RS;
        ba.rows = rows;
        ba.flags = flags;
        ba.contrib = bs.contrib;
        ba.sums_atomic = atomic_sums;
        ba.sums = sums;
        ba.SRS = SRS;
        {
            ProfScope ps(R3DG_PROF_RENDER_BWD, st);
            R3DG_CHECK_HIP(launch_render_backward(ba, st));
        }
        R3DG_CHECK_LAUNCH(s->debug, st);
    }
    GatherBwdArgs ga{};
    ga.P = P; ga.D = s->D; ga.M = s->M; ga.S = S; ga.RS = RS;
    ga.W = W; ga.H = H; ga.grid_x = gx; ga.grid_y = gy;
    ga.rows = rows;
    ga.sums = sums;
    ga.sums_moments = atomic_sums;
    ga.SRS = SRS;
    ga.flags = reinterpret_cast<const uint32_t*>(flags);
    ga.means2D = gs.means2D;
    ga.conic_opacity = gs.conic_opacity;
    ga.offsets = gs.point_offsets;
    ga.radii = radii;
    ga.means3D = g->means3D;
    ga.sh = g->sh;
    ga.clamped = gs.clamped;
    ga.scales = g->scales;
    ga.rotations = g->rotations;
    ga.scale_modifier = s->scale_modifier;
    ga.cov3D = g->cov3D_precomp ? g->cov3D_precomp : gs.cov3D;
    ga.view = s->viewmatrix;
    ga.proj = s->projmatrix;
    ga.campos = s->campos;
    ga.focal_x = W / (2.0f * s->tan_fovx);
    ga.focal_y = H / (2.0f * s->tan_fovy);
    ga.tan_fovx = s->tan_fovx;
    ga.tan_fovy = s->tan_fovy;
    ga.use_scales = (g->scales != nullptr && g->cov3D_precomp == nullptr);
    ga.dL_dmeans2D = out->dL_dmeans2D;
    ga.dL_dcolors = out->dL_dcolors;
    ga.dL_dopacity = out->dL_dopacity;
    ga.dL_dmeans3D = out->dL_dmeans3D;
    ga.dL_dfeatures = out->dL_dfeatures;
    ga.dL_dcov3D = out->dL_dcov3D;
    ga.dL_dsh = (s->M > 0) ? out->dL_dsh : nullptr;
    ga.dL_dscales = out->dL_dscales;
    ga.dL_drotations = out->dL_drotations;
    if (out->dense_stride > 0) {
        ga.ld_m3 = ga.ld_op = ga.ld_sc = ga.ld_rot = ga.ld_f = out->dense_stride;
    } else {
        ga.ld_m3 = 3; ga.ld_op = 1; ga.ld_sc = 3; ga.ld_rot = 4; ga.ld_f = S;
    }
    if (!g->sh) ga.sh = nullptr;
    // per-Gaussian phase over n_chunks 256-aligned ranges; chunk_done after each range's launch
    const int nchunks = std::max(1, std::min(out->n_chunks, (P + 255) / 256));
    const int per = ((P + nchunks - 1) / nchunks + 255) & ~255;
    for (int c = 0, g0 = 0; g0 < P; ++c, g0 += per) {
        ga.g_begin = g0;
        ga.g_end = std::min(P, g0 + per);
        if (!atomic_sums) {
            ProfScope ps(R3DG_PROF_ROW_SUM, st);
            R3DG_CHECK_HIP(launch_row_sum(ga, st));
        }
        {
            ProfScope ps(R3DG_PROF_GATHER_BWD, st);
            R3DG_CHECK_HIP(launch_gather_backward(ga, st));
        }
        R3DG_CHECK_LAUNCH(s->debug, st);
        if (out->chunk_done) out->chunk_done(out->chunk_ctx, c, ga.g_begin, ga.g_end);
    }
    return R3DG_OK;
}

extern "C" int r3dg_sh_color_grads(int P, int g0, int n, void* geom, const float* dL_dcolors, float* drgb,
                                   r3dg_stream_t stream) {
    R3DG_REQUIRE(P >= 0 && g0 >= 0 && n >= 0 && g0 + n <= P && geom && (n == 0 || (dL_dcolors && drgb)),
                 "sh_color_grads: invalid arguments");
    const GeomState gs = geom_state_from(geom, (size_t)P);
    R3DG_CHECK_HIP(launch_sh_color_grads(n, gs.clamped + g0, dL_dcolors + 3 * (size_t)g0, drgb, (hipStream_t)stream));
    return R3DG_OK;
}

extern "C" int r3dg_sh_grad_from_views(int g0, int n, int degree, int M, int N, const float* means3D,
                                       const float* campos, const float* drgb, float* dL_dsh, r3dg_stream_t stream) {
    R3DG_REQUIRE(g0 >= 0 && n >= 0 && N >= 1 && degree >= 0 && degree <= 3 && (degree + 1) * (degree + 1) <= M &&
                     M <= 16 && (n == 0 || (means3D && campos && drgb && dL_dsh)),
                 "sh_grad_from_views: invalid arguments (degree 0..3, (degree+1)^2 <= M <= 16)");
    R3DG_CHECK_HIP(launch_sh_grad_views(g0, n, degree, M, N, means3D, campos, drgb, dL_dsh, (hipStream_t)stream));
    return R3DG_OK;
}

extern "C" int r3dg_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                                 uint8_t* present, r3dg_stream_t stream) {
    (void)projmatrix;
    if (P <= 0) return R3DG_OK;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, means3D,
                       viewmatrix, present);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}

extern "C" int r3dg_shader_count(int kind) { return (int)shader_names(kind).size(); }
extern "C" const char* r3dg_shader_name(int kind, int index) {
    const auto& n = shader_names(kind);
    return (index >= 0 && index < (int)n.size()) ? n[index].c_str() : nullptr;
}
extern "C" int64_t r3dg_shader_handle(int kind, int index) {
    const auto& n = shader_names(kind);
    return (index >= 0 && index < (int)n.size()) ? make_handle(kind, index) : 0;
}

extern "C" int r3dg_preprocess_model(int P, const float* xyz, int64_t* sh_manager, int64_t* splat_manager,
                                     r3dg_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    R3DG_REQUIRE(P >= 0 && sh_manager && splat_manager, "PreprocessModel: invalid arguments");
    std::vector<int8_t> hs(P), hp(P);
    if (P > 0) {
        int8_t *ds = nullptr, *dp = nullptr;
        R3DG_CHECK_HIP(hipMalloc(&ds, P));
        R3DG_CHECK_HIP(hipMalloc(&dp, P));
        hipLaunchKernelGGL(select_shaders_kernel, dim3((P + 255) / 256), dim3(256), 0, st, P, xyz, ds, dp,
                           name_index(R3DG_SHADER_SH, "ShDefault"), name_index(R3DG_SHADER_SH, "Heartbeat"),
                           name_index(R3DG_SHADER_SH, "GaussDissolve"), name_index(R3DG_SHADER_SPLAT, "SplatDefault"),
                           name_index(R3DG_SHADER_SPLAT, "Wireframe"), name_index(R3DG_SHADER_SPLAT, "NaiveOutline"),
                           name_index(R3DG_SHADER_SPLAT, "Dissolve"));
        R3DG_CHECK_HIP(hipGetLastError());
        R3DG_CHECK_HIP(hipMemcpyAsync(hs.data(), ds, P, hipMemcpyDeviceToHost, st));
        R3DG_CHECK_HIP(hipMemcpyAsync(hp.data(), dp, P, hipMemcpyDeviceToHost, st));
        R3DG_CHECK_HIP(hipStreamSynchronize(st));
        R3DG_CHECK_HIP(hipFree(ds));
        R3DG_CHECK_HIP(hipFree(dp));
    }
    std::vector<int> is(hs.begin(), hs.end()), ip(hp.begin(), hp.end());
    int rc = build_manager(R3DG_SHADER_SH, P, is, sh_manager, st);
    if (rc) return rc;
    return build_manager(R3DG_SHADER_SPLAT, P, ip, splat_manager, st);
}

extern "C" int r3dg_create_shader_manager(int kind, int P, const int64_t* handles, int64_t* manager,
                                          r3dg_stream_t stream) {
    R3DG_REQUIRE(kind == R3DG_SHADER_SH || kind == R3DG_SHADER_SPLAT, "create_shader_manager: bad kind");
    R3DG_REQUIRE(P >= 0 && manager && (P == 0 || handles), "create_shader_manager: invalid arguments");
    std::vector<int> idx(P);
    for (int i = 0; i < P; ++i) {
        R3DG_REQUIRE(handle_kind(handles[i]) == kind, "create_shader_manager: handle of the wrong shader kind");
        idx[i] = handle_index(handles[i]);
    }
    return build_manager(kind, P, idx, manager, (hipStream_t)stream);
}

extern "C" int r3dg_shader_manager_info(int64_t manager, int* n_shaders, int64_t* handles, int* counts) {
    ShaderManagerObj* m = lookup_manager(manager);
    R3DG_REQUIRE(m, "shader_manager_info: unknown handle");
    const int n = (int)m->counts.size();
    if (n_shaders) *n_shaders = n;
    for (int i = 0; i < n; ++i) {
        if (handles) handles[i] = make_handle(m->kind, i);
        if (counts) counts[i] = m->counts[i];
    }
    return R3DG_OK;
}

// utils/texture.cu:33-76
extern "C" int r3dg_encode_texture_mode(const char* mode) {
    static const char* names[] = {"1", "L", "P", "RGB", "RGBA", "CMYK", "YCbCr", "LAB", "HSV", "I", "F"};
    for (int i = 0; i < 11; ++i)
        if (mode && strcmp(mode, names[i]) == 0) return i;
    return -1;
}
extern "C" int r3dg_encode_wrap_mode(const char* mode) {
    if (!mode) return -1;
    if (!strcmp(mode, "Border")) return (int)hipAddressModeBorder;
    if (!strcmp(mode, "Clamp")) return (int)hipAddressModeClamp;
    if (!strcmp(mode, "Mirror")) return (int)hipAddressModeMirror;
    if (!strcmp(mode, "Wrap")) return (int)hipAddressModeWrap;
    return -1;
}

extern "C" int r3dg_profile_enable(int max_records) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (int k = 0; k < R3DG_PROF_KINDS; ++k) {
        for (int e = 0; e < 2; ++e) {
            for (hipEvent_t ev : g_prof.ev[k][e]) R3DG_CHECK_HIP(hipEventDestroy(ev));
            g_prof.ev[k][e].clear();
        }
        g_prof.n[k] = 0;
    }
    g_prof.max_records = max_records > 0 ? max_records : 0;
    for (int k = 0; k < R3DG_PROF_KINDS; ++k)
        for (int e = 0; e < 2; ++e) {
            g_prof.ev[k][e].resize(g_prof.max_records);
            for (auto& ev : g_prof.ev[k][e]) R3DG_CHECK_HIP(hipEventCreate(&ev));
        }
    return R3DG_OK;
}

extern "C" int r3dg_profile_read(int kernel, int* count, float* total_ms) {
    R3DG_REQUIRE(kernel >= 0 && kernel < R3DG_PROF_KINDS && count && total_ms, "profile_read: bad arguments");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    float sum = 0.f;
    const int n = g_prof.n[kernel];
    for (int i = 0; i < n; ++i) {
        R3DG_CHECK_HIP(hipEventSynchronize(g_prof.ev[kernel][1][i]));
        float ms = 0.f;
        R3DG_CHECK_HIP(hipEventElapsedTime(&ms, g_prof.ev[kernel][0][i], g_prof.ev[kernel][1][i]));
        sum += ms;
    }
    g_prof.n[kernel] = 0;
    *count = n;
    *total_ms = sum;
    return R3DG_OK;
}
