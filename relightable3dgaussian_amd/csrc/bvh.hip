// bvh.hip -- linear BVH over the Gaussians and visibility ray tracing.
//
// Replaces the reference's `bvh_tracing._C` (bvh/src/bindings.cpp:9-11): create_bvh
// (bvh/src/bvh.cu:8-26, construct.cu:148-265), trace_bvh_opacity (bvh.cu:87-117,
// trace.cu:199-286), trace_bvh (bvh.cu:28-85, trace.cu:8-196), and the leaf-box math of
// RayTracer.__init__ (bvh/__init__.py:29-59), which the reference runs as ~40 torch launches.
//
// MI355X design (not a translation of the thrust lambdas):
//   * build = 5-7 launches + one rocPRIM radix sort on the caller's stream, no host syncs:
//     partial bounds -> final bounds -> Morton codes (also snapshots the leaf boxes) ->
//     stable 30-bit radix sort of (code, Gaussian) -> leaf rows + 61-bit keys ->
//     segment tree over the sorted leaf boxes (log2(P)/8 launches) -> Karras split per internal
//     node, whose subtree count is its key range's length and whose box is that range's merge
//     (no atomics, no fences: see range_box).
//   * traces: one lane per ray, depth-first with a 64-entry stack (16 entries in LDS), over
//     64-B node / Gaussian records packed per call (bvh_pack_kernel). The 61-bit keys are distinct,
//     so the tree depth is at most 61 and the stack can never overflow (the reference's 32-entry
//     IndexStack can, trace.cuh:22-45, with a printf and an out-of-bounds write).
//   * the arithmetic is the reference's, operation for operation, and this file is compiled with
//     -ffp-contract=off (build.py) so the result is bit-identical to the C restatement
//     oracle/r3dg_bvh.c (only the trace's exp differs: __expf as the reference).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "r3dg_common.h"

#include <rocprim/rocprim.hpp>

namespace r3dg {
namespace {

constexpr int kBvhStack = 64;

// aabb_type (bvh/include/utility.cuh:6-9): lower xyz, upper xyz
struct Box {
    float lx, ly, lz, ux, uy, uz;
};

__device__ __forceinline__ Box load_box(const float* a, int i) {
    const float2* p = reinterpret_cast<const float2*>(a + 6 * (size_t)i);  // 24-B rows: 8-B aligned
    const float2 u = p[0], v = p[1], w = p[2];
    return Box{u.x, u.y, v.x, v.y, w.x, w.y};
}

__device__ __forceinline__ void store_box(float* a, int i, const Box& b) {
    float2* p = reinterpret_cast<float2*>(a + 6 * (size_t)i);
    p[0] = make_float2(b.lx, b.ly);
    p[1] = make_float2(b.lz, b.ux);
    p[2] = make_float2(b.uy, b.uz);
}

// merge (utility.cuh:22-33)
__device__ __forceinline__ Box merge(const Box& a, const Box& b) {
    return Box{fminf(a.lx, b.lx), fminf(a.ly, b.ly), fminf(a.lz, b.lz),
               fmaxf(a.ux, b.ux), fmaxf(a.uy, b.uy), fmaxf(a.uz, b.uz)};
}

// ray_intersects(aabb, o, d) (utility.cuh:35-86): slab test in the reference's comparison order
__device__ __forceinline__ float2 ray_box(const Box& b, float3 o, float3 d) {
    float tmin = (b.lx - o.x) / d.x, tmax = (b.ux - o.x) / d.x;
    if (tmin > tmax) { const float s = tmin; tmin = tmax; tmax = s; }
    float tymin = (b.ly - o.y) / d.y, tymax = (b.uy - o.y) / d.y;
    if (tymin > tymax) { const float s = tymin; tymin = tymax; tymax = s; }
    if (tmin > tymax || tymin > tmax) return make_float2(-1.f, -1.f);
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.lz - o.z) / d.z, tzmax = (b.uz - o.z) / d.z;
    if (tzmin > tzmax) { const float s = tzmin; tzmin = tzmax; tzmax = s; }
    if (tmin > tzmax || tzmin > tmax) return make_float2(-1.f, -1.f);
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return make_float2(tmin, tmax);
}

// ray_intersects(mean, cov3D_inverse, o, d) (utility.cuh:94-104): t of the density maximum
__device__ __forceinline__ float ray_gauss_t(float3 m, const float* c, float3 o, float3 d) {
    const float mx = m.x - o.x, my = m.y - o.y, mz = m.z - o.z;
    const float c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3], c4 = c[4], c5 = c[5];
    const float t1 = c0 * mx * d.x + c1 * mx * d.y + c2 * mx * d.z + c1 * my * d.x + c3 * my * d.y +
                     c4 * my * d.z + c2 * mz * d.x + c4 * mz * d.y + c5 * mz * d.z;
    const float t2 = c0 * d.x * d.x + c1 * d.x * d.y + c2 * d.x * d.z + c1 * d.y * d.x + c3 * d.y * d.y +
                     c4 * d.y * d.z + c2 * d.z * d.x + c4 * d.z * d.y + c5 * d.z * d.z;
    return t1 / t2;
}

// gaussian_fn (utility.cuh:106-113); -0.5 (double in the reference) scales exactly
__device__ __forceinline__ float gauss_power(float3 m, float3 p, const float* c) {
    const float dx = m.x - p.x, dy = m.y - p.y, dz = m.z - p.z;
    return -0.5f * (dx * dx * c[0] + dy * dy * c[3] + dz * dz * c[5] + 2.f * dx * dy * c[1] +
                    2.f * dx * dz * c[2] + 2.f * dy * dz * c[4]);
}

__device__ __forceinline__ float3 ld3(const float* p, int i) {
    return make_float3(p[3 * (size_t)i], p[3 * (size_t)i + 1], p[3 * (size_t)i + 2]);
}

// ---- build -----------------------------------------------------------------------------------

// RayTracer.__init__ leaf boxes (bvh/__init__.py:29-59): build_rotation
// (utils/general_utils.py:82-103, re-normalising the quaternion), the 8 corners
// mean ± 3 s_a a ± 3 s_b b ± 3 s_c c with the torch evaluation order, min / max over them.
__global__ void __launch_bounds__(256) bvh_leaf_aabb_kernel(int P, const float* __restrict__ means,
                                                            const float* __restrict__ scales,
                                                            const float* __restrict__ rots,
                                                            float* __restrict__ leaf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float4 q4 = reinterpret_cast<const float4*>(rots)[i];
    const float norm = sqrtf(q4.x * q4.x + q4.y * q4.y + q4.z * q4.z + q4.w * q4.w);
    const float r = q4.x / norm, x = q4.y / norm, y = q4.z / norm, z = q4.w / norm;
    // columns of R: a = R[:, :, 0], b = R[:, :, 1], c = R[:, :, 2]
    const float a[3] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y + r * z), 2.f * (x * z - r * y)};
    const float b[3] = {2.f * (x * y - r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z + r * x)};
    const float c[3] = {2.f * (x * z + r * y), 2.f * (y * z - r * x), 1.f - 2.f * (x * x + y * y)};
    const float3 s = ld3(scales, i);
    const float sa = 3.f * s.x, sb = 3.f * s.y, sc = 3.f * s.z;
    const float3 m = ld3(means, i);
    const float mm[3] = {m.x, m.y, m.z};
    float lo[3], hi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float as = a[k] * sa, bs = b[k] * sb, cs = c[k] * sc;
        const float p1 = mm[k] + as, m1 = mm[k] - as;
        const float pp = p1 + bs, pm = p1 - bs, mp = m1 + bs, mn = m1 - bs;
        const float v[8] = {pp + cs, pp - cs, pm + cs, pm - cs, mp + cs, mp - cs, mn + cs, mn - cs};
        float l = v[0], h = v[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            l = fminf(l, v[j]);
            h = fmaxf(h, v[j]);
        }
        lo[k] = l;
        hi[k] = h;
    }
    store_box(leaf, i, Box{lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
}

// scene bounds (construct.cu:161-170 thrust::reduce with merge): per-block partial boxes
__global__ void __launch_bounds__(256) bvh_bounds_partial_kernel(int P, const float* __restrict__ leaf,
                                                                 float* __restrict__ partial) {
    __shared__ Box sb[256];
    Box acc{100000.f, 100000.f, 100000.f, -100000.f, -100000.f, -100000.f};  // default_aabb
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x)
        acc = merge(acc, load_box(leaf, i));
    sb[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) sb[threadIdx.x] = merge(sb[threadIdx.x], sb[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) store_box(partial, blockIdx.x, sb[0]);
}

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {  // construct.cu:6-13
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// morton_code_calculator (construct.cu:35-53, 22-33): the box centroid normalised to the scene
// bounds, 10 bits per axis. Also snapshots the leaf box for the gather after the sort.
__global__ void __launch_bounds__(256) bvh_morton_kernel(int P, int n_partial, const float* __restrict__ partial,
                                                         const float* __restrict__ leaf, uint32_t* __restrict__ code,
                                                         uint32_t* __restrict__ index, float* __restrict__ leaf_copy) {
    __shared__ Box red[256];  // n_partial <= 256 partial boxes, reduced cooperatively per block
    red[threadIdx.x] = (int)threadIdx.x < n_partial
                           ? load_box(partial, threadIdx.x)
                           : Box{100000.f, 100000.f, 100000.f, -100000.f, -100000.f, -100000.f};
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = merge(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const Box b = load_box(leaf, i);
    store_box(leaf_copy, i, b);
    const Box w = red[0];
    // centroid: (upper + lower) * 0.5 in double, rounded to float -- exact as 0.5f in float
    float px = (b.ux + b.lx) * 0.5f, py = (b.uy + b.ly) * 0.5f, pz = (b.uz + b.lz) * 0.5f;
    px -= w.lx; py -= w.ly; pz -= w.lz;
    px /= (w.ux - w.lx); py /= (w.uy - w.ly); pz /= (w.uz - w.lz);
    const float res = 1024.f;
    px = fminf(fmaxf(px * res, 0.f), res - 1.f);
    py = fminf(fmaxf(py * res, 0.f), res - 1.f);
    pz = fminf(fmaxf(pz * res, 0.f), res - 1.f);
    code[i] = expand_bits((uint32_t)px) * 4 + expand_bits((uint32_t)py) * 2 + expand_bits((uint32_t)pz);
    index[i] = (uint32_t)i;
}

// after the stable sort: leaf rows (construct.cu:200-205), sorted leaf boxes (the sort's zipped
// aabbs, :184-187) and the 61-bit keys code << 31 | Gaussian (:188-198)
__global__ void __launch_bounds__(256) bvh_leaf_rows_kernel(int P, const uint32_t* __restrict__ code,
                                                            const uint32_t* __restrict__ index,
                                                            const float* __restrict__ leaf_copy,
                                                            int32_t* __restrict__ nodes, float* __restrict__ aabbs,
                                                            uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint32_t g = index[i];
    keys[i] = ((uint64_t)code[i] << 31) | g;
    const int n = P - 1 + i;
    store_box(aabbs, n, load_box(leaf_copy, (int)g));
    int32_t* row = nodes + 5 * (size_t)n;
    if (P == 1) row[0] = -1;  // the root is a leaf; nobody else writes its parent
    row[1] = -1;
    row[2] = -1;
    row[3] = (int32_t)g;
    row[4] = 1;
}

// Internal-node boxes without a bottom-up climb. A Karras node covers the contiguous sorted
// leaves [first, last], and min / max are exact, so its box is the merge of the leaf boxes in that
// range -- the same bits the reference's pairwise child merges produce (construct.cu:231-264).
// The range merge is answered from an implicit segment tree over the sorted leaves (heap order,
// n = pow2 >= P; level above the leaves in seg[1..n), the leaves themselves are the aabbs rows):
// log2(n)/8 launches build it, then every internal node merges <= 2 log2(n) boxes. This replaces
// the reference's atomic climb, whose agent-scope fences flush the per-XCD L2 of MI355X on every
// step (5.6 ms at 1M Gaussians measured).
__device__ __forceinline__ Box box_identity() {
    return Box{INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
}

__device__ __forceinline__ Box seg_get(const float* seg, const float* leaf, int P, int n, int h) {
    if (h < n) return load_box(seg, h);
    return h - n < P ? load_box(leaf, h - n) : box_identity();
}

// one block: 256 consecutive nodes of the level starting at heap index in_lo (or all of them when
// the level is narrower) -> the up to 8 levels above
__global__ void __launch_bounds__(256) bvh_seg_level_kernel(int P, int n, int in_lo, const float* __restrict__ leaf,
                                                            float* seg) {
    __shared__ Box lv[256];
    const int cnt = in_lo < 256 ? in_lo : 256;
    const int first = in_lo + blockIdx.x * cnt;
    if ((int)threadIdx.x < cnt) lv[threadIdx.x] = seg_get(seg, leaf, P, n, first + threadIdx.x);
    __syncthreads();
    for (int step = 1, w = cnt >> 1; w >= 1; ++step, w >>= 1) {
        Box m;
        if ((int)threadIdx.x < w) m = merge(lv[2 * threadIdx.x], lv[2 * threadIdx.x + 1]);
        __syncthreads();
        if ((int)threadIdx.x < w) {
            lv[threadIdx.x] = m;
            store_box(seg, (first >> step) + threadIdx.x, m);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ Box range_box(const float* seg, const float* leaf, int P, int n, int first, int last) {
    Box acc = box_identity();
    for (int l = first + n, r = last + n + 1; l < r; l >>= 1, r >>= 1) {
        if (l & 1) acc = merge(acc, seg_get(seg, leaf, P, n, l++));
        if (r & 1) acc = merge(acc, seg_get(seg, leaf, P, n, --r));
    }
    return acc;
}

__device__ __forceinline__ int cub64(uint64_t a, uint64_t b) { return __clzll(a ^ b); }  // common_upper_bits

// one internal node per lane: determine_range (construct.cu:55-115) + find_split (:117-146),
// children and parent links (:207-229); the subtree leaf count is the range length, which is
// what the reference's bottom-up atomicAdd chain (:240) accumulates.
__global__ void __launch_bounds__(256) bvh_internal_kernel(int P, int n, const uint64_t* __restrict__ key,
                                                           int32_t* __restrict__ nodes, const float* __restrict__ seg,
                                                           float* __restrict__ aabbs) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int n_int = P - 1;
    if (idx >= n_int) return;
    int first, last;
    if (idx == 0) {
        first = 0;
        last = P - 1;
    } else {
        const uint64_t self = key[idx];
        const int dl = cub64(self, key[idx - 1]);
        const int dr = cub64(self, key[idx + 1]);
        const int d = dr > dl ? 1 : -1;
        const int dmin = dl < dr ? dl : dr;
        int lmax = 2, delta = -1, it = idx + d * lmax;
        if (0 <= it && it < P) delta = cub64(self, key[it]);
        while (delta > dmin) {
            lmax <<= 1;
            it = idx + d * lmax;
            delta = -1;
            if (0 <= it && it < P) delta = cub64(self, key[it]);
        }
        int l = 0;
        for (int t = lmax >> 1; t > 0; t >>= 1) {
            it = idx + (l + t) * d;
            delta = -1;
            if (0 <= it && it < P) delta = cub64(self, key[it]);
            if (delta > dmin) l += t;
        }
        const int j = idx + l * d;
        first = d < 0 ? j : idx;
        last = d < 0 ? idx : j;
    }
    int gamma;
    const uint64_t fc = key[first], lc = key[last];
    if (fc == lc) {
        gamma = (first + last) >> 1;
    } else {
        const int dn = cub64(fc, lc);
        int split = first, stride = last - first;
        do {
            stride = (stride + 1) >> 1;
            const int middle = split + stride;
            if (middle < last && cub64(fc, key[middle]) > dn) split = middle;
        } while (stride > 1);
        gamma = split;
    }
    int lc_id = gamma, rc_id = gamma + 1;
    if (first == gamma) lc_id += n_int;
    if (last == gamma + 1) rc_id += n_int;
    int32_t* row = nodes + 5 * (size_t)idx;
    if (idx == 0) row[0] = -1;
    row[1] = lc_id;
    row[2] = rc_id;
    row[3] = -1;
    row[4] = last - first + 1;
    nodes[5 * (size_t)lc_id] = idx;
    nodes[5 * (size_t)rc_id] = idx;
    store_box(aabbs, idx, range_box(seg, aabbs + 6 * (size_t)n_int, P, n, first, last));
}

// ---- traces ----------------------------------------------------------------------------------

// the reference's child visit order: the child whose exit distance is larger is pushed first
// (so the nearer-exiting one is popped first), children with exit <= 0 are dropped
template <typename Push>
__device__ __forceinline__ void push_children(const float* aabbs, int lid, int rid, float3 o, float3 d, Push push) {
    const float2 il = ray_box(load_box(aabbs, lid), o, d);
    const float2 ir = ray_box(load_box(aabbs, rid), o, d);
    if (il.y > ir.y) {
        if (il.y > 0) push(lid, il);
        if (ir.y > 0) push(rid, ir);
    } else {
        if (ir.y > 0) push(rid, ir);
        if (il.y > 0) push(lid, il);
    }
}

// Trace layouts, packed per call from the reference's tables (one pass, 64 B per node and per
// Gaussian, ~0.03 ms at 1M): a visited internal node costs ONE 64-B record (both child boxes and
// both child references) instead of a 20-B row plus two 24-B boxes in three dependent rounds, and
// a leaf costs one 64-B Gaussian record instead of four scattered arrays.
//   node record k (internal node k): {lbox[6], rbox[6], lref, rref, -, -}; ref >= 0 is an
//   internal node, ref < 0 is ~gaussian (a leaf: count <= 1, the reference's test)
//   gaussian record g: {mean xyz, opacity, normal xyz, -, cov_inv[6], -, -}
__global__ void __launch_bounds__(256) bvh_pack_kernel(int P, const int32_t* __restrict__ nodes,
                                                       const float* __restrict__ aabbs, const float* __restrict__ means,
                                                       const float* __restrict__ cov, const float* __restrict__ opac,
                                                       const float* __restrict__ normals, float4* __restrict__ nrec,
                                                       float4* __restrict__ grec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < P - 1) {
        const int l = nodes[5 * (size_t)i + 1], r = nodes[5 * (size_t)i + 2];
        const Box bl = load_box(aabbs, l), br = load_box(aabbs, r);
        const int lref = nodes[5 * (size_t)l + 4] <= 1 ? ~nodes[5 * (size_t)l + 3] : l;
        const int rref = nodes[5 * (size_t)r + 4] <= 1 ? ~nodes[5 * (size_t)r + 3] : r;
        float4* o = nrec + 4 * (size_t)i;
        o[0] = make_float4(bl.lx, bl.ly, bl.lz, bl.ux);
        o[1] = make_float4(bl.uy, bl.uz, br.lx, br.ly);
        o[2] = make_float4(br.lz, br.ux, br.uy, br.uz);
        o[3] = make_float4(__int_as_float(lref), __int_as_float(rref), 0.f, 0.f);
    }
    if (i < P) {
        const float* c = cov + 6 * (size_t)i;
        float4* o = grec + 4 * (size_t)i;
        const float3 m = ld3(means, i), n = ld3(normals, i);
        o[0] = make_float4(m.x, m.y, m.z, opac[i]);
        o[1] = make_float4(n.x, n.y, n.z, 0.f);
        o[2] = make_float4(c[0], c[1], c[2], c[3]);
        o[3] = make_float4(c[4], c[5], 0.f, 0.f);
    }
}

struct TraceOpacityArgs {
    int n_rays;
    int root_leaf;  // P == 1: the root is the leaf of Gaussian 0
    int g_bits;     // 2^g_bits lanes per ray (same wave), 0..6
    const float4* nrec;
    const float4* grec;
    const float* rays_o;
    const float* rays_d;
    int32_t* contrib;
    float* vis;
    int max_visits;  // 2 * nodes: a bound no valid tree reaches (each node is visited at most once)
    const uint32_t* perm;  // rays in Morton order of their origins (NULL: input order)
};

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch): give each
// XCD a contiguous range of the Morton-sorted rays, so the rays sharing an L2 share tree nodes.
__device__ __forceinline__ int xcd_block() {
    const int nb = gridDim.x, b = blockIdx.x, x = b % 8;
    int first = 0;
    for (int k = 0; k < x; ++k) first += (nb - k + 7) / 8;
    return first + b / 8;
}

// Morton code of each ray origin in the root box (the leaf-code formula of bvh_morton_kernel)
__global__ void __launch_bounds__(256) bvh_ray_morton_kernel(int R, const float* __restrict__ rays_o,
                                                             const float* __restrict__ aabbs,
                                                             uint32_t* __restrict__ code,
                                                             uint32_t* __restrict__ index) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const Box w = load_box(aabbs, 0);
    const float3 o = ld3(rays_o, i);
    const float px = fminf(fmaxf((o.x - w.lx) / (w.ux - w.lx) * 1024.f, 0.f), 1023.f);
    const float py = fminf(fmaxf((o.y - w.ly) / (w.uy - w.ly) * 1024.f, 0.f), 1023.f);
    const float pz = fminf(fmaxf((o.z - w.lz) / (w.uz - w.lz) * 1024.f, 0.f), 1023.f);
    code[i] = expand_bits((uint32_t)px) * 4 + expand_bits((uint32_t)py) * 2 + expand_bits((uint32_t)pz);
    index[i] = (uint32_t)i;
}

#ifndef R3DG_BVH_LDS
#define R3DG_BVH_LDS 16  // measured: 8 / 12 / 16 / 24 / 32 entries (tools/exp_bvh.sh); 16 fills 7 waves per SIMD
#endif
constexpr int kLdsStack = R3DG_BVH_LDS;  // per-lane stack entries in LDS ([entry][lane]: conflict-free)
// Group cut in the log domain. Every term a lane adds is __logf(1 - alpha) + kLogSlack, where
// kLogSlack bounds, per term, everything that separates the running sum from log of the
// reference's single-chain product: v_log_f32 (<= 1 ulp of a log2 in [-0.152, 0]: 1.5e-8), the ln 2
// scaling (4e-9), the LDS sum's rounding (|sum| < 0.2: 7.5e-9) and the reference chain's own
// f32 multiply per factor (2^-24 relative: 6e-8) -- 8.7e-8 in all, taken as 2e-7. A factor below
// 0.9 never reaches the sum (its lane's own product cuts exactly first). So a sum below
// log(0.9) - 1e-7 proves the reference's transmittance fell below 0.9: the ray is occluded
// whatever the remaining terms, and only then does the group stop early. Rays that never prove
// it finish, and the group's exact product decides.
constexpr float kLogCut = -0.10536052f - 1e-7f;
constexpr float kLogSlack = 2e-7f;

// trace_bvh_opacity_cuda (trace.cu:199-286): transmittance along the ray through every Gaussian
// whose box it crosses (front-facing normals, opacity >= 1/255, density maximum at t >= 0.01);
// once it drops below 0.9 the ray is occluded: visibility 0 and contribute 0 (the reference
// returns before storing its count into the zero-initialised output). The stack lives in LDS,
// deeper entries (> 16) in a private overflow array (scratch, L1/L2-cached).
//
// Few rays (the lambda_visibility loss traces 10k) cannot fill 256 CUs one lane per ray, and the
// time is then the longest traversal's latency. So a ray gets G = 2^g_bits lanes of one wave:
// lane j walks down g_bits levels along the bits of j (pruning as the reference does) and
// traverses that subtree in the reference's order; the group multiplies its partial
// transmittances and sums its counts. The cut is monotone (every factor is <= 1), so "the product
// fell below 0.9" is the same event whatever the order: the group keeps a running log-domain sum
// in LDS and every lane stops once it crosses the cut. Only the rounding of the product differs
// from the reference's single chain (G = 1 keeps the reference's order exactly).
__global__ void __launch_bounds__(256) bvh_trace_opacity_kernel(TraceOpacityArgs a) {
    __shared__ int lstack[kLdsStack][256];
    __shared__ float lsum[256];  // per group: sum of log(1 - alpha) so far (-inf: cut)
    const int tid = threadIdx.x;
    const int gb = a.g_bits;
    const int j = tid & ((1 << gb) - 1);
    const int gid = tid >> gb;  // group slot in this block
    const int slot = (int)(((long long)xcd_block() * blockDim.x + tid) >> gb);
    const bool live = slot < a.n_rays;
    const int ray = live && a.perm ? (int)a.perm[slot] : slot;
    if (j == 0) lsum[gid] = 0.f;
    __syncthreads();
    float3 o = make_float3(0.f, 0.f, 0.f), d = make_float3(0.f, 0.f, 1.f);
    if (live) {
        o = ld3(a.rays_o, ray);
        d = ld3(a.rays_d, ray);
    }
    int ostack[kBvhStack - kLdsStack];
    int sp = 0;
    auto push = [&](int v) {
        if (sp < kLdsStack) lstack[sp][tid] = v;
        else if (sp < kBvhStack) ostack[sp - kLdsStack] = v;
        if (sp < kBvhStack) ++sp;
    };
    // descend g_bits levels along the bits of j; a leaf met early belongs to the lane whose
    // remaining bits are zero, a pruned child to nobody
    int ref = a.root_leaf ? ~0 : 0;
    bool mine = live;
    for (int lv = 0; lv < gb && mine; ++lv) {
        if (ref < 0) {
            mine = (j >> lv) == 0;
            break;
        }
        const float4* r = a.nrec + 4 * (size_t)ref;
        const int right = (j >> lv) & 1;
        const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
        const float2 iv = right ? ray_box(Box{r1.z, r1.w, r2.x, r2.y, r2.z, r2.w}, o, d)
                                : ray_box(Box{r0.x, r0.y, r0.z, r0.w, r1.x, r1.y}, o, d);
        mine = iv.y > 0;
        ref = __float_as_int(right ? r3.y : r3.x);
    }
    if (mine) push(ref);
    int count = 0, visits = 0;
    float T = 1.f;
    bool occluded = false;
    while (sp > 0) {
        // the group's certified log-domain sum crossed the cut (kLogCut): occluded, stop
        if (gb > 0 && *(volatile float*)&lsum[gid] < kLogCut) break;
        --sp;
        const int rf = sp < kLdsStack ? lstack[sp][tid] : ostack[sp - kLdsStack];
        if (rf < 0) {
            const float4* g = a.grec + 4 * (size_t)(~rf);
            const float4 g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3];  // one 64-B line, one round trip
            if (g0.w < 1.f / 255.f) continue;
            if (g1.x * d.x + g1.y * d.y + g1.z * d.z > 0) continue;
            const float c[6] = {g2.x, g2.y, g2.z, g2.w, g3.x, g3.y};
            const float3 m = make_float3(g0.x, g0.y, g0.z);
            const float t = ray_gauss_t(m, c, o, d);
            if ((double)t < 0.01) continue;
            const float3 p = make_float3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
            const float power = gauss_power(m, p, c);
            if (power > 0) continue;
            count += 1;
            const float alpha = g0.w * __expf(power);
            T *= 1 - alpha;
            if ((double)T < 0.9) {
                occluded = true;
                if (gb > 0) lsum[gid] = -INFINITY;
                break;
            }
            if (gb > 0) atomicAdd(&lsum[gid], __logf(1 - alpha) + kLogSlack);
        } else {
            const float4* r = a.nrec + 4 * (size_t)rf;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
            const float2 il = ray_box(Box{r0.x, r0.y, r0.z, r0.w, r1.x, r1.y}, o, d);
            const float2 ir = ray_box(Box{r1.z, r1.w, r2.x, r2.y, r2.z, r2.w}, o, d);
            const int lid = __float_as_int(r3.x), rid = __float_as_int(r3.y);
            if (il.y > ir.y) {
                if (il.y > 0) push(lid);
                if (ir.y > 0) push(rid);
            } else {
                if (ir.y > 0) push(rid);
                if (il.y > 0) push(lid);
            }
        }
        if (++visits > a.max_visits) break;  // only a malformed tree gets here
    }
    if (gb > 0) {  // combine the group's partial results (butterfly within the wave)
        for (int m = 1; m < (1 << gb); m <<= 1) {
            T *= __shfl_xor(T, m, 64);
            count += __shfl_xor(count, m, 64);
        }
        __syncthreads();  // every lane's updates are visible
        occluded = lsum[gid] < kLogCut || (double)T < 0.9;
    }
    if (live && j == 0) {
        a.contrib[ray] = occluded ? 0 : count;
        a.vis[ray] = occluded ? 0.f : T;
    }
}

// Few-rays variant with dynamic balancing: the G lanes of a ray's group share one LDS stack
// (kShared entries per lane). Every round each idle lane (empty private stack) pops one entry from
// the top of the shared stack, all lanes process their node, and the children are pushed back in
// lane order through a group prefix sum (pushes that do not fit go to the pushing lane's private
// stack, which it drains first). Uniform per group: the stack pointer lives in a register of every
// lane of the group, so no LDS atomics or barriers are needed -- a group never leaves its wave.
// The subtree split of bvh_trace_opacity_kernel leaves most of an escaping ray's work in the one
// subtree around its origin; here every lane keeps taking the next pending node.
constexpr int kShared = 16;

__device__ __forceinline__ int group_incl_scan(int v, int width) {
    for (int o = 1; o < width; o <<= 1) {
        const int u = __shfl_up(v, o, width);
        if ((threadIdx.x & (width - 1)) >= o) v += u;
    }
    return v;
}

__global__ void __launch_bounds__(256) bvh_trace_opacity_shared_kernel(TraceOpacityArgs a) {
    __shared__ int sstack[256 * kShared];
    __shared__ float lsum[256];
    const int tid = threadIdx.x;
    const int gb = a.g_bits, G = 1 << gb;
    const int j = tid & (G - 1);
    const int gid = tid >> gb;
    const int lane = tid & 63;
    const uint64_t gmask = G == 64 ? ~0ull : (((1ull << G) - 1) << (lane & ~(G - 1)));
    const uint64_t below = (1ull << lane) - 1;
    const int slot = (int)(((long long)xcd_block() * blockDim.x + tid) >> gb);
    const bool live = slot < a.n_rays;
    const int ray = live && a.perm ? (int)a.perm[slot] : slot;
    const int C = kShared * G;
    int* st = sstack + gid * C;
    if (j == 0) lsum[gid] = 0.f;
    float3 o = make_float3(0.f, 0.f, 0.f), d = make_float3(0.f, 0.f, 1.f);
    if (live) {
        o = ld3(a.rays_o, ray);
        d = ld3(a.rays_d, ray);
    }
    int pstack[kBvhStack];
    int psp = 0;
    int sp = live ? 1 : 0;  // uniform within the group
    if (live && j == 0) st[0] = a.root_leaf ? ~0 : 0;
    int count = 0, visits = 0;
    float T = 1.f;
    bool occluded = false;
    while (true) {
        const uint64_t busy = __ballot(psp > 0) & gmask;
        if (sp == 0 && busy == 0) break;
        if (*(volatile float*)&lsum[gid] < kLogCut) break;
        const uint64_t idle = ~busy & gmask;
        const int n_idle = __popcll(idle), rank = __popcll(idle & below);
        const int take = sp < n_idle ? sp : n_idle;
        bool have = false;
        int rf = 0;
        if (psp > 0) {
            rf = pstack[--psp];
            have = true;
        } else if (rank < take) {
            rf = st[sp - 1 - rank];
            have = true;
        }
        sp -= take;
        int e0 = 0, e1 = 0, nc = 0;  // children to push, e1 ends on top
        if (have) {
            ++visits;
            if (rf < 0) {
                const float4* g = a.grec + 4 * (size_t)(~rf);
                const float4 g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3];
                bool hit = !(g0.w < 1.f / 255.f) && !(g1.x * d.x + g1.y * d.y + g1.z * d.z > 0);
                const float c[6] = {g2.x, g2.y, g2.z, g2.w, g3.x, g3.y};
                const float3 m = make_float3(g0.x, g0.y, g0.z);
                float t = 0.f;
                if (hit) {
                    t = ray_gauss_t(m, c, o, d);
                    hit = !((double)t < 0.01);
                }
                if (hit) {
                    const float3 p = make_float3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
                    const float power = gauss_power(m, p, c);
                    if (!(power > 0)) {
                        count += 1;
                        const float alpha = g0.w * __expf(power);
                        T *= 1 - alpha;
                        if ((double)T < 0.9) {
                            occluded = true;
                            lsum[gid] = -INFINITY;
                        } else {
                            atomicAdd(&lsum[gid], __logf(1 - alpha) + kLogSlack);
                        }
                    }
                }
            } else {
                const float4* r = a.nrec + 4 * (size_t)rf;
                const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
                const float2 il = ray_box(Box{r0.x, r0.y, r0.z, r0.w, r1.x, r1.y}, o, d);
                const float2 ir = ray_box(Box{r1.z, r1.w, r2.x, r2.y, r2.z, r2.w}, o, d);
                const int lid = __float_as_int(r3.x), rid = __float_as_int(r3.y);
                const bool lfirst = il.y > ir.y;  // the reference's push order
                const int f = lfirst ? lid : rid, s2 = lfirst ? rid : lid;
                const bool hf = lfirst ? il.y > 0 : ir.y > 0, hs = lfirst ? ir.y > 0 : il.y > 0;
                if (hf) e0 = f;
                if (hs) {
                    if (hf) e1 = s2;
                    else e0 = s2;
                }
                nc = (hf ? 1 : 0) + (hs ? 1 : 0);
            }
        }
        const int incl = group_incl_scan(nc, G);
        const int total = __shfl(incl, G - 1, G);
        const int room = C - sp;
        for (int k = 0; k < nc; ++k) {
            const int pos = incl - nc + k;
            const int e = k == 0 ? e0 : e1;
            if (pos < room) st[sp + pos] = e;
            else if (psp < kBvhStack) pstack[psp++] = e;
        }
        sp += total < room ? total : room;
        if (visits > a.max_visits) psp = 0, sp = 0;  // only a malformed tree gets here
    }
    for (int m = 1; m < G; m <<= 1) {
        T *= __shfl_xor(T, m, 64);
        count += __shfl_xor(count, m, 64);
    }
    occluded = occluded || lsum[gid] < kLogCut || (double)T < 0.9;
    occluded = __ballot(occluded) & gmask;
    if (live && j == 0) {
        a.contrib[ray] = occluded ? 0 : count;
        a.vis[ray] = occluded ? 0.f : T;
    }
}

struct TraceListArgs {
    int n_rays;
    const int32_t* nodes;
    const float* aabbs;
    const float* rays_o;
    const float* rays_d;
    const float* means;
    int32_t* contrib;      // [n_rays] leaves in every crossed <=4-leaf subtree
    const int32_t* offs;   // inclusive scan of contrib
    uint64_t* keys;        // ray << 32 | bits(t)
    uint32_t* order;       // emission slot (sort value)
    int32_t* point;        // emission order
    float* position;       // emission order, [L, 3]
    int32_t* ray_id;
    int max_visits;
};

// trace_bvh_cuda pass 1 (trace.cu:20-59): leaves of every crossed subtree with <= 4 leaves
__global__ void __launch_bounds__(256) bvh_trace_count_kernel(TraceListArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.n_rays) return;
    const float3 o = ld3(a.rays_o, idx), d = ld3(a.rays_d, idx);
    int stack[kBvhStack];
    int sp = 0;
    stack[sp++] = 0;
    int count = 0, visits = 0;
    while (sp > 0) {
        const int node = stack[--sp];
        const int32_t* row = a.nodes + 5 * (size_t)node;
        if (row[4] <= 4) {
            count += row[4];
        } else {
            push_children(a.aabbs, row[1], row[2], o, d, [&](int id, float2) {
                if (sp < kBvhStack) stack[sp++] = id;
            });
        }
        if (++visits > a.max_visits) break;  // only a malformed tree gets here
    }
    a.contrib[idx] = count;
}

// trace_bvh_cuda pass 2 (trace.cu:88-183): one record per leaf of those subtrees, in the
// reference's traversal order: the point's t along the ray (dot with the unnormalised
// direction), rejected (-1, t = 1e6) outside [max(0.01, box entry), box exit]
__global__ void __launch_bounds__(256) bvh_trace_emit_kernel(TraceListArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.n_rays || a.contrib[idx] == 0) return;
    const int base = idx == 0 ? 0 : a.offs[idx - 1];
    const float3 o = ld3(a.rays_o, idx), d = ld3(a.rays_d, idx);
    int stack[kBvhStack];
    float2 span[kBvhStack];
    int sp = 0;
    stack[sp] = 0;
    span[sp++] = make_float2(-1000.f, 1000.f);
    int count = 0, visits = 0;
    const int cap = a.contrib[idx];  // the count pass's total: never write past this ray's slots
    while (sp > 0 && count < cap) {
        --sp;
        const int node = stack[sp];
        const float2 in = span[sp];
        const int32_t* row = a.nodes + 5 * (size_t)node;
        if (row[4] <= 4) {
            int st2[8];  // a <= 4-leaf subtree has depth <= 3: at most 4 pending entries
            int sp2 = 0;
            st2[sp2++] = node;
            while (sp2 > 0 && sp2 <= 6 && count < cap) {
                const int n2 = st2[--sp2];
                const int32_t* r2 = a.nodes + 5 * (size_t)n2;
                if (r2[3] >= 0) {
                    int g = r2[3];
                    const float3 m = ld3(a.means, g);
                    float t = (m.x - o.x) * d.x + (m.y - o.y) * d.y + (m.z - o.z) * d.z;
                    if ((double)t < 0.01 || t < in.x || t > in.y) {
                        t = 1000000.f;
                        g = -1;
                    }
                    const int slot = base + count;
                    a.keys[slot] = ((uint64_t)(uint32_t)idx << 32) | __float_as_uint(t);
                    a.order[slot] = (uint32_t)slot;
                    a.point[slot] = g;
                    a.ray_id[slot] = idx;
                    a.position[3 * (size_t)slot] = o.x + t * d.x;
                    a.position[3 * (size_t)slot + 1] = o.y + t * d.y;
                    a.position[3 * (size_t)slot + 2] = o.z + t * d.z;
                    ++count;
                } else {
                    st2[sp2++] = r2[1];
                    st2[sp2++] = r2[2];
                }
            }
        } else {
            push_children(a.aabbs, row[1], row[2], o, d, [&](int id, float2 iv) {
                if (sp < kBvhStack) {
                    stack[sp] = id;
                    span[sp++] = iv;
                }
            });
        }
        if (++visits > a.max_visits) break;  // only a malformed tree gets here
    }
}

// the stable sort by (ray, t) permutes point and position (trace.cu:188-192); ray_id stays in
// emission order (the reference does not zip it into the sort; rays are contiguous, so it is
// unchanged by the permutation anyway)
__global__ void __launch_bounds__(256) bvh_trace_gather_kernel(int L, const uint32_t* __restrict__ order,
                                                               const int32_t* __restrict__ point_in,
                                                               const float* __restrict__ pos_in,
                                                               int32_t* __restrict__ point_out,
                                                               float* __restrict__ pos_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L) return;
    const uint32_t s = order[i];
    point_out[i] = point_in[s];
    pos_out[3 * (size_t)i] = pos_in[3 * (size_t)s];
    pos_out[3 * (size_t)i + 1] = pos_in[3 * (size_t)s + 1];
    pos_out[3 * (size_t)i + 2] = pos_in[3 * (size_t)s + 2];
}

inline unsigned blocks(long long n) { return (unsigned)((n + 255) / 256); }
inline size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

}  // namespace
}  // namespace r3dg

using namespace r3dg;

extern "C" int r3dg_bvh_leaf_aabbs(int P, const float* means3D, const float* scales, const float* rotations,
                                   float* leaf_aabbs, r3dg_stream_t stream) {
    R3DG_REQUIRE(P >= 0, "bvh_leaf_aabbs: negative P");
    if (P == 0) return R3DG_OK;
    R3DG_REQUIRE(means3D && scales && rotations && leaf_aabbs, "bvh_leaf_aabbs: null buffer");
    R3DG_REQUIRE(((uintptr_t)rotations & 15) == 0 && ((uintptr_t)leaf_aabbs & 7) == 0,
                 "bvh_leaf_aabbs: rotations must be 16-B and boxes 8-B aligned");
    hipLaunchKernelGGL(bvh_leaf_aabb_kernel, dim3(blocks(P)), dim3(256), 0, (hipStream_t)stream, P, means3D, scales,
                       rotations, leaf_aabbs);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}

extern "C" int r3dg_bvh_build(int P, int32_t* nodes, float* aabbs, uint64_t* morton, r3dg_alloc_fn scratch_alloc,
                              void* scratch_ctx, r3dg_stream_t stream) {
    R3DG_REQUIRE(P >= 1, "create_bvh: at least one Gaussian is required (the reference's 2P-1 nodes)");
    R3DG_REQUIRE(P < (1 << 30), "create_bvh: too many Gaussians");
    R3DG_REQUIRE(nodes && aabbs && morton && scratch_alloc, "create_bvh: null argument");
    R3DG_REQUIRE(((uintptr_t)aabbs & 7) == 0, "create_bvh: aabbs must be 8-B aligned");
    hipStream_t st = (hipStream_t)stream;
    const int n_int = P - 1;
    float* leaf = aabbs + 6 * (size_t)n_int;
    const int n_partial = (int)std::min<long long>(256, blocks(P));
    int n = 1;
    while (n < P) n <<= 1;
    size_t sort_bytes = 0;
    R3DG_CHECK_HIP(rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)P, 0, 30, st));
    const size_t b_partial = align256(24 * (size_t)n_partial), b_u32 = align256(4 * (size_t)P),
                 b_copy = align256(24 * (size_t)P), b_seg = align256(24 * (size_t)n);
    char* s = (char*)scratch_alloc(scratch_ctx, b_partial + 4 * b_u32 + b_copy + b_seg + align256(sort_bytes) + 256);
    R3DG_REQUIRE(s, "create_bvh: scratch allocation failed");
    s = (char*)(((uintptr_t)s + 255) & ~(uintptr_t)255);
    float* partial = (float*)s; s += b_partial;
    uint32_t* code = (uint32_t*)s; s += b_u32;
    uint32_t* index = (uint32_t*)s; s += b_u32;
    uint32_t* code_s = (uint32_t*)s; s += b_u32;
    uint32_t* index_s = (uint32_t*)s; s += b_u32;
    float* leaf_copy = (float*)s; s += b_copy;
    float* seg = (float*)s; s += b_seg;
    void* tmp = s;
    hipLaunchKernelGGL(bvh_bounds_partial_kernel, dim3(n_partial), dim3(256), 0, st, P, leaf, partial);
    R3DG_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(bvh_morton_kernel, dim3(blocks(P)), dim3(256), 0, st, P, n_partial, partial, leaf, code, index,
                       leaf_copy);
    R3DG_CHECK_HIP(hipGetLastError());
    // thrust::stable_sort_by_key (construct.cu:184-187): LSD radix sort is stable
    R3DG_CHECK_HIP(rocprim::radix_sort_pairs(tmp, sort_bytes, code, code_s, index, index_s, (size_t)P, 0, 30, st));
    hipLaunchKernelGGL(bvh_leaf_rows_kernel, dim3(blocks(P)), dim3(256), 0, st, P, code_s, index_s, leaf_copy, nodes,
                       aabbs, morton);
    R3DG_CHECK_HIP(hipGetLastError());
    if (n_int > 0) {
        for (int in_lo = n; in_lo > 1;) {
            const int cnt = in_lo < 256 ? in_lo : 256;
            hipLaunchKernelGGL(bvh_seg_level_kernel, dim3(in_lo / cnt), dim3(256), 0, st, P, n, in_lo, leaf, seg);
            R3DG_CHECK_HIP(hipGetLastError());
            in_lo /= cnt;
        }
        hipLaunchKernelGGL(bvh_internal_kernel, dim3(blocks(n_int)), dim3(256), 0, st, P, n, morton, nodes, seg,
                           aabbs);
        R3DG_CHECK_HIP(hipGetLastError());
    }
    return R3DG_OK;
}

extern "C" int r3dg_bvh_trace_opacity(int num_rays, int num_gaussians, const int32_t* nodes, const float* aabbs,
                                      const float* rays_o, const float* rays_d, const float* means3D,
                                      const float* cov3D_inv, const float* opacities, const float* normals,
                                      int32_t* num_contributes, float* rendered_opacity, r3dg_alloc_fn scratch_alloc,
                                      void* scratch_ctx, r3dg_stream_t stream) {
    R3DG_REQUIRE(num_rays >= 0, "trace_bvh_opacity: negative ray count");
    if (num_rays == 0) return R3DG_OK;
    R3DG_REQUIRE(num_gaussians >= 1, "trace_bvh_opacity: empty tree");
    R3DG_REQUIRE(nodes && aabbs && rays_o && rays_d && means3D && cov3D_inv && opacities && normals &&
                     num_contributes && rendered_opacity && scratch_alloc,
                 "trace_bvh_opacity: null buffer");
    R3DG_REQUIRE(((uintptr_t)aabbs & 7) == 0, "trace_bvh_opacity: aabbs must be 8-B aligned");
    hipStream_t st = (hipStream_t)stream;
    const int P = num_gaussians;
    const size_t b_n = align256(64 * (size_t)std::max(P - 1, 1)), b_g = align256(64 * (size_t)P);
    char* s = (char*)scratch_alloc(scratch_ctx, b_n + b_g + 256);
    R3DG_REQUIRE(s, "trace_bvh_opacity: scratch allocation failed");
    s = (char*)(((uintptr_t)s + 255) & ~(uintptr_t)255);
    float4* nrec = (float4*)s;
    float4* grec = (float4*)(s + b_n);
    hipLaunchKernelGGL(bvh_pack_kernel, dim3(blocks(P)), dim3(256), 0, st, P, nodes, aabbs, means3D, cov3D_inv,
                       opacities, normals, nrec, grec);
    R3DG_CHECK_HIP(hipGetLastError());
    // lanes per ray (one wave's group, shared LDS stack): measured on 1M-Gaussian scenes
    // (tools/gpu_bvh_lanes*.sh), 32 lanes is best or near-best from 100k to 1M rays (1M rays:
    // 24.2 / 14.2 / 13.2 / 10.5 / 9.2 / 8.8 / 10.6 ms at 1 / 2 / ... / 64 lanes, volume scene), 64
    // below ~32k rays; never more lanes than Gaussians. r3dg_options.test_bvh_lanes overrides (1, 2,
    // 4, ... 64)
    const r3dg_options opt = options();
    int g_bits = num_rays <= 32768 ? 6 : 5;
    while (g_bits > 0 && (1ll << g_bits) > P) --g_bits;
    if (opt.test_bvh_lanes > 0) {
        g_bits = 0;
        while (g_bits < 6 && (2 << g_bits) <= opt.test_bvh_lanes) ++g_bits;
    }
    TraceOpacityArgs a{num_rays, P == 1 ? 1 : 0, g_bits, nrec, grec, rays_o, rays_d, num_contributes,
                       rendered_opacity, 2 * (2 * P - 1), nullptr};
    // rays in Morton order of their origins, each XCD taking a contiguous range (independent rays:
    // the results do not depend on it). Measured 1-3 % at 1M rays (8.84 -> 8.73 ms volume, 30.8 ->
    // 29.9 ms surface), a loss at 10k (the sort costs more than the locality gains), so only for
    // >= 256k rays; test_bvh_sort = 1 / 2 forces it off / on
    const bool sort_rays = opt.test_bvh_sort ? opt.test_bvh_sort == 2 : num_rays >= 262144;
    if (P > 1 && sort_rays) {
        size_t sb = 0;
        R3DG_CHECK_HIP(rocprim::radix_sort_pairs(nullptr, sb, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                 (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)num_rays, 0, 30, st));
        const size_t b4 = align256(4 * (size_t)num_rays);
        char* r = (char*)scratch_alloc(scratch_ctx, 4 * b4 + align256(sb) + 256);
        R3DG_REQUIRE(r, "trace_bvh_opacity: scratch allocation failed");
        r = (char*)(((uintptr_t)r + 255) & ~(uintptr_t)255);
        uint32_t *code = (uint32_t*)r, *idx = (uint32_t*)(r + b4), *code_s = (uint32_t*)(r + 2 * b4),
                 *perm = (uint32_t*)(r + 3 * b4);
        hipLaunchKernelGGL(bvh_ray_morton_kernel, dim3(blocks(num_rays)), dim3(256), 0, st, num_rays, rays_o, aabbs,
                           code, idx);
        R3DG_CHECK_HIP(hipGetLastError());
        R3DG_CHECK_HIP(rocprim::radix_sort_pairs(r + 4 * b4, sb, code, code_s, idx, perm, (size_t)num_rays, 0, 30, st));
        a.perm = perm;
    }
    // G > 1: shared-stack groups (test_bvh_split: the static subtree split, for comparison)
    if (g_bits > 0 && !opt.test_bvh_split)
        hipLaunchKernelGGL(bvh_trace_opacity_shared_kernel, dim3(blocks((long long)num_rays << g_bits)), dim3(256), 0,
                           st, a);
    else
        hipLaunchKernelGGL(bvh_trace_opacity_kernel, dim3(blocks((long long)num_rays << g_bits)), dim3(256), 0, st, a);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}

extern "C" int r3dg_bvh_trace(int num_rays, int num_gaussians, const int32_t* nodes, const float* aabbs, const float* rays_o,
                              const float* rays_d, const float* means3D, int32_t* num_contributes,
                              r3dg_alloc_fn alloc, void* alloc_ctx, int* num_rendered, int32_t** point_list,
                              float** position_list, int32_t** ray_id_list, r3dg_stream_t stream) {
    R3DG_REQUIRE(num_rays >= 0, "trace_bvh: negative ray count");
    R3DG_REQUIRE(num_rendered && point_list && position_list && ray_id_list && alloc, "trace_bvh: null argument");
    *num_rendered = 0;
    *point_list = nullptr;
    *position_list = nullptr;
    *ray_id_list = nullptr;
    if (num_rays == 0) return R3DG_OK;
    R3DG_REQUIRE(num_gaussians >= 1, "trace_bvh: empty tree");
    R3DG_REQUIRE(nodes && aabbs && rays_o && rays_d && means3D && num_contributes, "trace_bvh: null buffer");
    R3DG_REQUIRE(((uintptr_t)aabbs & 7) == 0, "trace_bvh: aabbs must be 8-B aligned");
    hipStream_t st = (hipStream_t)stream;
    TraceListArgs a{};
    a.n_rays = num_rays; a.nodes = nodes; a.aabbs = aabbs; a.rays_o = rays_o; a.rays_d = rays_d; a.means = means3D;
    a.contrib = num_contributes;
    a.max_visits = 2 * (2 * num_gaussians - 1);
    size_t scan_bytes = 0;
    R3DG_CHECK_HIP(rocprim::inclusive_scan(nullptr, scan_bytes, (int32_t*)nullptr, (int32_t*)nullptr,
                                           (size_t)num_rays, rocprim::plus<int32_t>(), st));
    char* s = (char*)alloc(alloc_ctx, align256(4 * (size_t)num_rays) + align256(scan_bytes) + 256);
    R3DG_REQUIRE(s, "trace_bvh: scratch allocation failed");
    s = (char*)(((uintptr_t)s + 255) & ~(uintptr_t)255);
    int32_t* offs = (int32_t*)s;
    void* scan_tmp = s + align256(4 * (size_t)num_rays);
    hipLaunchKernelGGL(bvh_trace_count_kernel, dim3(blocks(num_rays)), dim3(256), 0, st, a);
    R3DG_CHECK_HIP(hipGetLastError());
    R3DG_CHECK_HIP(rocprim::inclusive_scan(scan_tmp, scan_bytes, num_contributes, offs, (size_t)num_rays,
                                           rocprim::plus<int32_t>(), st));
    int L = 0;  // the reference's blocking D2H of num_rendered (trace.cu:64-66)
    R3DG_CHECK_HIP(hipMemcpyAsync(&L, offs + num_rays - 1, sizeof(int), hipMemcpyDeviceToHost, st));
    R3DG_CHECK_HIP(hipStreamSynchronize(st));
    *num_rendered = L;
    if (L == 0) return R3DG_OK;
    int bits = 32;
    while (bits < 64 && ((uint64_t)(num_rays - 1) >> (bits - 32)) != 0) ++bits;
    size_t sort_bytes = 0;
    R3DG_CHECK_HIP(rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)L, 0, bits, st));
    const size_t nL = (size_t)L;
    char* w = (char*)alloc(alloc_ctx, 2 * align256(8 * nL) + 2 * align256(4 * nL) + align256(4 * nL) +
                                          align256(12 * nL) + align256(sort_bytes) + 256);
    int32_t* point = (int32_t*)alloc(alloc_ctx, 4 * nL);
    float* position = (float*)alloc(alloc_ctx, 12 * nL);
    int32_t* ray_id = (int32_t*)alloc(alloc_ctx, 4 * nL);
    R3DG_REQUIRE(w && point && position && ray_id, "trace_bvh: allocation failed");
    w = (char*)(((uintptr_t)w + 255) & ~(uintptr_t)255);
    uint64_t* keys = (uint64_t*)w; w += align256(8 * nL);
    uint64_t* keys_s = (uint64_t*)w; w += align256(8 * nL);
    uint32_t* order = (uint32_t*)w; w += align256(4 * nL);
    uint32_t* order_s = (uint32_t*)w; w += align256(4 * nL);
    int32_t* point_e = (int32_t*)w; w += align256(4 * nL);
    float* pos_e = (float*)w; w += align256(12 * nL);
    void* sort_tmp = w;
    a.offs = offs; a.keys = keys; a.order = order; a.point = point_e; a.position = pos_e; a.ray_id = ray_id;
    hipLaunchKernelGGL(bvh_trace_emit_kernel, dim3(blocks(num_rays)), dim3(256), 0, st, a);
    R3DG_CHECK_HIP(hipGetLastError());
    R3DG_CHECK_HIP(rocprim::radix_sort_pairs(sort_tmp, sort_bytes, keys, keys_s, order, order_s, nL, 0, bits, st));
    hipLaunchKernelGGL(bvh_trace_gather_kernel, dim3(blocks(L)), dim3(256), 0, st, L, order_s, point_e, pos_e, point,
                       position);
    R3DG_CHECK_HIP(hipGetLastError());
    *point_list = point;
    *position_list = position;
    *ray_id_list = ray_id;
    return R3DG_OK;
}
