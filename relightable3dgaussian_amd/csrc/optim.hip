// optim.hip -- the training step around the rasterizer on the device (gfx950): Adam over the flat
// parameter buffer, densification statistics, densify / prune and opacity reset.
//
// Restates reference scene/gaussian_model.py:581-620 (param groups, torch.optim.Adam step),
// :688-691 (reset_opacity), :822-1062 (prune_points, cat_tensors_to_optimizer,
// densification_postfix, densify_and_split, densify_and_clone, densify_and_prune, prune,
// add_densification_stats) and train.py:172-193.
//
// MI355X design: the reference issues one small torch op per attribute group and per step
// (7-14 groups x ~8 foreach ops, plus mask indexing and torch.cat of every group and both Adam
// states at densification). Here every group of a model lives in one flat fp32 buffer (layout in
// include/r3dg_hip.h), so:
//   * Adam is ONE HBM-streaming launch over [lo, hi) (28 B per float: p, g, m, v read; p, m, v
//     written), float4-vectorised, with the group's learning rate found per float4 from the
//     segment bounds -- which also makes the ZeRO-style shard [lo, hi) of a rank a plain range;
//   * densify / prune is a classification pass (clone / split / keep per Gaussian, both prune
//     tests), one rocPRIM scan of the four per-Gaussian counts, and one scatter pass that writes
//     every group and both Adam states of the new model -- instead of ~3 x 14 x 3 torch.cat /
//     index kernels.
#include <cmath>
#include <cstring>

#include "r3dg_common.h"
#include "r3dg_hip.h"

#include <rocprim/rocprim.hpp>

namespace r3dg {

// ---- Adam -------------------------------------------------------------------------------------

struct AdamArgs {
    float* param;           // global indexing
    const float* grad;      // shard-local
    float* m;
    float* v;
    long long lo, hi;
    int nseg;
    long long seg_end[R3DG_MAX_GROUPS];   // global end of each group
    float neg_step[R3DG_MAX_GROUPS];      // -(lr / (1 - b1^t)); t = the group's own step count
    float bc2_sqrt[R3DG_MAX_GROUPS];      // sqrt(1 - b2^t): torch divides sqrt(v) by it
    unsigned skip;                        // bit g: group g has no gradient this step (grad None)
    float omb1, beta2, omb2, eps;
};

__device__ __forceinline__ float adam_elem(const AdamArgs& a, float p, float g, float& m, float& v, float ns,
                                           float bc2_sqrt, bool skip) {
    // torch.optim.Adam leaves a parameter whose .grad is None untouched (p, m, v and its step)
    if (skip) return p;
    // torch._foreach_lerp_(exp_avgs, grads, 1 - beta1): weight < 0.5 -> self + w * (end - self)
    m = __builtin_fmaf(a.omb1, g - m, m);
    // _foreach_mul_(exp_avg_sqs, beta2); _foreach_addcmul_(exp_avg_sqs, grads, grads, 1 - beta2)
    v = v * a.beta2;
    v = __builtin_fmaf(a.omb2, g * g, v);
    // denom = sqrt(v) / bias_correction2_sqrt + eps; param += step_size * m / denom
    const float denom = sqrtf(v) / bc2_sqrt + a.eps;
    return __builtin_fmaf(ns, m / denom, p);
}

__global__ void __launch_bounds__(256) adam_kernel(AdamArgs a) {
    const long long n = a.hi - a.lo;
    const long long i4 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i4 >= n) return;
    const long long gi = a.lo + i4;
    // group of each of the 4 floats (segments are few; a float4 may straddle a boundary)
    float ns[4], bc[4];
    bool sk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        int s = 0;
        while (s < a.nseg - 1 && gi + e >= a.seg_end[s]) ++s;
        ns[e] = a.neg_step[s];
        bc[e] = a.bc2_sqrt[s];
        sk[e] = (a.skip >> s) & 1u;
    }
    const bool vec = i4 + 4 <= n && (((uintptr_t)(a.param + gi) | (uintptr_t)(a.grad + i4) |
                                      (uintptr_t)(a.m + i4) | (uintptr_t)(a.v + i4)) & 15) == 0;
    if (vec) {
        float4 p = *reinterpret_cast<const float4*>(a.param + gi);
        const float4 g = *reinterpret_cast<const float4*>(a.grad + i4);
        float4 m = *reinterpret_cast<const float4*>(a.m + i4);
        float4 v = *reinterpret_cast<const float4*>(a.v + i4);
        p.x = adam_elem(a, p.x, g.x, m.x, v.x, ns[0], bc[0], sk[0]);
        p.y = adam_elem(a, p.y, g.y, m.y, v.y, ns[1], bc[1], sk[1]);
        p.z = adam_elem(a, p.z, g.z, m.z, v.z, ns[2], bc[2], sk[2]);
        p.w = adam_elem(a, p.w, g.w, m.w, v.w, ns[3], bc[3], sk[3]);
        *reinterpret_cast<float4*>(a.param + gi) = p;
        *reinterpret_cast<float4*>(a.m + i4) = m;
        *reinterpret_cast<float4*>(a.v + i4) = v;
    } else {
        for (int e = 0; e < 4 && i4 + e < n; ++e) {
            float m = a.m[i4 + e], v = a.v[i4 + e];
            a.param[gi + e] = adam_elem(a, a.param[gi + e], a.grad[i4 + e], m, v, ns[e], bc[e], sk[e]);
            a.m[i4 + e] = m;
            a.v[i4 + e] = v;
        }
    }
}

static int check_layout(const r3dg_param_layout* L) {
    R3DG_REQUIRE(L && L->P >= 0 && L->n_groups > 0 && L->n_groups <= R3DG_MAX_GROUPS, "param layout: bad sizes");
    for (int g = 0; g < L->n_groups; ++g) R3DG_REQUIRE(L->width[g] > 0, "param layout: group width must be > 0");
    return R3DG_OK;
}

static long long layout_width(const r3dg_param_layout* L) {
    long long w = 0;
    for (int g = 0; g < L->n_groups; ++g) w += L->width[g];
    return w;
}

// ---- densification statistics (train.py:172-176, gaussian_model.py:1055-1062) ----------------

__global__ void __launch_bounds__(256) densification_stats_kernel(int P, const float* __restrict__ d2, int stride,
                                                                   const float* __restrict__ ngrad,
                                                                   const int* __restrict__ radii, float* xyz_accum,
                                                                   float* normal_accum, float* denom, float* max_r) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P || !(radii[i] > 0)) return;
    max_r[i] = fmaxf(max_r[i], (float)radii[i]);
    const float gx = d2[(size_t)i * stride], gy = d2[(size_t)i * stride + 1];
    xyz_accum[i] += sqrtf(gx * gx + gy * gy);
    if (ngrad) {
        // torch.nn.functional.normalize(x, dim=-1, eps=1e-3) = x / max(|x|, 1e-3), then its norm
        const float nx = ngrad[3 * (size_t)i], ny = ngrad[3 * (size_t)i + 1], nz = ngrad[3 * (size_t)i + 2];
        const float len = sqrtf(nx * nx + ny * ny + nz * nz);
        const float d = fmaxf(len, 1e-3f);
        const float ux = nx / d, uy = ny / d, uz = nz / d;
        normal_accum[i] += sqrtf(ux * ux + uy * uy + uz * uz);
    }
    denom[i] += 1.f;
}

// ---- densify / prune --------------------------------------------------------------------------

struct DensifyArgs {
    int P, n_groups;
    int width[R3DG_MAX_GROUPS];
    long long off[R3DG_MAX_GROUPS];      // group offsets in the source buffer (P * sum(width[<g]))
    long long noff[R3DG_MAX_GROUPS];     // group offsets in the new buffer
    int gxyz, gscale, grot, gopac;
    r3dg_densify_args d;
    const float* param;
    const float* m;
    const float* v;
    const float* xyz_accum;
    const float* normal_accum;
    const float* denom;
    const float* max_radii;
    uint4* codes;                        // per Gaussian: keep original, keep clone, keep children, split
    const uint4* pos;                    // exclusive scan of codes
    uint4 tot;                           // totals
    const float* noise;                  // [N * n_split, 3]
    float* out_param;
    float* out_m;
    float* out_v;
    int* out_source;                     // [P_new] source Gaussian of a kept original, -1 for new rows
};

__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float max_scale(const DensifyArgs& a, int i) {
    const float* s = a.param + a.off[a.gscale] + 3 * (size_t)i;
    return fmaxf(fmaxf(expf(s[0]), expf(s[1])), expf(s[2]));
}

// prune tests of a row with raw opacity `op` and activated max scale `ms`
// (densify_and_prune :1034-1040 / prune :1045-1050)
__device__ __forceinline__ bool pruned(const DensifyArgs& a, float op, float ms, float max_r) {
    bool p = sigmoidf(op) < a.d.min_opacity;
    if (a.d.max_screen_size > 0.f) p = p || (max_r > a.d.max_screen_size) || (ms > 0.1f * a.d.extent);
    return p;
}

__global__ void __launch_bounds__(256) densify_classify_kernel(DensifyArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.P) return;
    const float op = a.param[a.off[a.gopac] + i];
    const float ms = max_scale(a, i);
    bool clone = false, split = false;
    if (!a.d.prune_only) {
        // grads = accum / denom with NaN -> 0 (:1026-1029); torch.norm of a [P,1] row = |x|
        float g = a.xyz_accum[i] / a.denom[i], gn = a.normal_accum[i] / a.denom[i];
        if (g != g) g = 0.f;
        if (gn != gn) gn = 0.f;
        const bool sel = fabsf(g) >= a.d.grad_threshold || fabsf(gn) >= a.d.grad_normal_threshold;
        clone = sel && ms <= a.d.percent_dense * a.d.extent;  // :984-991
        split = sel && ms > a.d.percent_dense * a.d.extent;   // :928-938
    }
    // densify_and_prune's postfix zeroed max_radii2D before its prune test; `prune` reads it
    const float mr = (a.d.prune_only && a.max_radii) ? a.max_radii[i] : 0.f;
    const bool prune_o = pruned(a, op, ms, mr);
    bool prune_c = true;
    if (split) {
        // children: scaling_inverse_activation(get_scaling / (0.8 N)) then activated again (:945)
        const float* s = a.param + a.off[a.gscale] + 3 * (size_t)i;
        const float div = 0.8f * (float)a.d.N;
        float cm = 0.f;
        for (int k = 0; k < 3; ++k) cm = fmaxf(cm, expf(logf(expf(s[k]) / div)));
        prune_c = pruned(a, op, cm, 0.f);
    }
    a.codes[i] = make_uint4((!split && !prune_o) ? 1u : 0u, (clone && !prune_o) ? 1u : 0u,
                            (split && !prune_c) ? 1u : 0u, split ? 1u : 0u);
}

struct Uint4Plus {
    __device__ __host__ uint4 operator()(const uint4& x, const uint4& y) const {
        return make_uint4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
};

// build_rotation (utils/general_utils.py:82-103) of the normalised quaternion (r, x, y, z)
__device__ __forceinline__ void rotation_matrix(const float* q4, float R[3][3]) {
    const float n = sqrtf(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]);
    const float r = q4[0] / n, x = q4[1] / n, y = q4[2] / n, z = q4[3] / n;
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// One thread per (group, Gaussian, element) of the source buffer -- consecutive threads touch
// consecutive floats of a group, so every read and write is coalesced -- writes that float of
// the Gaussian's surviving rows: original, clone, and the N split children.
__global__ void __launch_bounds__(256) densify_scatter_kernel(DensifyArgs a, long long total) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    int g = 0;
    while (g < a.n_groups - 1 && t >= a.off[g + 1]) ++g;
    const int w = a.width[g];
    const long long local = t - a.off[g];
    const int i = (int)(local / w), e = (int)(local - (long long)i * w);
    const uint4 c = a.codes[i], p = a.pos[i];
    if (!(c.x | c.y | c.z)) return;
    const long long nO = a.tot.x, nC = a.tot.y, nS = a.tot.z, nSplit = a.tot.w;
    const float val = a.param[t];
    if (c.x) {
        const long long d = a.noff[g] + (long long)p.x * w + e;
        a.out_param[d] = val;
        a.out_m[d] = a.m[t];
        a.out_v[d] = a.v[t];
        if (a.out_source && g == 0 && e == 0) a.out_source[p.x] = i;
    }
    if (c.y) {  // clone (densify_and_clone :993-1023): copied values, zero Adam state
        const long long d = a.noff[g] + (nO + p.y) * w + e;
        a.out_param[d] = val;
        a.out_m[d] = 0.f;
        a.out_v[d] = 0.f;
        if (a.out_source && g == 0 && e == 0) a.out_source[nO + p.y] = -1;
    }
    if (!c.z) return;
    // split children (densify_and_split :940-954): xyz = R(q) (std * z) + xyz, scaling =
    // log(exp(s) / (0.8 N)), every other group copied; child k of split rank r takes noise row
    // k * nSplit + r (torch.normal over the .repeat(N, 1) stack)
    const float* sc = a.param + a.off[a.gscale] + 3 * (size_t)i;
    for (int k = 0; k < a.d.N; ++k) {
        const long long row = nO + nC + (long long)k * nS + p.z;
        float out = val;
        if (g == a.gxyz) {
            float R[3][3];
            rotation_matrix(a.param + a.off[a.grot] + 4 * (size_t)i, R);
            const float* z = a.noise + 3 * ((size_t)k * nSplit + p.w);
            float smp[3];
            for (int r = 0; r < 3; ++r) smp[r] = 0.f + expf(sc[r]) * z[r];
            out = R[e][0] * smp[0] + R[e][1] * smp[1] + R[e][2] * smp[2] + val;
        } else if (g == a.gscale) {
            out = logf(expf(val) / (0.8f * (float)a.d.N));
        }
        const long long d = a.noff[g] + row * w + e;
        a.out_param[d] = out;
        a.out_m[d] = 0.f;
        a.out_v[d] = 0.f;
        if (a.out_source && g == 0 && e == 0) a.out_source[row] = -1;
    }
}

__global__ void __launch_bounds__(256) reset_opacity_kernel(int P, float* op, float* m, float* v) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    // inverse_sigmoid(min(sigmoid(x), 0.01)) = log(y / (1 - y)) (utils/general_utils.py:17-18)
    const float y = fminf(sigmoidf(op[i]), 0.01f);
    op[i] = logf(y / (1.f - y));
    if (m) m[i] = 0.f;
    if (v) v[i] = 0.f;
}

}  // namespace r3dg

using namespace r3dg;

extern "C" int r3dg_adam_step_groups(const r3dg_param_layout* L, float* param, const float* grad, float* exp_avg,
                                     float* exp_avg_sq, int64_t lo, int64_t hi, const float* lr_host,
                                     const int* steps_host, double beta1, double beta2, double eps,
                                     r3dg_stream_t stream) {
    if (int e = check_layout(L)) return e;
    const long long total = (long long)L->P * layout_width(L);
    R3DG_REQUIRE(0 <= lo && lo <= hi && hi <= total, "adam_step: shard [lo, hi) outside the parameter buffer");
    R3DG_REQUIRE(lr_host && steps_host, "adam_step: lr and steps given");
    if (hi == lo) return R3DG_OK;
    R3DG_REQUIRE(param && grad && exp_avg && exp_avg_sq, "adam_step: null buffer");
    AdamArgs a{};
    a.param = param; a.grad = grad; a.m = exp_avg; a.v = exp_avg_sq; a.lo = lo; a.hi = hi;
    a.nseg = L->n_groups;
    long long end = 0;
    bool any = false;
    for (int g = 0; g < L->n_groups; ++g) {
        end += (long long)L->P * L->width[g];
        a.seg_end[g] = end;
        const int t = steps_host[g];
        if (t <= 0) {
            a.skip |= 1u << g;
            a.bc2_sqrt[g] = 1.f;
            continue;
        }
        any = true;
        const double bc1 = 1.0 - std::pow(beta1, (double)t), bc2 = 1.0 - std::pow(beta2, (double)t);
        a.neg_step[g] = (float)(-((double)lr_host[g] / bc1));
        a.bc2_sqrt[g] = (float)std::sqrt(bc2);
    }
    if (!any) return R3DG_OK;
    a.omb1 = (float)(1.0 - beta1); a.beta2 = (float)beta2; a.omb2 = (float)(1.0 - beta2); a.eps = (float)eps;
    const long long n4 = (hi - lo + 3) / 4;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}

extern "C" int r3dg_adam_step(const r3dg_param_layout* L, float* param, const float* grad, float* exp_avg,
                              float* exp_avg_sq, int64_t lo, int64_t hi, const float* lr_host, double beta1,
                              double beta2, double eps, int step, r3dg_stream_t stream) {
    if (int e = check_layout(L)) return e;
    R3DG_REQUIRE(step >= 1 && lr_host, "adam_step: step must be >= 1 and lr given");
    int steps[R3DG_MAX_GROUPS];
    for (int g = 0; g < L->n_groups; ++g) steps[g] = step;
    return r3dg_adam_step_groups(L, param, grad, exp_avg, exp_avg_sq, lo, hi, lr_host, steps, beta1, beta2, eps,
                                 stream);
}

extern "C" int r3dg_densification_stats(int P, const float* dL_dmeans2D, int stride2d, const float* normal_grad,
                                        const int* radii, float* xyz_accum, float* normal_accum, float* denom,
                                        float* max_radii2D, r3dg_stream_t stream) {
    R3DG_REQUIRE(P >= 0 && stride2d >= 2, "densification_stats: bad sizes");
    if (P == 0) return R3DG_OK;
    R3DG_REQUIRE(dL_dmeans2D && radii && xyz_accum && denom && max_radii2D && (normal_accum || !normal_grad),
                 "densification_stats: null buffer");
    hipLaunchKernelGGL(densification_stats_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, P,
                       dL_dmeans2D, stride2d, normal_grad, radii, xyz_accum, normal_accum, denom, max_radii2D);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}

extern "C" int r3dg_densify_and_prune(const r3dg_param_layout* L, const float* param, const float* exp_avg,
                                      const float* exp_avg_sq, const float* xyz_accum, const float* normal_accum,
                                      const float* denom, const float* max_radii2D, const r3dg_densify_args* args,
                                      r3dg_alloc_fn alloc, void* alloc_ctx, r3dg_alloc_fn randn, void* randn_ctx,
                                      float** out_param, float** out_exp_avg, float** out_exp_avg_sq,
                                      int** out_source, int* P_new, int* counts, r3dg_stream_t stream) {
    if (int e = check_layout(L)) return e;
    R3DG_REQUIRE(args && alloc && out_param && out_exp_avg && out_exp_avg_sq && P_new, "densify: null argument");
    R3DG_REQUIRE(args->prune_only || (args->N >= 1 && randn && xyz_accum && normal_accum && denom),
                 "densify: clone/split need N >= 1, the gradient statistics and a noise source");
    const int roles[4] = {L->xyz, L->scaling, L->rotation, L->opacity};
    const int need[4] = {3, 3, 4, 1};
    for (int k = 0; k < 4; ++k)
        R3DG_REQUIRE(roles[k] >= 0 && roles[k] < L->n_groups && L->width[roles[k]] == need[k],
                     "densify: xyz / scaling / rotation / opacity groups must have widths 3 / 3 / 4 / 1");
    hipStream_t st = (hipStream_t)stream;
    const int P = L->P;
    const long long W = layout_width(L);
    DensifyArgs a{};
    a.P = P; a.n_groups = L->n_groups;
    long long o = 0;
    for (int g = 0; g < L->n_groups; ++g) {
        a.width[g] = L->width[g];
        a.off[g] = o;
        o += (long long)P * L->width[g];
    }
    a.gxyz = L->xyz; a.gscale = L->scaling; a.grot = L->rotation; a.gopac = L->opacity;
    a.d = *args;
    a.param = param; a.m = exp_avg; a.v = exp_avg_sq;
    a.xyz_accum = xyz_accum; a.normal_accum = normal_accum; a.denom = denom; a.max_radii = max_radii2D;
    uint4 tot = make_uint4(0, 0, 0, 0);
    if (P > 0) {
        size_t scan_bytes = 0;
        R3DG_CHECK_HIP(rocprim::exclusive_scan(nullptr, scan_bytes, (uint4*)nullptr, (uint4*)nullptr,
                                               make_uint4(0, 0, 0, 0), (size_t)P, Uint4Plus(), st));
        char* scratch = (char*)alloc(alloc_ctx, 2 * sizeof(uint4) * (size_t)(P + 1) + scan_bytes + 256);
        R3DG_REQUIRE(scratch, "densify: scratch allocation failed");
        uint4* codes = reinterpret_cast<uint4*>(scratch);
        uint4* pos = codes + (P + 1);
        void* tmp = reinterpret_cast<void*>(((uintptr_t)(pos + (P + 1)) + 255) & ~(uintptr_t)255);
        a.codes = codes;
        hipLaunchKernelGGL(densify_classify_kernel, dim3((P + 255) / 256), dim3(256), 0, st, a);
        R3DG_CHECK_HIP(hipGetLastError());
        R3DG_CHECK_HIP(rocprim::exclusive_scan(tmp, scan_bytes, codes, pos, make_uint4(0, 0, 0, 0), (size_t)P,
                                               Uint4Plus(), st));
        uint4 last[2];
        R3DG_CHECK_HIP(hipMemcpyAsync(&last[0], pos + P - 1, sizeof(uint4), hipMemcpyDeviceToHost, st));
        R3DG_CHECK_HIP(hipMemcpyAsync(&last[1], codes + P - 1, sizeof(uint4), hipMemcpyDeviceToHost, st));
        R3DG_CHECK_HIP(hipStreamSynchronize(st));
        tot = Uint4Plus()(last[0], last[1]);
        a.pos = pos;
    }
    a.tot = tot;
    const long long Pn = (long long)tot.x + tot.y + (long long)args->N * tot.z;
    R3DG_REQUIRE(Pn < (1ll << 31), "densify: too many Gaussians");
    long long no = 0;
    for (int g = 0; g < L->n_groups; ++g) {
        a.noff[g] = no;
        no += Pn * L->width[g];
    }
    const size_t nbytes = sizeof(float) * (size_t)(Pn * W > 0 ? Pn * W : 1);
    a.out_param = (float*)alloc(alloc_ctx, nbytes);
    a.out_m = (float*)alloc(alloc_ctx, nbytes);
    a.out_v = (float*)alloc(alloc_ctx, nbytes);
    R3DG_REQUIRE(a.out_param && a.out_m && a.out_v, "densify: output allocation failed");
    if (out_source) {
        a.out_source = (int*)alloc(alloc_ctx, sizeof(int) * (size_t)(Pn > 0 ? Pn : 1));
        R3DG_REQUIRE(a.out_source, "densify: output allocation failed");
        *out_source = a.out_source;
    }
    if (tot.w > 0) {
        a.noise = (const float*)randn(randn_ctx, (size_t)3 * args->N * tot.w);
        R3DG_REQUIRE(a.noise, "densify: noise source failed");
    }
    if (P > 0) {
        const long long total = (long long)P * W;
        hipLaunchKernelGGL(densify_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a, total);
        R3DG_CHECK_HIP(hipGetLastError());
    }
    *out_param = a.out_param; *out_exp_avg = a.out_m; *out_exp_avg_sq = a.out_v;
    *P_new = (int)Pn;
    if (counts) {
        counts[0] = (int)tot.x; counts[1] = (int)tot.y; counts[2] = (int)tot.w; counts[3] = (int)tot.z;
    }
    return R3DG_OK;
}

extern "C" int r3dg_reset_opacity(const r3dg_param_layout* L, float* param, float* exp_avg, float* exp_avg_sq,
                                  r3dg_stream_t stream) {
    if (int e = check_layout(L)) return e;
    R3DG_REQUIRE(L->opacity >= 0 && L->opacity < L->n_groups && L->width[L->opacity] == 1,
                 "reset_opacity: the opacity group must have width 1");
    if (L->P == 0) return R3DG_OK;
    R3DG_REQUIRE(param, "reset_opacity: null buffer");
    long long off = 0;
    for (int g = 0; g < L->opacity; ++g) off += (long long)L->P * L->width[g];
    hipLaunchKernelGGL(reset_opacity_kernel, dim3((L->P + 255) / 256), dim3(256), 0, (hipStream_t)stream, L->P,
                       param + off, exp_avg ? exp_avg + off : nullptr, exp_avg_sq ? exp_avg_sq + off : nullptr);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}
