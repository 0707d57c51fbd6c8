// brdf.hip -- per-Gaussian render-equation integration (gfx950).
//
// Restates reference render_equation.cu: Fibonacci-hemisphere sampling rotated to the
// normal (:89-113), SH evaluation of incident / environment / visibility light (:17-50,
// :114-136), Lambert + SG-GGX specular (:138-161), the training forward (:552-663), the eval
// forward with per-sample outputs (:52-187) and the backward (:277-460).
//
// One thread per Gaussian loops over the samples, keeping the Gaussian's SH coefficients and
// all per-Gaussian gradient accumulators in registers; the environment SH (same for every
// Gaussian) is read through the scalar path. The backward is bug-compatible with the
// reference kernel (ReLU/clamp gradients never zeroed, dL_dn_d_i overwritten, no projection
// term for the half-vector normalisation, dL_dincidents_shs bounded by S_direct) EXCEPT the
// racy global `dL_ddirect_shs += ...` (render_equation.cu:443-445): here each block reduces its
// Gaussians' contributions and a second kernel sums the block partials in a fixed order.
#include "r3dg_common.h"
#include "r3dg_kernels.h"

namespace r3dg {

constexpr float kPi = 3.14159f;  // the reference's literal
constexpr float kInvPi = 1.0f / kPi;  // products in place of per-sample divisions by kPi (as the oracle)

__device__ __forceinline__ void sh_coef16(float x, float y, float z, float* coef) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    coef[0] = SH_C0;
    coef[1] = -SH_C1 * y; coef[2] = SH_C1 * z; coef[3] = -SH_C1 * x;
    coef[4] = SH_C2_0 * xy; coef[5] = SH_C2_1 * yz; coef[6] = SH_C2_2 * (2.0f * zz - xx - yy);
    coef[7] = SH_C2_3 * xz; coef[8] = SH_C2_4 * (xx - yy);
    coef[9] = SH_C3_0 * y * (3.0f * xx - yy); coef[10] = SH_C3_1 * xy * z;
    coef[11] = SH_C3_2 * y * (4.0f * zz - xx - yy); coef[12] = SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
    coef[13] = SH_C3_4 * x * (4.0f * zz - xx - yy); coef[14] = SH_C3_5 * z * (xx - yy);
    coef[15] = SH_C3_6 * x * (xx - 3.0f * yy);
}

__device__ __forceinline__ float3 fib_dir(float3 n, int ray, int Ns, float rot) {
    const float delta = kPi * (3.0f - sqrtf(5.0f));
    const float z = 1 - (float)ray * (2.0f / (2 * (float)Ns - 1));  // the quotient hoisted (oracle: same)
    const float rad = sqrtf(1 - z * z);
    const float theta = rot + delta * ray;
    float sn, cs;
    r3dg_sincosf(theta, &sn, &cs);  // bit-identical to the oracle's (r3dg_common.h)
    const float y = cs * rad, x = sn * rad;
    const float v1 = -n.y, v2 = n.x, v3 = 0.f;
    const float v11 = v1 * v1, v22 = v2 * v2, v33 = v3 * v3, v12 = v1 * v2, v13 = v1 * v3, v23 = v2 * v3;
    // the reference divides six times by cp1 and three times by norm (render_equation.cu:104-112);
    // here (and in the oracle) one IEEE division each and products with the reciprocal: within an
    // ulp of the quotients, 7 divisions (~10 VALU each) fewer per sample
    const float cp1 = fmaxf(n.z + 1, 0.0000001f), rc = 1.0f / cp1;
    const float ox = (1 + (-v33 - v22) * rc) * x + (-v3 + v12 * rc) * y + (v2 + v13 * rc) * z;
    const float oy = (v3 + v12 * rc) * x + (1 + (-v33 - v11) * rc) * y + (-v1 + v23 * rc) * z;
    const float oz = (-v2 + v13 * rc) * x + (v1 + v23 * rc) * y + (1 + (-v22 - v11) * rc) * z;
    const float norm = sqrtf(fmaxf(0.0000001f, ox * ox + oy * oy + oz * oz)), rn = 1.0f / norm;
    return make_float3(ox * rn, oy * rn, oz * rn);
}

struct Sample {
    float local[3], global[3], vis, light[3];
    float hdn, hdo, ndi, ndo, half_norm, half[3];
    float fd[3], fs[3], D, F[3], V;
    float e_amp;
};

struct GaussBRDF {
    float3 n, v, base;
    float rough, metal;
};

// SH light evaluation: coefficient arrays are either register arrays (NI/ND/NV > 0, the
// common S = 16 case) or read from memory with runtime bounds (NI = 0 generic path).
template <int NI, int ND, int NV>
__device__ __forceinline__ void eval_lights(const float* coef, const float* inc, int S_inc, const float* dir,
                                            int S_dir, const float* vis, int S_vis, Sample& s) {
    float lx = 0.f, ly = 0.f, lz = 0.f;
    if constexpr (NI > 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            lx = __builtin_fmaf(inc[3 * i], coef[i], lx);
            ly = __builtin_fmaf(inc[3 * i + 1], coef[i], ly);
            lz = __builtin_fmaf(inc[3 * i + 2], coef[i], lz);
        }
    } else {
        for (int i = 0; i < S_inc; ++i) {
            lx = __builtin_fmaf(inc[3 * i], coef[i], lx);
            ly = __builtin_fmaf(inc[3 * i + 1], coef[i], ly);
            lz = __builtin_fmaf(inc[3 * i + 2], coef[i], lz);
        }
    }
    s.local[0] = fmaxf(lx, 0.0f); s.local[1] = fmaxf(ly, 0.0f); s.local[2] = fmaxf(lz, 0.0f);
    float gx = 0.5f, gy = 0.5f, gz = 0.5f;
    if constexpr (ND > 0) {
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            gx = __builtin_fmaf(dir[3 * i], coef[i], gx);
            gy = __builtin_fmaf(dir[3 * i + 1], coef[i], gy);
            gz = __builtin_fmaf(dir[3 * i + 2], coef[i], gz);
        }
    } else {
        for (int i = 0; i < S_dir; ++i) {
            gx = __builtin_fmaf(dir[3 * i], coef[i], gx);
            gy = __builtin_fmaf(dir[3 * i + 1], coef[i], gy);
            gz = __builtin_fmaf(dir[3 * i + 2], coef[i], gz);
        }
    }
    s.global[0] = fmaxf(gx, 0.0f); s.global[1] = fmaxf(gy, 0.0f); s.global[2] = fmaxf(gz, 0.0f);
    float vv = 0.5f;
    if constexpr (NV > 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) vv = __builtin_fmaf(vis[i], coef[i], vv);
    } else {
        for (int i = 0; i < S_vis; ++i) vv = __builtin_fmaf(vis[i], coef[i], vv);
    }
    s.vis = fmaxf(0.0f, fminf(vv, 1.0f));
#pragma unroll
    for (int c = 0; c < 3; ++c) s.light[c] = __builtin_fmaf(s.vis, s.global[c], s.local[c]);
}

// The SH light sums (render_equation.cu:118-136), their backward accumulations (:436-452) and the
// light composition are explicit fmaf chains in sample / coefficient order, as the oracle's (what
// nvcc's default contraction makes of the reference's `+= a * b` loops, and one instruction each).
// render_equation.cu:138-161 for one sample, with the per-Gaussian terms (amp, sharp, r2v, the
// view-side GGX factor g2 = 0.5 / denom2) hoisted by the caller -- the same IEEE operations in the
// same order as the oracle's brdf_eval (true divisions, FP contraction off for this file), so D,
// F, V and f_d / f_s are bit-identical to it. The reference's transcendentals (expf, powf; their
// bits are CUDA-implementation-defined) are stated once for both: r3dg_expf_wide, and powf(t, 5)
// as the products (t^2)^2 t.
__device__ __forceinline__ void eval_brdf(const GaussBRDF& G, float3 d, float amp, float sharp, float r2v, float g2,
                                          Sample& s) {
    const float hx = d.x + G.v.x, hy = d.y + G.v.y, hz = d.z + G.v.z;
    s.half_norm = fmaxf(sqrtf(hx * hx + hy * hy + hz * hz), 0.0000001f);
    const float rh = 1.0f / s.half_norm;  // one division, three products (as the oracle)
    s.half[0] = hx * rh; s.half[1] = hy * rh; s.half[2] = hz * rh;
    s.hdn = fmaxf(s.half[0] * G.n.x + s.half[1] * G.n.y + s.half[2] * G.n.z, 0.0f);
    s.hdo = fmaxf(s.half[0] * G.v.x + s.half[1] * G.v.y + s.half[2] * G.v.z, 0.0f);
    s.ndi = fmaxf(G.n.x * d.x + G.n.y * d.y + G.n.z * d.z, 0.0f);
    s.ndo = fmaxf(G.n.x * G.v.x + G.n.y * G.v.y + G.n.z * G.v.z, 0.0f);
    const float base[3] = {G.base.x, G.base.y, G.base.z};
    s.e_amp = r3dg_expf_wide(sharp * (s.hdn - 1.0f));
    s.D = amp * s.e_amp;
    const float t1 = 1.0f - s.hdo, t2 = t1 * t1, p5 = t2 * t2 * t1;
    s.V = (0.5f / fmaxf(s.ndi * (1 - r2v) + r2v, 0.0000001f)) * g2;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        s.fd[c] = (1 - G.metal) * base[c] / kPi;
        const float F0 = 0.04f * (1.0f - G.metal) + base[c] * G.metal;
        s.F[c] = F0 + (1.0f - F0) * p5;
        s.fs[c] = s.D * s.F[c] * s.V;
    }
}

struct BrdfKArgs {
    r3dg_brdf_inputs in;
    int is_training;
    const float* rand_float;
    // training forward outputs
    float* pbr;
    float* incident_dirs;
    float* diffuse;
    // complex outputs
    r3dg_brdf_complex_outputs cx;
    // backward
    const float* dirs_in;
    const float* dL_dpbr;
    const float* dL_ddiff;
    r3dg_brdf_grads gr;
    float* dir_partials;  // [gridDim.x, S_direct*3]
};

template <int NI, int ND, int NV>
__device__ __forceinline__ void load_gauss(const r3dg_brdf_inputs& in, int idx, GaussBRDF& G, float* inc, float* vis) {
    G.n = make_float3(in.normals[3 * idx], in.normals[3 * idx + 1], in.normals[3 * idx + 2]);
    G.v = make_float3(in.viewdirs[3 * idx], in.viewdirs[3 * idx + 1], in.viewdirs[3 * idx + 2]);
    G.base = make_float3(in.base_color[3 * idx], in.base_color[3 * idx + 1], in.base_color[3 * idx + 2]);
    G.rough = in.roughness[idx];
    G.metal = in.metallic[idx];
    if constexpr (NI > 0) {
#pragma unroll
        for (int i = 0; i < 3 * NI; ++i) inc[i] = in.incidents_shs[(size_t)idx * 3 * NI + i];
    }
    if constexpr (NV > 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) vis[i] = in.visibility_shs[(size_t)idx * NV + i];
    }
}

// render_equation.cu:552-663 (training forward) and :52-187 (complex) share this kernel.
template <int NI, int ND, int NV, bool COMPLEX>
__global__ void __launch_bounds__(256) brdf_fwd_kernel(BrdfKArgs a) {
    const r3dg_brdf_inputs& in = a.in;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= in.P) return;
    GaussBRDF G;
    float inc_r[NI > 0 ? 3 * NI : 1], vis_r[NV > 0 ? NV : 1];
    load_gauss<NI, ND, NV>(in, idx, G, inc_r, vis_r);
    const float* inc_g = in.incidents_shs + (size_t)idx * 3 * in.S_incident;
    const float* vis_g = in.visibility_shs + (size_t)idx * in.S_visibility;
    const int Ns = in.sample_num;
    float pbr[3] = {0.f, 0.f, 0.f}, dl[3] = {0.f, 0.f, 0.f}, ldl[3] = {0.f, 0.f, 0.f};
    float rd[3] = {0.f, 0.f, 0.f}, rs[3] = {0.f, 0.f, 0.f};
    // per-Gaussian BRDF terms (eval_brdf_fast)
    const float r2 = fmaxf(G.rough * G.rough, 0.0000001f);
    const float amp = 1.0f / (r2 * kPi), sharp = 2.0f / r2;
    const float r2v = (1.0f + G.rough) * (1.0f + G.rough) / 8.0f;
    const float ndo = fmaxf(G.n.x * G.v.x + G.n.y * G.v.y + G.n.z * G.v.z, 0.0f);
    const float g2 = 0.5f / fmaxf(ndo * (1 - r2v) + r2v, 0.0000001f);
    const bool rnd = !COMPLEX && a.is_training;
    float rnext = rnd && Ns > 0 ? a.rand_float[(size_t)idx * Ns] : 0.f;  // one sample ahead
    for (int r = 0; r < Ns; ++r) {
        const size_t w = (size_t)idx * Ns + r;
        float rot = 0.f;
        if (rnd) {
            rot = rnext * 2 * kPi;
            if (r + 1 < Ns) rnext = a.rand_float[w + 1];
        }
        const float3 d = fib_dir(G.n, r, Ns, rot);
        float coef[16];
        sh_coef16(d.x, d.y, d.z, coef);
        Sample s;
        if constexpr (NI > 0)
            eval_lights<NI, ND, NV>(coef, inc_r, NI, in.direct_shs, ND, vis_r, NV, s);
        else
            eval_lights<0, 0, 0>(coef, inc_g, in.S_incident, in.direct_shs, in.S_direct, vis_g, in.S_visibility, s);
        eval_brdf(G, d, amp, sharp, r2v, g2, s);
        const float tmp = s.ndi * (2.0f * kPi / (float)Ns);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float tr = s.light[c] * tmp;
            if constexpr (COMPLEX) {
                dl[c] += tr;
                ldl[c] += s.local[c] * tmp;
                rd[c] += s.fd[c] * tr;
                rs[c] += s.fs[c] * tr;
            } else {
                pbr[c] += (s.fd[c] + s.fs[c]) * tr;
                dl[c] += tr;
            }
        }
        if constexpr (COMPLEX) {
            const r3dg_brdf_complex_outputs& o = a.cx;
            o.incident_dirs[3 * w] = d.x; o.incident_dirs[3 * w + 1] = d.y; o.incident_dirs[3 * w + 2] = d.z;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                o.incident_lights[3 * w + c] = s.light[c];
                o.local_incident_lights[3 * w + c] = s.local[c];
                o.global_incident_lights[3 * w + c] = s.vis * s.global[c];
            }
            o.incident_visibility[w] = s.vis;
        } else {
            a.incident_dirs[3 * w] = d.x; a.incident_dirs[3 * w + 1] = d.y; a.incident_dirs[3 * w + 2] = d.z;
        }
    }
    if constexpr (COMPLEX) {
        const r3dg_brdf_complex_outputs& o = a.cx;
        float av[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) av[c] = dl[c] * kInvPi + rs[c];
        o.accum[idx] = (av[0] + av[1] + av[2]) / 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            o.pbr[3 * idx + c] = rd[c] + rs[c];
            o.rgb_d[3 * idx + c] = rd[c];
            o.rgb_s[3 * idx + c] = rs[c];
            o.diffuse_light[3 * idx + c] = dl[c];
            o.local_diffuse_light[3 * idx + c] = ldl[c];
        }
    } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            a.pbr[3 * idx + c] = pbr[c];
            a.diffuse[3 * idx + c] = dl[c];
        }
    }
}

// render_equation.cu:277-460 (bug-compatible, see header); S <= 16 is checked on the host. One
// thread per Gaussian, samples in the reference's order, the Gaussian's SH coefficients and all
// 112 SH-gradient accumulators in registers (one wave per SIMD: 256 VGPR + ~50 AGPR). Measured
// alternatives, all slower at P = 1M: the coefficients staged in LDS at 2 waves/SIMD (spills;
// 3.9 ms incl. the old reducer), 2 waves/SIMD with registers only (spills, 3.3 ms), the sample
// loop unrolled by 2 / 3 (accumulators move to AGPRs), the environment SH re-read through the
// scalar cache each sample (R3DG_BRDF_ENV_RELOAD: no SGPR spills but exposed latency, +0.27 ms).
// What paid: the next sample's direction loaded one iteration ahead, per-Gaussian BRDF terms
// hoisted (eval_brdf_fast), reciprocal multiplications instead of divisions, products instead of
// powf, compile-time loop bounds in the S = 16 specialisation (1051 -> 514 VALU per sample), and
// a parallel env-gradient reducer (brdf_dir_reduce_kernel): 2.33 -> 0.58 ms in all.
#ifndef R3DG_BRDF_REG_WAVES
#define R3DG_BRDF_REG_WAVES 1
#endif
template <int NI, int ND, int NV>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R3DG_BRDF_REG_WAVES)))
brdf_bwd_kernel(BrdfKArgs a) {
    constexpr int NDA = 16;  // register accumulators for dL_ddirect_shs (S_direct <= 16)
    const r3dg_brdf_inputs& in = a.in;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = idx < in.P;
    const int S_dir = ND > 0 ? ND : in.S_direct;  // compile-time bounds in the S = 16 specialisation
    float ddir[3 * NDA];
#pragma unroll
    for (int i = 0; i < 3 * NDA; ++i) ddir[i] = 0.f;
    if (valid) {
        GaussBRDF G;
        float inc_r[NI > 0 ? 3 * NI : 1], vis_r[NV > 0 ? NV : 1];
        load_gauss<NI, ND, NV>(in, idx, G, inc_r, vis_r);
        const float* inc_g = in.incidents_shs + (size_t)idx * 3 * in.S_incident;
        const float* vis_g = in.visibility_shs + (size_t)idx * in.S_visibility;
        const int Ns = in.sample_num;
        const float gp[3] = {a.dL_dpbr[3 * idx], a.dL_dpbr[3 * idx + 1], a.dL_dpbr[3 * idx + 2]};
        const float gdl[3] = {a.dL_ddiff[3 * idx], a.dL_ddiff[3 * idx + 1], a.dL_ddiff[3 * idx + 2]};
        const float n[3] = {G.n.x, G.n.y, G.n.z}, v[3] = {G.v.x, G.v.y, G.v.z};
        const float b[3] = {G.base.x, G.base.y, G.base.z};
        float dinc_r[NI > 0 ? 3 * NI : 1], dvis_r[NV > 0 ? NV : 1];
#pragma unroll
        for (int i = 0; i < (NI > 0 ? 3 * NI : 1); ++i) dinc_r[i] = 0.f;
#pragma unroll
        for (int i = 0; i < (NV > 0 ? NV : 1); ++i) dvis_r[i] = 0.f;
        float* dinc_g = a.gr.dL_dincidents_shs + (size_t)idx * 3 * in.S_incident;
        float* dvis_g = a.gr.dL_dvisibility_shs + (size_t)idx * in.S_visibility;
        if (NI == 0) for (int i = 0; i < 3 * in.S_incident; ++i) dinc_g[i] = 0.f;
        if (NV == 0) for (int i = 0; i < in.S_visibility; ++i) dvis_g[i] = 0.f;
        float dbase_acc[3] = {0.f, 0.f, 0.f}, dn_acc[3] = {0.f, 0.f, 0.f}, dv_acc[3] = {0.f, 0.f, 0.f};
        float dmetal_acc = 0.f, drough_acc = 0.f;
        const int n_inc_upd = min(S_dir, NI > 0 ? NI : in.S_incident);  // reference loop bound is S_direct (:450)
        const float rough = G.rough, metal = G.metal;
        const float r2 = fmaxf(rough * rough, 0.0000001f);
        const float amp = 1.0f / (r2 * kPi), sharp = 2.0f / r2;
        const float r2v = (1.0f + rough) * (1.0f + rough) / 8.0f;
        const float ndo = fmaxf(G.n.x * G.v.x + G.n.y * G.v.y + G.n.z * G.v.z, 0.0f);
        const float den2 = fmaxf(ndo * (1 - r2v) + r2v, 0.0000001f);
        const float g2 = 0.5f / den2;
        const float* dirs = a.dirs_in + (size_t)idx * Ns * 3;
        float dn0 = Ns > 0 ? dirs[0] : 0.f, dn1 = Ns > 0 ? dirs[1] : 0.f, dn2 = Ns > 0 ? dirs[2] : 0.f;
#pragma unroll 1  // unrolling by 2 / 3 measured slower (accumulators move to AGPRs)
        for (int r = 0; r < Ns; ++r) {
            const float3 d = make_float3(dn0, dn1, dn2);
            if (r + 1 < Ns) {  // next sample's direction one iteration ahead
                dn0 = dirs[3 * r + 3];
                dn1 = dirs[3 * r + 4];
                dn2 = dirs[3 * r + 5];
            }
            const float dd[3] = {d.x, d.y, d.z};
            float coef[16];
            sh_coef16(d.x, d.y, d.z, coef);
            Sample s;
            // R3DG_BRDF_ENV_RELOAD: the environment SH pointer laundered per sample, so its 48
            // values are re-read through the scalar cache instead of held in SGPRs (no SGPR spills,
            // but the reloads' latency shows at one wave per SIMD: measured slower)
            const float* env = in.direct_shs;
#ifdef R3DG_BRDF_ENV_RELOAD
            asm volatile("" : "+s"(env));
#endif
            if constexpr (NI > 0)
                eval_lights<NI, ND, NV>(coef, inc_r, NI, env, ND, vis_r, NV, s);
            else
                eval_lights<0, 0, 0>(coef, inc_g, in.S_incident, env, S_dir, vis_g, in.S_visibility, s);
            eval_brdf(G, d, amp, sharp, r2v, g2, s);
            const float e_amp = s.e_amp;
            const float den1 = fmaxf(s.ndi * (1 - r2v) + r2v, 0.0000001f);
            const float g1 = 0.5f / den1;
            const float Tn = s.ndi * (2.0f * kPi / (float)Ns);
            float dfd[3], dfs[3], dli[3], fsum[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                fsum[c] = s.fd[c] + s.fs[c];
                dfd[c] = gp[c] * s.light[c] * Tn;
                dfs[c] = gp[c] * s.light[c] * Tn;
                dli[c] = gp[c] * fsum[c] * Tn;
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) dli[c] += gdl[c] * Tn;
            // dL_dn_d_i of :372 / :376 is overwritten at :403 before any use (bug-compatible): not formed
            float dbase[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) dbase[c] = dfd[c] * ((1 - metal) / kPi);
            float dmetal = -(dfd[0] * b[0] + dfd[1] * b[1] + dfd[2] * b[2]) * kInvPi;
            const float dD = dfs[0] * s.V * s.F[0] + dfs[1] * s.V * s.F[1] + dfs[2] * s.V * s.F[2];
            float dF[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) dF[c] = dfs[c] * s.D * s.V;
            const float dV = dfs[0] * s.D * s.F[0] + dfs[1] * s.D * s.F[1] + dfs[2] * s.D * s.F[2];
            const float damp = dD * e_amp, de = dD * amp;
            const float dsharp = (s.hdn - 1.0f) * e_amp * de;
            const float dhdn = sharp * e_amp * de;
            const float dr2 = -2.0f / (r2 * r2) * dsharp - 1.0f / (r2 * r2 * kPi) * damp;
            float drough = dr2 * 2.0f * rough;
            const float t1 = 1.0f - s.hdo, t2 = t1 * t1, p4 = t2 * t2, p5 = p4 * t1;
            float dF0[3], dhdo = 0.f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float F0 = 0.04f * (1.0f - metal) + b[c] * metal;
                dF0[c] = (1.0f - p5) * dF[c];
                dhdo += (1.0f - F0) * dF[c];
            }
            dhdo = dhdo * -5.0f * p4;
#pragma unroll
            for (int c = 0; c < 3; ++c) dbase[c] += metal * dF0[c];
            dmetal += (b[0] - 0.04f) * dF0[0] + (b[1] - 0.04f) * dF0[1] + (b[2] - 0.04f) * dF0[2];
            const float dg1 = dV * g2, dg2 = dV * g1;
            // -0.5 / den1^2 = -2 g1^2 (one division per sample fewer; oracle: same)
            const float dden1 = -2.0f * (g1 * g1) * dg1, dden2 = -0.5f / (den2 * den2) * dg2;
            const float dndi2 = dden1 * (1 - r2v);
            const float dndo = dden2 * (1 - r2v);
            const float dr2v = (1.0f - s.ndi) * dden1 + (1.0f - s.ndo) * dden2;
            drough += (1.0f + rough) / 4.0f * dr2v;
            float dhalf[3] = {0.f, 0.f, 0.f}, dn[3] = {0.f, 0.f, 0.f}, dv[3] = {0.f, 0.f, 0.f};
            if (s.hdn > 0.0f) {
#pragma unroll
                for (int c = 0; c < 3; ++c) { dhalf[c] += n[c] * dhdn; dn[c] += s.half[c] * dhdn; }
            }
            if (s.hdo > 0.0f) {
#pragma unroll
                for (int c = 0; c < 3; ++c) { dhalf[c] += v[c] * dhdo; dv[c] += s.half[c] * dhdo; }
            }
            if (s.ndi > 0.0f) {
#pragma unroll
                for (int c = 0; c < 3; ++c) dn[c] += dd[c] * dndi2;
            }
            if (s.ndo > 0.0f) {
#pragma unroll
                for (int c = 0; c < 3; ++c) { dn[c] += v[c] * dndo; dv[c] += n[c] * dndo; }
            }
            const float rh = 1.0f / s.half_norm;
#pragma unroll
            for (int c = 0; c < 3; ++c) dv[c] += dhalf[c] * rh;
            float dglob[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) dglob[c] = dli[c] * s.vis;
            const float dvis_s = dli[0] * s.global[0] + dli[1] * s.global[1] + dli[2] * s.global[2];
            if constexpr (NV > 0) {
#pragma unroll
                for (int i = 0; i < NV; ++i) dvis_r[i] = __builtin_fmaf(dvis_s, coef[i], dvis_r[i]);
            } else {
                for (int i = 0; i < in.S_visibility; ++i) dvis_g[i] = __builtin_fmaf(dvis_s, coef[i], dvis_g[i]);
            }
#pragma unroll
            for (int i = 0; i < NDA; ++i)
                if (i < S_dir) {
                    ddir[3 * i] = __builtin_fmaf(dglob[0], coef[i], ddir[3 * i]);
                    ddir[3 * i + 1] = __builtin_fmaf(dglob[1], coef[i], ddir[3 * i + 1]);
                    ddir[3 * i + 2] = __builtin_fmaf(dglob[2], coef[i], ddir[3 * i + 2]);
                }
            if constexpr (NI > 0) {
#pragma unroll
                for (int i = 0; i < NI; ++i)
                    if (i < n_inc_upd) {
                        dinc_r[3 * i] = __builtin_fmaf(dli[0], coef[i], dinc_r[3 * i]);
                        dinc_r[3 * i + 1] = __builtin_fmaf(dli[1], coef[i], dinc_r[3 * i + 1]);
                        dinc_r[3 * i + 2] = __builtin_fmaf(dli[2], coef[i], dinc_r[3 * i + 2]);
                    }
            } else {
                for (int i = 0; i < n_inc_upd; ++i)
                    for (int c = 0; c < 3; ++c) dinc_g[3 * i + c] = __builtin_fmaf(dli[c], coef[i], dinc_g[3 * i + c]);
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                dv_acc[c] += dv[c];
                dn_acc[c] += dn[c];
                dbase_acc[c] += dbase[c];
            }
            dmetal_acc += dmetal;
            drough_acc += drough;
        }
        if constexpr (NI > 0) {
#pragma unroll
            for (int i = 0; i < 3 * NI; ++i) dinc_g[i] = dinc_r[i];
        }
        if constexpr (NV > 0) {
#pragma unroll
            for (int i = 0; i < NV; ++i) dvis_g[i] = dvis_r[i];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            a.gr.dL_dbase_color[3 * idx + c] = dbase_acc[c];
            a.gr.dL_dnormals[3 * idx + c] = dn_acc[c];
            a.gr.dL_dviewdirs[3 * idx + c] = dv_acc[c];
        }
        a.gr.dL_dmetallic[idx] = dmetal_acc;
        a.gr.dL_droughness[idx] = drough_acc;
    }
    // deterministic block partial of dL_ddirect_shs
    __shared__ float s_part[4][3 * NDA];
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 3 * NDA; ++i) {
        const float sum = wave_sum_to_lane63(ddir[i]);
        if (l == 63) s_part[wv][i] = sum;
    }
    __syncthreads();
    if (threadIdx.x < 3 * NDA) {
        const int i = threadIdx.x;
        a.dir_partials[(size_t)blockIdx.x * 3 * NDA + i] = ((s_part[0][i] + s_part[1][i]) + s_part[2][i]) + s_part[3][i];
    }
}

// Sum of the block partials of dL_ddirect_shs: one workgroup per output, a strided per-thread sum
// (fixed order) then a fixed-shape tree over the workgroup -- deterministic. (The first version
// ran one thread per output over all block partials in sequence: 1.27 ms at P = 1M, more than
// the backward kernel itself.)
__global__ void __launch_bounds__(256) brdf_dir_reduce_kernel(const float* partials, int nblocks, int n, float* out) {
    const int i = blockIdx.x, t = threadIdx.x;
    if (i >= n) return;  // workgroup-uniform
    float s = 0.f;
    for (int b = t; b < nblocks; b += 256) s += partials[(size_t)b * 48 + i];
    __shared__ float s_red[256];
    s_red[t] = s;
    __syncthreads();
#pragma unroll
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) s_red[t] += s_red[t + h];
        __syncthreads();
    }
    if (t == 0) out[i] = s_red[0];
}

// Lane-per-sample forward (render_equation.cu:552-663 training / :52-187 complex): a workgroup
// of 256 lanes holds GB = 256 / Ns whole Gaussians, lane t = (Gaussian t / Ns, sample t % Ns).
// A lane's per-sample outputs sit at w = g * Ns + r = g0 * Ns + t, so every per-sample store of
// the workgroup is one contiguous span (the thread-per-Gaussian kernel stores at a 288-byte lane
// stride, Ns * 3 floats, and spent most of its time there). The per-Gaussian sums over the
// samples run in the reference's order (r = 0, 1, ...) from an LDS column per output channel, so
// they are the thread-per-Gaussian kernel's sums bit for bit.
template <int NI, int ND, int NV, bool COMPLEX>
__global__ void __launch_bounds__(256) brdf_fwd_lane_kernel(BrdfKArgs a, int GB) {
    constexpr int NC = COMPLEX ? 12 : 6;  // per-Gaussian sums: complex dl ldl rd rs, else pbr dl
    __shared__ float s_c[256 * (NC + 1)];
    __shared__ float s_sum[256][NC];
    const r3dg_brdf_inputs& in = a.in;
    const int Ns = in.sample_num;
    const int t = threadIdx.x;
    const int gl = t / Ns, r = t - gl * Ns;
    const int g0 = blockIdx.x * GB;
    const int ng = min(GB, in.P - g0);
    const bool active = gl < ng;
    float c[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) c[k] = 0.f;
    if (active) {
        const int idx = g0 + gl;
        GaussBRDF G;
        float inc_r[NI > 0 ? 3 * NI : 1], vis_r[NV > 0 ? NV : 1];
        load_gauss<NI, ND, NV>(in, idx, G, inc_r, vis_r);
        const float* inc_g = in.incidents_shs + (size_t)idx * 3 * in.S_incident;
        const float* vis_g = in.visibility_shs + (size_t)idx * in.S_visibility;
        const float r2 = fmaxf(G.rough * G.rough, 0.0000001f);
        const float amp = 1.0f / (r2 * kPi), sharp = 2.0f / r2;
        const float r2v = (1.0f + G.rough) * (1.0f + G.rough) / 8.0f;
        const float ndo = fmaxf(G.n.x * G.v.x + G.n.y * G.v.y + G.n.z * G.v.z, 0.0f);
        const float g2 = 0.5f / fmaxf(ndo * (1 - r2v) + r2v, 0.0000001f);
        const size_t w = (size_t)idx * Ns + r;
        float rot = 0.f;
        if (!COMPLEX && a.is_training) rot = a.rand_float[w] * 2 * kPi;
        const float3 d = fib_dir(G.n, r, Ns, rot);
        float coef[16];
        sh_coef16(d.x, d.y, d.z, coef);
        Sample s;
        if constexpr (NI > 0)
            eval_lights<NI, ND, NV>(coef, inc_r, NI, in.direct_shs, ND, vis_r, NV, s);
        else
            eval_lights<0, 0, 0>(coef, inc_g, in.S_incident, in.direct_shs, in.S_direct, vis_g, in.S_visibility, s);
        eval_brdf(G, d, amp, sharp, r2v, g2, s);
        const float tmp = s.ndi * (2.0f * kPi / (float)Ns);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float tr = s.light[k] * tmp;
            if constexpr (COMPLEX) {
                c[k] = tr;
                c[3 + k] = s.local[k] * tmp;
                c[6 + k] = s.fd[k] * tr;
                c[9 + k] = s.fs[k] * tr;
            } else {
                c[k] = (s.fd[k] + s.fs[k]) * tr;
                c[3 + k] = tr;
            }
        }
        if constexpr (COMPLEX) {
            const r3dg_brdf_complex_outputs& o = a.cx;
            o.incident_dirs[3 * w] = d.x; o.incident_dirs[3 * w + 1] = d.y; o.incident_dirs[3 * w + 2] = d.z;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                o.incident_lights[3 * w + k] = s.light[k];
                o.local_incident_lights[3 * w + k] = s.local[k];
                o.global_incident_lights[3 * w + k] = s.vis * s.global[k];
            }
            o.incident_visibility[w] = s.vis;
        } else {
            a.incident_dirs[3 * w] = d.x; a.incident_dirs[3 * w + 1] = d.y; a.incident_dirs[3 * w + 2] = d.z;
        }
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) s_c[t * (NC + 1) + k] = c[k];
    __syncthreads();
    // per (Gaussian, channel): the samples' contributions summed in sample order (the reference's
    // per-thread accumulation, render_equation.cu:630-655)
    for (int e = t; e < ng * NC; e += 256) {
        const int gg = e / NC, k = e - gg * NC;
        float acc = 0.f;
        for (int rr = 0; rr < Ns; ++rr) acc += s_c[(gg * Ns + rr) * (NC + 1) + k];
        s_sum[gg][k] = acc;
    }
    __syncthreads();
    if (t < ng) {
        const int idx = g0 + t;
        const float* v = s_sum[t];
        if constexpr (COMPLEX) {
            const r3dg_brdf_complex_outputs& o = a.cx;
            float av[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) av[k] = v[k] * kInvPi + v[9 + k];
            o.accum[idx] = (av[0] + av[1] + av[2]) / 3;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                o.pbr[3 * idx + k] = v[6 + k] + v[9 + k];
                o.rgb_d[3 * idx + k] = v[6 + k];
                o.rgb_s[3 * idx + k] = v[9 + k];
                o.diffuse_light[3 * idx + k] = v[k];
                o.local_diffuse_light[3 * idx + k] = v[3 + k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                a.pbr[3 * idx + k] = v[k];
                a.diffuse[3 * idx + k] = v[3 + k];
            }
        }
    }
}

template <bool COMPLEX>
static hipError_t launch_fwd(const BrdfKArgs& a, hipStream_t st) {
    const r3dg_brdf_inputs& in = a.in;
    const bool s16 = in.S_incident == 16 && in.S_direct == 16 && in.S_visibility == 16;
    const int Ns = in.sample_num;
    // a lane per (Gaussian, sample) while a workgroup holds at least one whole Gaussian; beyond 256
    // samples the thread-per-Gaussian kernel (no call site uses more than 24)
    if (Ns >= 1 && Ns <= 256) {
        const int GB = 256 / Ns;
        const dim3 grid((in.P + GB - 1) / GB), block(256);
        if (s16)
            hipLaunchKernelGGL((brdf_fwd_lane_kernel<16, 16, 16, COMPLEX>), grid, block, 0, st, a, GB);
        else
            hipLaunchKernelGGL((brdf_fwd_lane_kernel<0, 0, 0, COMPLEX>), grid, block, 0, st, a, GB);
        return hipGetLastError();
    }
    const dim3 grid((in.P + 255) / 256), block(256);
    if (in.S_incident == 16 && in.S_direct == 16 && in.S_visibility == 16)
        hipLaunchKernelGGL((brdf_fwd_kernel<16, 16, 16, COMPLEX>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((brdf_fwd_kernel<0, 0, 0, COMPLEX>), grid, block, 0, st, a);
    return hipGetLastError();
}

}  // namespace r3dg

using namespace r3dg;

static int check_brdf_inputs(const r3dg_brdf_inputs* in) {
    R3DG_REQUIRE(in && in->P >= 0 && in->sample_num >= 0, "render_equation: invalid sizes");
    R3DG_REQUIRE(in->S_incident <= 16 && in->S_direct <= 16 && in->S_visibility <= 16,
                 "render_equation: at most 16 SH coefficients (degree 3) are supported, as the reference "
                 "computeSHcoef(3) (render_equation.cu:17-50)");
    return R3DG_OK;
}

extern "C" int r3dg_render_equation_forward(const r3dg_brdf_inputs* in, int is_training, const float* rand_float,
                                            float* pbr, float* incident_dirs, float* diffuse_light,
                                            r3dg_stream_t stream) {
    int rc = check_brdf_inputs(in);
    if (rc) return rc;
    R3DG_REQUIRE(!is_training || rand_float || in->P == 0, "render_equation_forward: training needs rand_float");
    if (in->P == 0) return R3DG_OK;
    BrdfKArgs a{};
    a.in = *in;
    a.is_training = is_training;
    a.rand_float = rand_float;
    a.pbr = pbr;
    a.incident_dirs = incident_dirs;
    a.diffuse = diffuse_light;
    R3DG_CHECK_HIP(launch_fwd<false>(a, (hipStream_t)stream));
    return R3DG_OK;
}

extern "C" int r3dg_render_equation_forward_complex(const r3dg_brdf_inputs* in, const r3dg_brdf_complex_outputs* out,
                                                    r3dg_stream_t stream) {
    int rc = check_brdf_inputs(in);
    if (rc) return rc;
    if (in->P == 0) return R3DG_OK;
    BrdfKArgs a{};
    a.in = *in;
    a.cx = *out;
    R3DG_CHECK_HIP(launch_fwd<true>(a, (hipStream_t)stream));
    return R3DG_OK;
}

extern "C" int r3dg_render_equation_backward(const r3dg_brdf_inputs* in, const float* incident_dirs,
                                             const float* dL_dpbr, const float* dL_ddiffuse_light,
                                             r3dg_alloc_fn scratch_alloc, void* scratch_ctx, const r3dg_brdf_grads* out,
                                             r3dg_stream_t stream) {
    int rc = check_brdf_inputs(in);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int nb = (in->P + 255) / 256;
    if (in->P == 0) {
        R3DG_CHECK_HIP(hipMemsetAsync(out->dL_ddirect_shs, 0, sizeof(float) * 3 * in->S_direct, st));
        return R3DG_OK;
    }
    float* partials = (float*)scratch_alloc(scratch_ctx, sizeof(float) * 48 * (size_t)nb);
    if (!partials) {
        set_error("render_equation_backward: scratch allocation failed");
        return R3DG_ERR_ALLOC;
    }
    BrdfKArgs a{};
    a.in = *in;
    a.dirs_in = incident_dirs;
    a.dL_dpbr = dL_dpbr;
    a.dL_ddiff = dL_ddiffuse_light;
    a.gr = *out;
    a.dir_partials = partials;
    if (in->S_incident == 16 && in->S_direct == 16 && in->S_visibility == 16)
        hipLaunchKernelGGL((brdf_bwd_kernel<16, 16, 16>), dim3(nb), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((brdf_bwd_kernel<0, 0, 0>), dim3(nb), dim3(256), 0, st, a);
    R3DG_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(brdf_dir_reduce_kernel, dim3(max(1, 3 * in->S_direct)), dim3(256), 0, st, partials, nb,
                       3 * in->S_direct, out->dL_ddirect_shs);
    R3DG_CHECK_HIP(hipGetLastError());
    return R3DG_OK;
}
