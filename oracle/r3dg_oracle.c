/*
 * r3dg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference relightable Gaussian-splat rasterizer hot path
 * (Krapylet/Relightable3DGaussian, r3dg-rasterization). It is the parity checker for
 * the HIP product path in relightable3dgaussian_amd/csrc and is never linked into,
 * loaded by, or called from the product. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it.
 *
 * Every function cites the reference file:line it restates. Arithmetic that feeds the
 * tile|depth keys (preprocess, cov3D, cov2D, radius, rect) is written as plain IEEE ops in
 * a fixed order and this file is compiled with -ffp-contract=off; the HIP preprocess kernel
 * uses the same order with contraction off, so keys and sort order are bit-exact between
 * the two. (Bit-exactness against the CUDA binary itself is unverifiable offline: nvcc
 * contracts a*b+c into FMA by default, SURVEY.md §7 "Hard parts".)
 *
 * Pinning: the per-Gaussian sub-steps (SH colour, cov3D, BRDF) are checked against golden
 * vectors produced by the reference's own PyTorch code (tests/golden/, made by
 * tests/golden/make_golden.py). The tile blend itself has no reference fixture (the
 * reference ships no tests), see DESIGN.md "Parity".
 *
 * The blend's `power` and `exp(power)` (forward.cu:468-477, backward.cu:526-527) are the two
 * places where the reference's bits are compiler/libdevice-defined (nvcc's FMA contraction; CUDA
 * expf, <= 2 ulp). Both are stated here as ONE fixed sequence of IEEE f32 operations --
 * gauss_power (a fixed FMA pattern) and r3dg_expf (<= 0.90 ulp over [-80, 0], see below) -- that
 * the HIP kernels repeat operation for operation, so alpha, T, the early stop and n_contrib are
 * bit-identical between the two.
 *
 * Deliberate, documented deviations from the reference:
 *   - Stencil accumulator initialised to 0 (forward.cu:312 leaves it uninitialised).
 *   - dL_ddirect_shs accumulated sequentially (render_equation.cu:443-445 is a data race).
 *   - S-dependent feature output layout (feature_layout below): S=21 is the reference's
 *     block layout (forward.cu:537-558); S=11 uses groups [1,1,3,3,3]; else planar.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define BX 16
#define BY 16

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};
static const float PI_F = 3.14159f; /* render_equation.cu uses the literal 3.14159f */
#define INV_PI_F (1.0f / 3.14159f) /* products in place of per-sample divisions by PI_F (brdf.hip kInvPi) */

/* ------------------------------------------------------------------------------------------ */
/* small helpers (auxiliary.h:41-132)                                                          */
/* ------------------------------------------------------------------------------------------ */

/* auxiliary.h:41-44 -- note the double-precision literals */
static float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

/* auxiliary.h:46-56 */
static void get_rect(float px, float py, int max_radius, int gx, int gy, int* rmin, int* rmax)
{
    rmin[0] = imin(gx, imax(0, (int)((px - (float)max_radius) / BX)));
    rmin[1] = imin(gy, imax(0, (int)((py - (float)max_radius) / BY)));
    rmax[0] = imin(gx, imax(0, (int)((px + (float)max_radius + BX - 1) / BX)));
    rmax[1] = imin(gy, imax(0, (int)((py + (float)max_radius + BY - 1) / BY)));
}

/* forward.cu:468 / backward.cu:526: -0.5f * (a dx^2 + c dy^2) - b dx dy as one fixed FMA pattern
 * (the HIP kernels' gauss_power, r3dg_common.h): with the staged conic (A, B, C) = (-a/2, -b, -c/2)
 * (exact scalings, preprocess_kernel's render records), dx (A dx + B dy) + C dy^2. */
static int g_power_ref_ops = 0;
/* Measurement switch (tests/test_oracle.py test_power_ref_ops_c2): 0 = the staged
 * FMA pattern below (the HIP kernels'); 1 = forward.cu:478 / backward.cu:526 as written,
 * -0.5f * (a dx dx + c dy dy) - b dx dy, every product and sum rounded (no contraction); 2 = the
 * same expression with the two contractions nvcc's default -fmad=true may apply
 * (fma(a dx, dx, (c dy) dy), then fma(-0.5, s, -(b dx) dy)). The reference's own bits depend on
 * its compiler; these bracket them. */
void oracle_set_power_ref_ops(int mode) { g_power_ref_ops = mode; }
static float gauss_power(const float* co, float dx, float dy)
{
    if (g_power_ref_ops == 1) {
        const float s = co[0] * dx * dx + co[2] * dy * dy;
        return -0.5f * s - co[1] * dx * dy;
    }
    if (g_power_ref_ops == 2) {
        const float s = fmaf(co[0] * dx, dx, (co[2] * dy) * dy);
        return fmaf(-0.5f, s, -((co[1] * dx) * dy));
    }
    const float A = -0.5f * co[0], B = -co[1], C = -0.5f * co[2];
    const float f = fmaf(A, dx, B * dy);
    return fmaf(dx, f, (C * dy) * dy);
}

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* forward.cu:477 / backward.cu:527 exp(power): Cody-Waite reduction by ln2 (16 + 24-bit split),
 * degree-6 polynomial for e^r (1 + r exact), 2^k by an integer add to the exponent field (the
 * shifted kf holds k in its low bits, (0x4B400000 << 23) == 0 mod 2^32). Input clamped to
 * [-80, 0]. Identical operation sequence to r3dg_common.h r3dg_expf. */
float r3dg_expf(float x)
{
    x = fminf(fmaxf(x, -80.0f), 0.0f);
    const float kf = fmaf(x, 0x1.715476p+0f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = fmaf(k, -0x1.62e400p-1f, x);
    r = fmaf(k, -0x1.7f7d1cp-20f, r);
    float p = 0x1.6a959cp-10f;
    p = fmaf(p, r, 0x1.123a0ap-7f);
    p = fmaf(p, r, 0x1.555850p-5f);
    p = fmaf(p, r, 0x1.555492p-3f);
    p = fmaf(p, r, 0x1.fffffcp-2f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return u2f(f2u(p) + (f2u(kf) << 23));
}

/* render_equation.cu:151 / :351 expf(sharp * (h_d_n - 1)): r3dg_expf's operations over [-87, 88]
 * (p * 2^k a normal float there), 0 below -87. Identical operation sequence to r3dg_common.h
 * r3dg_expf_wide. */
float r3dg_expf_wide(float x)
{
    if (x < -87.0f) return 0.0f;
    x = fminf(x, 88.0f);
    const float kf = fmaf(x, 0x1.715476p+0f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = fmaf(k, -0x1.62e400p-1f, x);
    r = fmaf(k, -0x1.7f7d1cp-20f, r);
    float p = 0x1.6a959cp-10f;
    p = fmaf(p, r, 0x1.123a0ap-7f);
    p = fmaf(p, r, 0x1.555850p-5f);
    p = fmaf(p, r, 0x1.555492p-3f);
    p = fmaf(p, r, 0x1.fffffcp-2f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return u2f(f2u(p) + (f2u(kf) << 23));
}

/* render_equation.cu:93-94 cosf(theta) / sinf(theta) (CUDA: implementation-defined to 2 ulp):
 * k = rint(x 2/pi) by the 1.5 * 2^23 shift, r = x - k pi/2 with pi/2 split in three floats (C1 =
 * 0x1.921fb6p+0, C2 = -0x1.777a5cp-25, C3 = -0x1.ee59dap-50), Cephes minimax sin / cos on
 * [-pi/4, pi/4], quadrant k mod 4. Identical operation sequence to r3dg_common.h r3dg_sincosf. */
void r3dg_sincosf(float x, float* s_out, float* c_out)
{
    const float kf = fmaf(x, 0x1.45f306p-1f, 0x1.8p+23f);
    const float k = kf - 0x1.8p+23f;
    float r = fmaf(k, -0x1.921fb6p+0f, x);
    r = fmaf(k, 0x1.777a5cp-25f, r);
    r = fmaf(k, 0x1.ee59dap-50f, r);
    const float r2 = r * r;
    float ps = fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f);
    ps = fmaf(ps, r2, -1.6666654611e-1f);
    const float sn = fmaf(ps * r2, r, r);
    float pc = fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f);
    pc = fmaf(pc, r2, 4.166664568298827e-2f);
    const float cs = fmaf(pc * r2, r2, fmaf(-0.5f, r2, 1.0f));
    const uint32_t q = f2u(kf) & 3u;
    const float a = (q & 1u) ? cs : sn, b = (q & 1u) ? sn : cs;
    *s_out = (q & 2u) ? -a : a;
    *c_out = ((q + 1u) & 2u) ? -b : b;
}

/* The blend's exp: r3dg_expf (mode 0, what the HIP kernels evaluate) or glibc's expf (mode 1, a
 * stand-in for a vendor libm exp such as the reference's CUDA expf, forward.cu:477 / backward.cu:527).
 * Mode 1 exists only to measure how far n_contrib / final_T / the images move when the exp is not
 * the build's own (tests/test_oracle.py test_blend_exp_choice_c2). */
static int g_blend_exp_libm = 0;
void oracle_set_blend_exp(int libm) { g_blend_exp_libm = libm; }
static float blend_exp(float x) { return g_blend_exp_libm ? expf(x) : r3dg_expf(x); }

/* Accuracy check of r3dg_expf against double-precision exp over the floats x = lo, ... stepping
 * `stride` bit patterns through [lo, hi] (both <= 0): max error in ulp of the float result and the
 * count of correctly rounded results. */
double oracle_expf_max_ulp(float lo, float hi, uint32_t stride, long long* n, long long* exact)
{
    double maxe = 0.0;
    *n = 0;
    *exact = 0;
    const uint64_t end = f2u(lo);
    for (uint64_t u = f2u(hi) | 0x80000000u; u <= end; u += stride) {
        const float x = u2f((uint32_t)u);
        const double e = exp((double)x);
        const float y = r3dg_expf(x);
        const double ulp = ldexp(1.0, ilogb(e) - 23);
        const double err = fabs((double)y - e) / ulp;
        if (err > maxe) maxe = err;
        ++*n;
        if (y == (float)e) ++*exact;
    }
    return maxe;
}

/* auxiliary.h:58-66 */
static void xform_point4x3(const float* p, const float* m, float* o)
{
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}

/* auxiliary.h:68-77 */
static void xform_point4x4(const float* p, const float* m, float* o)
{
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* auxiliary.h:89-97 */
static void xform_vec4x3_transpose(const float* p, const float* m, float* o)
{
    o[0] = m[0] * p[0] + m[1] * p[1] + m[2] * p[2];
    o[1] = m[4] * p[0] + m[5] * p[1] + m[6] * p[2];
    o[2] = m[8] * p[0] + m[9] * p[1] + m[10] * p[2];
}

/* auxiliary.h:107-117 */
static void dnormvdv3(const float* v, const float* dv, float* o)
{
    float sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    o[0] = ((+sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    o[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    o[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* ------------------------------------------------------------------------------------------ */
/* feature output layout (forward.cu:537-558 for S=21; see header for other S)                 */
/* channel c of pixel pix lives at out[a[c] + pix * m[c]]                                      */
/* ------------------------------------------------------------------------------------------ */
int oracle_feature_groups(int S, int* groups)
{
    int n = 0;
    if (S == 21) {
        static const int g[9] = {1, 1, 1, 3, 3, 3, 3, 3, 3};
        for (n = 0; n < 9; ++n) groups[n] = g[n];
    } else if (S == 11) {
        static const int g[5] = {1, 1, 3, 3, 3};
        for (n = 0; n < 5; ++n) groups[n] = g[n];
    } else {
        for (n = 0; n < S; ++n) groups[n] = 1;
    }
    return n;
}

void oracle_feature_layout(int S, long long HW, long long* a, int* m)
{
    int groups[64];
    int ng = oracle_feature_groups(S, groups);
    int c = 0;
    for (int g = 0; g < ng; ++g) {
        for (int k = 0; k < groups[g]; ++k) {
            a[c + k] = HW * (long long)c + k;
            m[c + k] = groups[g];
        }
        c += groups[g];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* forward per-Gaussian math                                                                   */
/* ------------------------------------------------------------------------------------------ */

/* forward.cu:25-76 */
static void color_from_sh(int idx, int deg, int max_coeffs, const float* means, const float* campos,
                          const float* shs, uint8_t* clamped, float* out)
{
    float dir[3] = {means[3 * idx] - campos[0], means[3 * idx + 1] - campos[1], means[3 * idx + 2] - campos[2]};
    float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float x = dir[0], y = dir[1], z = dir[2];
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, yz = y * z, xz = x * z;
    uint8_t cl = 0;
    for (int c = 0; c < 3; ++c) {
        float r = SH_C0 * sh[0 * 3 + c];
        if (deg > 0) {
            r = r - SH_C1 * y * sh[1 * 3 + c] + SH_C1 * z * sh[2 * 3 + c] - SH_C1 * x * sh[3 * 3 + c];
            if (deg > 1) {
                r = r + SH_C2[0] * xy * sh[4 * 3 + c] + SH_C2[1] * yz * sh[5 * 3 + c] +
                    SH_C2[2] * (2.0f * zz - xx - yy) * sh[6 * 3 + c] + SH_C2[3] * xz * sh[7 * 3 + c] +
                    SH_C2[4] * (xx - yy) * sh[8 * 3 + c];
                if (deg > 2) {
                    r = r + SH_C3[0] * y * (3.0f * xx - yy) * sh[9 * 3 + c] + SH_C3[1] * xy * z * sh[10 * 3 + c] +
                        SH_C3[2] * y * (4.0f * zz - xx - yy) * sh[11 * 3 + c] +
                        SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3 + c] +
                        SH_C3[4] * x * (4.0f * zz - xx - yy) * sh[13 * 3 + c] +
                        SH_C3[5] * z * (xx - yy) * sh[14 * 3 + c] + SH_C3[6] * x * (xx - 3.0f * yy) * sh[15 * 3 + c];
                }
            }
        }
        r += 0.5f;
        if (r < 0) cl |= (uint8_t)(1u << c);
        out[c] = r < 0.0f ? 0.0f : r;
    }
    clamped[idx] = cl;
}

/* forward.cu:124-158 (quaternion deliberately NOT normalised, (r,x,y,z) order) */
static void rot_matrix(const float* q, float R[3][3])
{
    /* R[i][j] is the math (row i, col j) element of the glm matrix built at forward.cu:140-144
       (glm is column-major, so this is the transpose of the usual quaternion rotation). */
    float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y + r * z); R[0][2] = 2.f * (x * z - r * y);
    R[1][0] = 2.f * (x * y - r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z + r * x);
    R[2][0] = 2.f * (x * z + r * y); R[2][1] = 2.f * (y * z - r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

static void compute_cov3d(const float* scale, float mod, const float* rot, float* cov3D)
{
    float R[3][3], M[3][3];
    rot_matrix(rot, R);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[i][j] = s[i] * R[i][j];
    /* Sigma = M^T M */
    cov3D[0] = M[0][0] * M[0][0] + M[1][0] * M[1][0] + M[2][0] * M[2][0];
    cov3D[1] = M[0][0] * M[0][1] + M[1][0] * M[1][1] + M[2][0] * M[2][1];
    cov3D[2] = M[0][0] * M[0][2] + M[1][0] * M[1][2] + M[2][0] * M[2][2];
    cov3D[3] = M[0][1] * M[0][1] + M[1][1] * M[1][1] + M[2][1] * M[2][1];
    cov3D[4] = M[0][1] * M[0][2] + M[1][1] * M[1][2] + M[2][1] * M[2][2];
    cov3D[5] = M[0][2] * M[0][2] + M[1][2] * M[1][2] + M[2][2] * M[2][2];
}

/* forward.cu:79-118.  g0/g1 are the first two columns of T = W*J (glm T[0], T[1]). */
static void cov2d_T(const float* mean, float fx, float fy, float tanx, float tany, const float* view,
                    float* t_out, float* g0, float* g1, int* xmul, int* ymul)
{
    float t[3];
    xform_point4x3(mean, view, t);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    if (xmul) *xmul = (txtz < -limx || txtz > limx) ? 0 : 1;
    if (ymul) *ymul = (tytz < -limy || tytz > limy) ? 0 : 1;
    const float j00 = fx / t[2], j11 = fy / t[2];
    const float j20 = -(fx * t[0]) / (t[2] * t[2]);
    const float j21 = -(fy * t[1]) / (t[2] * t[2]);
    for (int r = 0; r < 3; ++r) {
        g0[r] = view[4 * r + 0] * j00 + view[4 * r + 2] * j20;
        g1[r] = view[4 * r + 1] * j11 + view[4 * r + 2] * j21;
    }
    t_out[0] = t[0]; t_out[1] = t[1]; t_out[2] = t[2];
}

static void cov2d_from_T(const float* g0, const float* g1, const float* c, float* abc)
{
    float u0 = c[0] * g0[0] + c[1] * g0[1] + c[2] * g0[2];
    float u1 = c[1] * g0[0] + c[3] * g0[1] + c[4] * g0[2];
    float u2 = c[2] * g0[0] + c[4] * g0[1] + c[5] * g0[2];
    float v0 = c[0] * g1[0] + c[1] * g1[1] + c[2] * g1[2];
    float v1 = c[1] * g1[0] + c[3] * g1[1] + c[4] * g1[2];
    float v2 = c[2] * g1[0] + c[4] * g1[1] + c[5] * g1[2];
    abc[0] = g0[0] * u0 + g0[1] * u1 + g0[2] * u2 + 0.3f;
    abc[1] = g1[0] * u0 + g1[1] * u1 + g1[2] * u2;
    abc[2] = g1[0] * v0 + g1[1] * v1 + g1[2] * v2 + 0.3f;
}

/* forward.cu:161-267 (preprocessCUDA) */
int oracle_preprocess(int P, int D, int M, const float* means3D, const float* scales, float scale_modifier,
                      const float* rotations, const float* opacities, const float* shs, const float* cov3D_precomp,
                      const float* colors_precomp, const float* view, const float* proj, const float* campos, int W,
                      int H, float tan_fovx, float tan_fovy, int* radii, float* means2D, float* depths,
                      float* cov3Ds, float* rgb, uint8_t* clamped, float* conic_opacity, uint32_t* tiles_touched)
{
    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    for (int idx = 0; idx < P; ++idx) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        const float* p = means3D + 3 * idx;
        float pv[3];
        xform_point4x3(p, view, pv); /* auxiliary.h:152 */
        if (pv[2] <= 0.2f) continue;  /* auxiliary.h:154 */
        float ph[4];
        xform_point4x4(p, proj, ph);
        float p_w = 1.0f / (ph[3] + 0.0000001f);
        float pp[3] = {ph[0] * p_w, ph[1] * p_w, ph[2] * p_w};
        const float* cov3D;
        if (cov3D_precomp) {
            cov3D = cov3D_precomp + 6 * idx;
        } else {
            compute_cov3d(scales + 3 * idx, scale_modifier, rotations + 4 * idx, cov3Ds + 6 * idx);
            cov3D = cov3Ds + 6 * idx;
        }
        float t[3], g0[3], g1[3], abc[3];
        cov2d_T(p, focal_x, focal_y, tan_fovx, tan_fovy, view, t, g0, g1, NULL, NULL);
        cov2d_from_T(g0, g1, cov3D, abc);
        float det = abc[0] * abc[2] - abc[1] * abc[1];
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {abc[2] * det_inv, -abc[1] * det_inv, abc[0] * det_inv};
        float mid = 0.5f * (abc[0] + abc[2]);
        float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        float px = ndc2pix(pp[0], W), py = ndc2pix(pp[1], H);
        int rmin[2], rmax[2];
        get_rect(px, py, (int)my_radius, gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (!colors_precomp) color_from_sh(idx, D, M, means3D, campos, shs, clamped, rgb + 3 * idx);
        depths[idx] = pv[2];
        radii[idx] = (int)my_radius;
        means2D[2 * idx] = px;
        means2D[2 * idx + 1] = py;
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = opacities[idx];
        tiles_touched[idx] = (uint32_t)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
    }
    return 0;
}

/* rasterizer_impl.cu:56-68 + auxiliary.h:139-164 */
void oracle_mark_visible(int P, const float* means3D, const float* view, uint8_t* present)
{
    for (int i = 0; i < P; ++i) {
        float pv[3];
        xform_point4x3(means3D + 3 * i, view, pv);
        present[i] = pv[2] <= 0.2f ? 0 : 1;
    }
}

/* rasterizer_impl.cu:37-52 */
uint32_t oracle_higher_msb(uint32_t n)
{
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

/* ------------------------------------------------------------------------------------------ */
/* binning: duplicateWithKeys + stable sort + identifyTileRanges                               */
/* ------------------------------------------------------------------------------------------ */

/* rasterizer_impl.cu:72-113; offsets is the inclusive prefix sum of tiles_touched (:343) */
void oracle_duplicate_with_keys(int P, const float* means2D, const float* depths, const uint32_t* offsets,
                                const int* radii, int W, int H, uint64_t* keys, uint32_t* vals)
{
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    for (int idx = 0; idx < P; ++idx) {
        if (radii[idx] <= 0) continue;
        uint32_t off = idx == 0 ? 0 : offsets[idx - 1];
        int rmin[2], rmax[2];
        get_rect(means2D[2 * idx], means2D[2 * idx + 1], radii[idx], gx, gy, rmin, rmax);
        uint32_t dbits;
        memcpy(&dbits, &depths[idx], 4);
        for (int y = rmin[1]; y < rmax[1]; ++y)
            for (int x = rmin[0]; x < rmax[0]; ++x) {
                uint64_t key = (uint64_t)(uint32_t)(y * gx + x);
                key <<= 32;
                key |= dbits;
                keys[off] = key;
                vals[off] = (uint32_t)idx;
                off++;
            }
    }
}

/* Stable LSD radix sort of (key, value) on bits [0, end_bit): restates the semantics of the
   cub::DeviceRadixSort::SortPairs call at rasterizer_impl.cu:369-374 (CUB 11.8, not vendored). */
void oracle_sort_pairs(long long L, const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                       uint32_t* vals_out, int end_bit)
{
    uint64_t* ka = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(L ? L : 1));
    uint64_t* kb = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(L ? L : 1));
    uint32_t* va = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(L ? L : 1));
    uint32_t* vb = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(L ? L : 1));
    memcpy(ka, keys_in, sizeof(uint64_t) * (size_t)L);
    memcpy(va, vals_in, sizeof(uint32_t) * (size_t)L);
    for (int shift = 0; shift < end_bit; shift += 8) {
        int bits = end_bit - shift < 8 ? end_bit - shift : 8;
        uint64_t mask = (1ull << bits) - 1;
        long long cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (long long i = 0; i < L; ++i) cnt[((ka[i] >> shift) & mask) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (long long i = 0; i < L; ++i) {
            long long dst = cnt[(ka[i] >> shift) & mask]++;
            kb[dst] = ka[i];
            vb[dst] = va[i];
        }
        uint64_t* tk = ka; ka = kb; kb = tk;
        uint32_t* tv = va; va = vb; vb = tv;
    }
    memcpy(keys_out, ka, sizeof(uint64_t) * (size_t)L);
    memcpy(vals_out, va, sizeof(uint32_t) * (size_t)L);
    free(ka); free(kb); free(va); free(vb);
}

/* rasterizer_impl.cu:118-140 (ranges zeroed first, :376) */
void oracle_identify_tile_ranges(long long L, const uint64_t* keys, int num_tiles, uint32_t* ranges)
{
    memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)num_tiles);
    for (long long idx = 0; idx < L; ++idx) {
        uint32_t cur = (uint32_t)(keys[idx] >> 32);
        if (idx == 0) ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(keys[idx - 1] >> 32);
            if (cur != prev) {
                ranges[2 * prev + 1] = (uint32_t)idx;
                ranges[2 * cur] = (uint32_t)idx;
            }
        }
        if (idx == L - 1) ranges[2 * cur + 1] = (uint32_t)L;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* tile blend, forward (forward.cu:388-561)                                                    */
/* ------------------------------------------------------------------------------------------ */
void oracle_render_forward(int W, int H, int S, const uint32_t* ranges, const uint32_t* point_list,
                           const float* means2D, const float* depths, const float* features,
                           const float* shader_colors, const float* colors, const float* conic_opacity,
                           const float* bg, float* final_T, uint32_t* n_contrib, float* out_color,
                           float* out_opacity, float* out_depth, float* out_feature, float* out_shader_color)
{
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const long long HW = (long long)H * W;
    long long fa[64];
    int fm[64];
    oracle_feature_layout(S, HW, fa, fm);
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const uint32_t* range = ranges + 2 * (ty * gx + tx);
            for (int ly = 0; ly < BY; ++ly)
                for (int lx = 0; lx < BX; ++lx) {
                    int px = tx * BX + lx, py = ty * BY + ly;
                    if (px >= W || py >= H) continue;
                    long long pix = (long long)py * W + px;
                    float pfx = (float)px, pfy = (float)py;
                    float T = 1.0f;
                    uint32_t contributor = 0, last = 0;
                    float C[3] = {0, 0, 0}, CS[3] = {0, 0, 0}, F[64], Dp = 0, Op = 0;
                    for (int c = 0; c < S; ++c) F[c] = 0;
                    for (uint32_t k = range[0]; k < range[1]; ++k) {
                        contributor++;
                        uint32_t id = point_list[k];
                        float dx = means2D[2 * id] - pfx, dy = means2D[2 * id + 1] - pfy;
                        const float* co = conic_opacity + 4 * id;
                        float power = gauss_power(co, dx, dy);
                        if (power > 0.0f) continue;
                        float alpha = fminf(0.99f, co[3] * blend_exp(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        float test_T = T * (1 - alpha);
                        if (test_T < 0.0001f) break; /* done = true */
                        float w = alpha * T;
                        for (int c = 0; c < 3; ++c) C[c] += colors[3 * id + c] * w;
                        for (int c = 0; c < 3; ++c) CS[c] += shader_colors[3 * id + c] * w;
                        for (int c = 0; c < S; ++c) F[c] += features[(size_t)id * S + c] * w;
                        Dp += depths[id] * w;
                        Op += w;
                        T = test_T;
                        last = contributor;
                    }
                    final_T[pix] = T;
                    n_contrib[pix] = last;
                    for (int c = 0; c < 3; ++c) out_color[pix * 3 + c] = C[c] + T * bg[c];
                    for (int c = 0; c < 3; ++c) out_shader_color[pix * 3 + c] = CS[c] + T * bg[c];
                    out_depth[pix] = Dp;
                    out_opacity[pix] = Op;
                    for (int c = 0; c < S; ++c) out_feature[fa[c] + pix * fm[c]] = F[c];
                }
        }
}

/* forward.cu:271-383 (RenderIntermediateTextures; Stencil initialised to 0, see header) */
void oracle_render_intermediate(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                                const float* means2D, const float* depths, const float* stencils,
                                const float* conic_opacity, const float* stencil_opacity, float* out_depth,
                                float* out_stencil)
{
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const uint32_t* range = ranges + 2 * (ty * gx + tx);
            for (int ly = 0; ly < BY; ++ly)
                for (int lx = 0; lx < BX; ++lx) {
                    int px = tx * BX + lx, py = ty * BY + ly;
                    if (px >= W || py >= H) continue;
                    long long pix = (long long)py * W + px;
                    float sT = 1.0f, T = 1.0f, St = 0.0f, Dp = 0.0f;
                    for (uint32_t k = range[0]; k < range[1]; ++k) {
                        uint32_t id = point_list[k];
                        float dx = means2D[2 * id] - (float)px, dy = means2D[2 * id + 1] - (float)py;
                        const float* co = conic_opacity + 4 * id;
                        float power = gauss_power(co, dx, dy);
                        if (power > 0.0f) continue;
                        float G = blend_exp(power);
                        float alpha = fminf(0.99f, co[3] * G);
                        float salpha = fminf(0.99f, stencil_opacity[id] * G);
                        if (alpha < 1.0f / 255.0f && salpha < 1.0f / 255.0f) continue;
                        float tT = T * (1 - alpha), tS = sT * (1 - salpha);
                        if (tT < 0.0001f && tS < 0.0001f) break;
                        Dp += depths[id] * (alpha * T);
                        T = tT;
                        St += stencils[id] * (salpha * sT);
                        sT = tS;
                    }
                    out_depth[pix] = Dp;
                    out_stencil[pix] = St;
                }
        }
}

/* forward.cu:564-591 and :593-658 */
void oracle_surface_xyz_normal(int W, int H, const float* view, float fx, float fy, float cx, float cy,
                               const float* opacity, const float* depth, float* normal, float* xyz)
{
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            long long pix = (long long)y * W + x;
            float d = depth[pix] / fmaxf(opacity[pix], 0.0000001f);
            xyz[pix * 3 + 0] = ((float)x - cx) / fx * d;
            xyz[pix * 3 + 1] = ((float)y - cy) / fy * d;
            xyz[pix * 3 + 2] = d;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int ym = y == 0 ? 0 : y - 1, yp = y == H - 1 ? H - 1 : y + 1;
            int xm = x == 0 ? 0 : x - 1, xp = x == W - 1 ? W - 1 : x + 1;
            const float* p00 = xyz + 3 * ((long long)W * ym + xm);
            const float* p01 = xyz + 3 * ((long long)W * ym + x);
            const float* p02 = xyz + 3 * ((long long)W * ym + xp);
            const float* p10 = xyz + 3 * ((long long)W * y + xm);
            const float* p12 = xyz + 3 * ((long long)W * y + xp);
            const float* p20 = xyz + 3 * ((long long)W * yp + xm);
            const float* p21 = xyz + 3 * ((long long)W * yp + x);
            const float* p22 = xyz + 3 * ((long long)W * yp + xp);
            float ga[3], gb[3];
            for (int i = 0; i < 3; ++i)
                ga[i] = -0.125f * p00[i] + 0.125f * p02[i] - 0.25f * p10[i] + 0.25f * p12[i] - 0.125f * p20[i] +
                        0.125f * p22[i];
            for (int i = 0; i < 3; ++i)
                gb[i] = -0.125f * p00[i] - 0.25f * p01[i] - 0.125f * p02[i] + 0.125f * p20[i] + 0.25f * p21[i] +
                        0.125f * p22[i];
            float n[3] = {ga[1] * gb[2] - ga[2] * gb[1], -ga[0] * gb[2] + ga[2] * gb[0], ga[0] * gb[1] - ga[1] * gb[0]};
            float norm = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            long long pix = (long long)y * W + x;
            if (norm <= 0.0f) {
                normal[pix * 3 + 0] = normal[pix * 3 + 1] = normal[pix * 3 + 2] = 0.0f;
                continue;
            }
            n[0] = -n[0] / norm; n[1] = -n[1] / norm; n[2] = -n[2] / norm;
            normal[pix * 3 + 0] = view[0] * n[0] + view[1] * n[1] + view[2] * n[2];
            normal[pix * 3 + 1] = view[4] * n[0] + view[5] * n[1] + view[6] * n[2];
            normal[pix * 3 + 2] = view[8] * n[0] + view[9] * n[1] + view[10] * n[2];
        }
}

/* ------------------------------------------------------------------------------------------ */
/* tile blend, backward (backward.cu:401-614). Gradients accumulate sequentially.               */
/* grad layouts: colour channel c of pixel pix at dcol[ca[c] + pix*cm[c]], same for features.  */
/* ------------------------------------------------------------------------------------------ */
/* Test-only accuracy reference (not the reference's arithmetic): when set, the per-pixel mean2D /
   conic / opacity terms below are formed in double from the same f32 per-pixel values and summed
   into these double accumulators instead of the f32 outputs -- the sums the reference's f32
   atomics approximate. tests/test_gpu_parity.py (needles) measures the f32 statement's own error
   against it. */
static double *g_acc64_mean2D = NULL, *g_acc64_conic = NULL, *g_acc64_opac = NULL;
void oracle_set_render_bwd_acc64(double* mean2D, double* conic, double* opac)
{
    g_acc64_mean2D = mean2D;
    g_acc64_conic = conic;
    g_acc64_opac = opac;
}

void oracle_render_backward(int W, int H, int S, const uint32_t* ranges, const uint32_t* point_list,
                            const float* bg, const float* means2D, const float* depths, const float* conic_opacity,
                            const float* colors, const float* features, const float* final_Ts,
                            const uint32_t* n_contrib, const float* dL_dpix, const long long* ca, const int* cm,
                            const float* dL_dpix_o, const float* dL_dpix_d, const float* dL_dpix_f,
                            const long long* fa, const int* fm, int backward_geometry, float* dL_dmean2D,
                            float* dL_dconic, float* dL_dopacity, float* dL_dcolors, float* dL_dfeature)
{
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const uint32_t* range = ranges + 2 * (ty * gx + tx);
            for (int ly = 0; ly < BY; ++ly)
                for (int lx = 0; lx < BX; ++lx) {
                    int px = tx * BX + lx, py = ty * BY + ly;
                    if (px >= W || py >= H) continue;
                    long long pix = (long long)py * W + px;
                    const float T_final = final_Ts[pix];
                    float T = T_final;
                    const uint32_t last = n_contrib[pix];
                    float g[3], gd = dL_dpix_d[pix], go = dL_dpix_o[pix], gf[64];
                    for (int c = 0; c < 3; ++c) g[c] = dL_dpix[ca[c] + pix * cm[c]];
                    for (int c = 0; c < S; ++c) gf[c] = dL_dpix_f[fa[c] + pix * fm[c]];
                    float acc[3] = {0, 0, 0}, acc_d = 0, acc_o = 0, acc_f[64];
                    for (int c = 0; c < S; ++c) acc_f[c] = 0;
                    float last_alpha = 0, last_depth = 0, last_color[3] = {0, 0, 0}, last_f[64];
                    for (int c = 0; c < S; ++c) last_f[c] = 0;
                    float bg_dot = 0;
                    for (int c = 0; c < 3; ++c) bg_dot += bg[c] * g[c];
                    for (long long k = (long long)range[1] - 1; k >= (long long)range[0]; --k) {
                        uint32_t pos = (uint32_t)(k - range[0]); /* `contributor` after decrement */
                        if (pos >= last) continue;
                        uint32_t id = point_list[k];
                        float dx = means2D[2 * id] - (float)px, dy = means2D[2 * id + 1] - (float)py;
                        const float* co = conic_opacity + 4 * id;
                        float power = gauss_power(co, dx, dy);
                        if (power > 0.0f) continue;
                        float G = blend_exp(power);
                        float alpha = fminf(0.99f, co[3] * G);
                        if (alpha < 1.0f / 255.0f) continue;
                        T = T / (1.f - alpha);
                        const float dchannel_dcolor = alpha * T;
                        float dL_dalpha = 0.0f;
                        for (int c = 0; c < 3; ++c) {
                            float col = colors[3 * id + c];
                            acc[c] = last_alpha * last_color[c] + (1.f - last_alpha) * acc[c];
                            last_color[c] = col;
                            dL_dalpha += (col - acc[c]) * g[c];
                            dL_dcolors[3 * id + c] += dchannel_dcolor * g[c];
                        }
                        for (int c = 0; c < S; ++c) {
                            float f = features[(size_t)id * S + c];
                            acc_f[c] = last_alpha * last_f[c] + (1.f - last_alpha) * acc_f[c];
                            last_f[c] = f;
                            if (backward_geometry) dL_dalpha += (f - acc_f[c]) * gf[c];
                            dL_dfeature[(size_t)id * S + c] += dchannel_dcolor * gf[c];
                        }
                        float dep = depths[id];
                        acc_d = last_alpha * last_depth + (1.f - last_alpha) * acc_d;
                        last_depth = dep;
                        dL_dalpha += (dep - acc_d) * gd;
                        acc_o = last_alpha + (1.f - last_alpha) * acc_o;
                        dL_dalpha += (1.0f - acc_o) * go;
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = co[3] * dL_dalpha;
                        if (g_acc64_mean2D) {
                            const double dG = (double)co[3] * dL_dalpha, gx = (double)G * dx, gy = (double)G * dy;
                            g_acc64_mean2D[3 * id + 0] += dG * (-gx * co[0] - gy * co[1]) * ddelx_dx;
                            g_acc64_mean2D[3 * id + 1] += dG * (-gy * co[2] - gx * co[1]) * ddely_dy;
                            g_acc64_mean2D[3 * id + 2] += (double)gd * dchannel_dcolor;
                            g_acc64_conic[4 * id + 0] += -0.5 * gx * dx * dG;
                            g_acc64_conic[4 * id + 1] += -0.5 * gx * dy * dG;
                            g_acc64_conic[4 * id + 3] += -0.5 * gy * dy * dG;
                            g_acc64_opac[id] += (double)G * dL_dalpha;
                            continue;
                        }
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                        const float dG_ddely = -gdy * co[2] - gdx * co[1];
                        dL_dmean2D[3 * id + 0] += dL_dG * dG_ddelx * ddelx_dx;
                        dL_dmean2D[3 * id + 1] += dL_dG * dG_ddely * ddely_dy;
                        dL_dmean2D[3 * id + 2] += gd * dchannel_dcolor;
                        dL_dconic[4 * id + 0] += -0.5f * gdx * dx * dL_dG;
                        dL_dconic[4 * id + 1] += -0.5f * gdx * dy * dL_dG;
                        dL_dconic[4 * id + 3] += -0.5f * gdy * dy * dL_dG;
                        dL_dopacity[id] += G * dL_dalpha;
                    }
                }
        }
}

/* ------------------------------------------------------------------------------------------ */
/* per-Gaussian backward (backward.cu:20-139, 144-276, 280-343, 348-398)                       */
/* ------------------------------------------------------------------------------------------ */
static void color_from_sh_backward(int idx, int deg, int max_coeffs, const float* means, const float* campos,
                                   const float* shs, const uint8_t* clamped, const float* dL_dcolor,
                                   float* dL_dmeans, float* dL_dshs)
{
    float dir_orig[3] = {means[3 * idx] - campos[0], means[3 * idx + 1] - campos[1], means[3 * idx + 2] - campos[2]};
    float len = sqrtf(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    float x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float* dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
    float dRGB[3];
    for (int c = 0; c < 3; ++c) dRGB[c] = dL_dcolor[3 * idx + c] * ((clamped[idx] >> c) & 1 ? 0.0f : 1.0f);
    float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; ++c) dsh[0 * 3 + c] = SH_C0 * dRGB[c];
    if (deg > 0) {
        float b1 = -SH_C1 * y, b2 = SH_C1 * z, b3 = -SH_C1 * x;
        for (int c = 0; c < 3; ++c) {
            dsh[1 * 3 + c] = b1 * dRGB[c];
            dsh[2 * 3 + c] = b2 * dRGB[c];
            dsh[3 * 3 + c] = b3 * dRGB[c];
            ddx[c] = -SH_C1 * sh[3 * 3 + c];
            ddy[c] = -SH_C1 * sh[1 * 3 + c];
            ddz[c] = SH_C1 * sh[2 * 3 + c];
        }
        if (deg > 1) {
            float b4 = SH_C2[0] * xy, b5 = SH_C2[1] * yz, b6 = SH_C2[2] * (2.f * zz - xx - yy), b7 = SH_C2[3] * xz,
                  b8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; ++c) {
                dsh[4 * 3 + c] = b4 * dRGB[c];
                dsh[5 * 3 + c] = b5 * dRGB[c];
                dsh[6 * 3 + c] = b6 * dRGB[c];
                dsh[7 * 3 + c] = b7 * dRGB[c];
                dsh[8 * 3 + c] = b8 * dRGB[c];
                ddx[c] += SH_C2[0] * y * sh[4 * 3 + c] + SH_C2[2] * 2.f * -x * sh[6 * 3 + c] +
                          SH_C2[3] * z * sh[7 * 3 + c] + SH_C2[4] * 2.f * x * sh[8 * 3 + c];
                ddy[c] += SH_C2[0] * x * sh[4 * 3 + c] + SH_C2[1] * z * sh[5 * 3 + c] +
                          SH_C2[2] * 2.f * -y * sh[6 * 3 + c] + SH_C2[4] * 2.f * -y * sh[8 * 3 + c];
                ddz[c] += SH_C2[1] * y * sh[5 * 3 + c] + SH_C2[2] * 2.f * 2.f * z * sh[6 * 3 + c] +
                          SH_C2[3] * x * sh[7 * 3 + c];
            }
            if (deg > 2) {
                float b9 = SH_C3[0] * y * (3.f * xx - yy), b10 = SH_C3[1] * xy * z,
                      b11 = SH_C3[2] * y * (4.f * zz - xx - yy), b12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy),
                      b13 = SH_C3[4] * x * (4.f * zz - xx - yy), b14 = SH_C3[5] * z * (xx - yy),
                      b15 = SH_C3[6] * x * (xx - 3.f * yy);
                for (int c = 0; c < 3; ++c) {
                    dsh[9 * 3 + c] = b9 * dRGB[c];
                    dsh[10 * 3 + c] = b10 * dRGB[c];
                    dsh[11 * 3 + c] = b11 * dRGB[c];
                    dsh[12 * 3 + c] = b12 * dRGB[c];
                    dsh[13 * 3 + c] = b13 * dRGB[c];
                    dsh[14 * 3 + c] = b14 * dRGB[c];
                    dsh[15 * 3 + c] = b15 * dRGB[c];
                    ddx[c] += (SH_C3[0] * sh[9 * 3 + c] * 3.f * 2.f * xy + SH_C3[1] * sh[10 * 3 + c] * yz +
                               SH_C3[2] * sh[11 * 3 + c] * -2.f * xy + SH_C3[3] * sh[12 * 3 + c] * -3.f * 2.f * xz +
                               SH_C3[4] * sh[13 * 3 + c] * (-3.f * xx + 4.f * zz - yy) +
                               SH_C3[5] * sh[14 * 3 + c] * 2.f * xz + SH_C3[6] * sh[15 * 3 + c] * 3.f * (xx - yy));
                    ddy[c] += (SH_C3[0] * sh[9 * 3 + c] * 3.f * (xx - yy) + SH_C3[1] * sh[10 * 3 + c] * xz +
                               SH_C3[2] * sh[11 * 3 + c] * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3[3] * sh[12 * 3 + c] * -3.f * 2.f * yz + SH_C3[4] * sh[13 * 3 + c] * -2.f * xy +
                               SH_C3[5] * sh[14 * 3 + c] * -2.f * yz + SH_C3[6] * sh[15 * 3 + c] * -3.f * 2.f * xy);
                    ddz[c] += (SH_C3[1] * sh[10 * 3 + c] * xy + SH_C3[2] * sh[11 * 3 + c] * 4.f * 2.f * yz +
                               SH_C3[3] * sh[12 * 3 + c] * 3.f * (2.f * zz - xx - yy) +
                               SH_C3[4] * sh[13 * 3 + c] * 4.f * 2.f * xz + SH_C3[5] * sh[14 * 3 + c] * (xx - yy));
                }
            }
        }
    }
    float dL_ddir[3] = {ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2],
                        ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2],
                        ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2]};
    float dm[3];
    dnormvdv3(dir_orig, dL_ddir, dm);
    dL_dmeans[3 * idx + 0] += dm[0];
    dL_dmeans[3 * idx + 1] += dm[1];
    dL_dmeans[3 * idx + 2] += dm[2];
}

static void cov3d_backward(int idx, const float* scale, float mod, const float* rot, const float* dL_dcov3Ds,
                           float* dL_dscales, float* dL_drots)
{
    float R[3][3], M[3][3];
    rot_matrix(rot, R);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[i][j] = s[i] * R[i][j];
    const float* d = dL_dcov3Ds + 6 * idx;
    float Dm[3][3] = {{d[0], 0.5f * d[1], 0.5f * d[2]}, {0.5f * d[1], d[3], 0.5f * d[4]}, {0.5f * d[2], 0.5f * d[4], d[5]}};
    float dM[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) dM[i][j] = 2.0f * (M[i][0] * Dm[0][j] + M[i][1] * Dm[1][j] + M[i][2] * Dm[2][j]);
    float* ds = dL_dscales + 3 * idx;
    for (int i = 0; i < 3; ++i) ds[i] = R[i][0] * dM[i][0] + R[i][1] * dM[i][1] + R[i][2] * dM[i][2];
    float E[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[i][j] = dM[i][j] * s[i];
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    float* dq = dL_drots + 4 * idx;
    dq[0] = 2 * z * (E[0][1] - E[1][0]) + 2 * y * (E[2][0] - E[0][2]) + 2 * x * (E[1][2] - E[2][1]);
    dq[1] = 2 * y * (E[1][0] + E[0][1]) + 2 * z * (E[2][0] + E[0][2]) + 2 * r * (E[1][2] - E[2][1]) -
            4 * x * (E[2][2] + E[1][1]);
    dq[2] = 2 * x * (E[1][0] + E[0][1]) + 2 * r * (E[2][0] - E[0][2]) + 2 * z * (E[1][2] + E[2][1]) -
            4 * y * (E[2][2] + E[0][0]);
    dq[3] = 2 * r * (E[0][1] - E[1][0]) + 2 * x * (E[2][0] + E[0][2]) + 2 * y * (E[1][2] + E[2][1]) -
            4 * z * (E[1][1] + E[0][0]);
}

/* BACKWARD::preprocess (backward.cu:616-680): computeCov2DCUDA then preprocessCUDA */
void oracle_preprocess_backward(int P, int D, int M, const float* means3D, const int* radii, const float* shs,
                                const uint8_t* clamped, const float* scales, const float* rotations,
                                float scale_modifier, const float* cov3Ds, const float* view, const float* proj,
                                int W, int H, float tan_fovx, float tan_fovy, const float* campos,
                                const float* dL_dmean2D, const float* dL_dconic, const float* dL_dcolor,
                                float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot)
{
    const float h_y = H / (2.0f * tan_fovy), h_x = W / (2.0f * tan_fovx);
    for (int idx = 0; idx < P; ++idx) {
        if (!(radii[idx] > 0)) continue;
        const float* cov3D = cov3Ds + 6 * idx;
        const float* mean = means3D + 3 * idx;
        float dcx = dL_dconic[4 * idx], dcy = dL_dconic[4 * idx + 1], dcz = dL_dconic[4 * idx + 3];
        float t[3], g0[3], g1[3], abc[3];
        int xm, ym;
        cov2d_T(mean, h_x, h_y, tan_fovx, tan_fovy, view, t, g0, g1, &xm, &ym);
        cov2d_from_T(g0, g1, cov3D, abc);
        float a = abc[0], b = abc[1], c = abc[2];
        float denom = a * c - b * b;
        float da = 0, db = 0, dc = 0;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float* dcov = dL_dcov3D + 6 * idx;
        if (denom2inv != 0) {
            da = denom2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
            dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
            db = denom2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
            dcov[0] = (g0[0] * g0[0] * da + g0[0] * g1[0] * db + g1[0] * g1[0] * dc);
            dcov[3] = (g0[1] * g0[1] * da + g0[1] * g1[1] * db + g1[1] * g1[1] * dc);
            dcov[5] = (g0[2] * g0[2] * da + g0[2] * g1[2] * db + g1[2] * g1[2] * dc);
            dcov[1] = 2 * g0[0] * g0[1] * da + (g0[0] * g1[1] + g0[1] * g1[0]) * db + 2 * g1[0] * g1[1] * dc;
            dcov[2] = 2 * g0[0] * g0[2] * da + (g0[0] * g1[2] + g0[2] * g1[0]) * db + 2 * g1[0] * g1[2] * dc;
            dcov[4] = 2 * g0[2] * g0[1] * da + (g0[1] * g1[2] + g0[2] * g1[1]) * db + 2 * g1[1] * g1[2] * dc;
        } else {
            for (int i = 0; i < 6; ++i) dcov[i] = 0;
        }
        /* V column k: (V[k][0], V[k][1], V[k][2]) */
        const float V[3][3] = {{cov3D[0], cov3D[1], cov3D[2]}, {cov3D[1], cov3D[3], cov3D[4]}, {cov3D[2], cov3D[4], cov3D[5]}};
        float dT0[3], dT1[3];
        for (int k = 0; k < 3; ++k) {
            float p0 = g0[0] * V[k][0] + g0[1] * V[k][1] + g0[2] * V[k][2];
            float p1 = g1[0] * V[k][0] + g1[1] * V[k][1] + g1[2] * V[k][2];
            dT0[k] = 2 * p0 * da + p1 * db;
            dT1[k] = 2 * p1 * dc + p0 * db;
        }
        float dJ00 = view[0] * dT0[0] + view[4] * dT0[1] + view[8] * dT0[2];
        float dJ02 = view[2] * dT0[0] + view[6] * dT0[1] + view[10] * dT0[2];
        float dJ11 = view[1] * dT1[0] + view[5] * dT1[1] + view[9] * dT1[2];
        float dJ12 = view[2] * dT1[0] + view[6] * dT1[1] + view[10] * dT1[2];
        float tz = 1.f / t[2], tz2 = tz * tz, tz3 = tz2 * tz;
        float dtx = (float)xm * -h_x * tz2 * dJ02;
        float dty = (float)ym * -h_y * tz2 * dJ12;
        float dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t[0]) * tz3 * dJ02 + (2 * h_y * t[1]) * tz3 * dJ12;
        float v3[3] = {dtx, dty, dtz + dL_dmean2D[3 * idx + 2]};
        float dm[3];
        xform_vec4x3_transpose(v3, view, dm);
        /* preprocessCUDA bwd (backward.cu:372-389) */
        float mh[4];
        xform_point4x4(mean, proj, mh);
        float m_w = 1.0f / (mh[3] + 0.0000001f);
        const float* m = mean;
        float mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * m_w * m_w;
        float gx2 = dL_dmean2D[3 * idx], gy2 = dL_dmean2D[3 * idx + 1];
        dm[0] += (proj[0] * m_w - proj[3] * mul1) * gx2 + (proj[1] * m_w - proj[3] * mul2) * gy2;
        dm[1] += (proj[4] * m_w - proj[7] * mul1) * gx2 + (proj[5] * m_w - proj[7] * mul2) * gy2;
        dm[2] += (proj[8] * m_w - proj[11] * mul1) * gx2 + (proj[9] * m_w - proj[11] * mul2) * gy2;
        dL_dmean3D[3 * idx + 0] = dm[0];
        dL_dmean3D[3 * idx + 1] = dm[1];
        dL_dmean3D[3 * idx + 2] = dm[2];
        if (shs) color_from_sh_backward(idx, D, M, means3D, campos, shs, clamped, dL_dcolor, dL_dmean3D, dL_dsh);
        if (scales) cov3d_backward(idx, scales + 3 * idx, scale_modifier, rotations + 4 * idx, dL_dcov3D, dL_dscale, dL_drot);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* BRDF: render_equation.cu                                                                    */
/* ------------------------------------------------------------------------------------------ */

/* render_equation.cu:17-50 */
static void sh_coef3(const float* d, float* coef)
{
    float x = d[0], y = d[1], z = d[2];
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    coef[0] = SH_C0;
    coef[1] = -SH_C1 * y; coef[2] = SH_C1 * z; coef[3] = -SH_C1 * x;
    coef[4] = SH_C2[0] * xy; coef[5] = SH_C2[1] * yz; coef[6] = SH_C2[2] * (2.0f * zz - xx - yy);
    coef[7] = SH_C2[3] * xz; coef[8] = SH_C2[4] * (xx - yy);
    coef[9] = SH_C3[0] * y * (3.0f * xx - yy); coef[10] = SH_C3[1] * xy * z;
    coef[11] = SH_C3[2] * y * (4.0f * zz - xx - yy); coef[12] = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
    coef[13] = SH_C3[4] * x * (4.0f * zz - xx - yy); coef[14] = SH_C3[5] * z * (xx - yy);
    coef[15] = SH_C3[6] * x * (xx - 3.0f * yy);
}

/* Two statements of the render equation's arithmetic. Default (0): the operation sequence brdf.hip
 * evaluates (shared r3dg_sincosf / r3dg_expf_wide, powers as products, one division per shared
 * denominator) -- the GPU matches it bit for bit. 1: the reference's own sequence as its CUDA source
 * writes it (render_equation.cu:89-161 / 351-403: libm sinf / cosf / expf / powf, every division
 * written out, `2 * ray / (2 Ns - 1)` and `2 pi n_d_i / Ns` as written) -- the check of how far
 * brdf.hip's shared statements sit from the reference's (tests/test_gpu_fullsize.py). */
static int g_brdf_ref_ops = 0;
void oracle_set_brdf_ref_ops(int on) { g_brdf_ref_ops = on; }

/* render_equation.cu:89-113 / 581-606: Fibonacci direction rotated to the normal */
static void fib_dir(const float* n, int ray, int Ns, float rand01, int use_rand, float* dir)
{
    const float delta = PI_F * (3.0f - sqrtf(5.0f));
    const float z = g_brdf_ref_ops ? 1 - 2 * (float)ray / (2 * (float)Ns - 1) : 1 - (float)ray * (2.0f / (2 * (float)Ns - 1));
    const float rad = sqrtf(1 - z * z);
    float theta = delta * ray;
    if (use_rand) theta = rand01 * 2 * PI_F + theta;
    float sn, cs;
    if (g_brdf_ref_ops) {
        sn = sinf(theta);
        cs = cosf(theta);
    } else {
        r3dg_sincosf(theta, &sn, &cs);
    }
    const float y = cs * rad, x = sn * rad;
    float zs[3] = {x, y, z};
    const float v1 = -n[1], v2 = n[0], v3 = 0.f;
    const float v11 = v1 * v1, v22 = v2 * v2, v33 = v3 * v3, v12 = v1 * v2, v13 = v1 * v3, v23 = v2 * v3;
    if (g_brdf_ref_ops) { /* render_equation.cu:106-112, each term divided */
        const float c = fmaxf(n[2] + 1, 0.0000001f);
        float o[3] = {(1 + (-v33 - v22) / c) * zs[0] + (-v3 + v12 / c) * zs[1] + (v2 + v13 / c) * zs[2],
                      (v3 + v12 / c) * zs[0] + (1 + (-v33 - v11) / c) * zs[1] + (-v1 + v23 / c) * zs[2],
                      (-v2 + v13 / c) * zs[0] + (v1 + v23 / c) * zs[1] + (1 + (-v22 - v11) / c) * zs[2]};
        const float norm = sqrtf(fmaxf(0.0000001f, o[0] * o[0] + o[1] * o[1] + o[2] * o[2]));
        dir[0] = o[0] / norm; dir[1] = o[1] / norm; dir[2] = o[2] / norm;
        return;
    }
    /* one division by cp1 and one by norm, then products with the reciprocals (brdf.hip fib_dir; the
     * reference divides each term, render_equation.cu:104-112: within an ulp) */
    const float cp1 = fmaxf(n[2] + 1, 0.0000001f), rc = 1.0f / cp1;
    float o[3] = {(1 + (-v33 - v22) * rc) * zs[0] + (-v3 + v12 * rc) * zs[1] + (v2 + v13 * rc) * zs[2],
                  (v3 + v12 * rc) * zs[0] + (1 + (-v33 - v11) * rc) * zs[1] + (-v1 + v23 * rc) * zs[2],
                  (-v2 + v13 * rc) * zs[0] + (v1 + v23 * rc) * zs[1] + (1 + (-v22 - v11) * rc) * zs[2]};
    const float norm = sqrtf(fmaxf(0.0000001f, o[0] * o[0] + o[1] * o[1] + o[2] * o[2])), rn = 1.0f / norm;
    dir[0] = o[0] * rn; dir[1] = o[1] * rn; dir[2] = o[2] * rn;
}

typedef struct {
    float local[3], global[3], vis, light[3];
    float hdn, hdo, ndi, ndo, fd[3], fs[3], D, F[3], V, half_norm, half[3];
} brdf_sample;

static float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static void brdf_eval(int idx, int S_inc, int S_dir, int S_vis, const float* base, float rough, float metal,
                      const float* n, const float* v, const float* inc, const float* dir_shs, const float* vis_shs,
                      const float* d, const float* coef, brdf_sample* s)
{
    for (int c = 0; c < 3; ++c) s->local[c] = 0.f;
    /* the SH light sums as fmaf chains in coefficient order (brdf.hip eval_lights; nvcc contracts the
     * reference's `+= a * b` the same way) */
    for (int i = 0; i < S_inc; ++i)
        for (int c = 0; c < 3; ++c) s->local[c] = fmaf(inc[((size_t)idx * S_inc + i) * 3 + c], coef[i], s->local[c]);
    for (int c = 0; c < 3; ++c) s->local[c] = fmaxf(s->local[c], 0.0f);
    for (int c = 0; c < 3; ++c) s->global[c] = 0.5f;
    for (int i = 0; i < S_dir; ++i)
        for (int c = 0; c < 3; ++c) s->global[c] = fmaf(dir_shs[i * 3 + c], coef[i], s->global[c]);
    for (int c = 0; c < 3; ++c) s->global[c] = fmaxf(s->global[c], 0.0f);
    float vis = 0.5f;
    for (int i = 0; i < S_vis; ++i) vis = fmaf(vis_shs[(size_t)idx * S_vis + i], coef[i], vis);
    s->vis = fmaxf(0.0f, fminf(vis, 1.0f));
    for (int c = 0; c < 3; ++c) s->light[c] = fmaf(s->vis, s->global[c], s->local[c]);
    float h[3] = {d[0] + v[0], d[1] + v[1], d[2] + v[2]};
    s->half_norm = fmaxf(sqrtf(dot3(h, h)), 0.0000001f);
    const float rh = 1.0f / s->half_norm;
    for (int c = 0; c < 3; ++c) s->half[c] = g_brdf_ref_ops ? h[c] / s->half_norm : h[c] * rh;
    s->hdn = fmaxf(dot3(s->half, n), 0.0f);
    s->hdo = fmaxf(dot3(s->half, v), 0.0f);
    s->ndi = fmaxf(dot3(n, d), 0.0f);
    s->ndo = fmaxf(dot3(n, v), 0.0f);
    for (int c = 0; c < 3; ++c) s->fd[c] = (1 - metal) * base[c] / PI_F;
    float r2 = fmaxf(rough * rough, 0.0000001f);
    float amp = 1.0f / (r2 * PI_F), sharp = 2.0f / r2;
    s->D = amp * (g_brdf_ref_ops ? expf(sharp * (s->hdn - 1.0f)) : r3dg_expf_wide(sharp * (s->hdn - 1.0f)));
    /* powf(1 - h_d_o, 5) (render_equation.cu:155): CUDA powf's bits are implementation-defined;
     * stated as products (t^2)^2 t, as brdf.hip */
    const float t1 = 1.0f - s->hdo, t2 = t1 * t1;
    float p5 = g_brdf_ref_ops ? powf(t1, 5.0f) : t2 * t2 * t1;
    for (int c = 0; c < 3; ++c) {
        float F0 = 0.04f * (1.0f - metal) + base[c] * metal;
        s->F[c] = F0 + (1.0f - F0) * p5;
    }
    float r2v = g_brdf_ref_ops ? powf(1.0f + rough, 2.0f) / 8.0f
                               : (1.0f + rough) * (1.0f + rough) / 8.0f; /* __powf(1 + rough, 2) / 8 (:158) */
    s->V = (0.5f / fmaxf(s->ndi * (1 - r2v) + r2v, 0.0000001f)) * (0.5f / fmaxf(s->ndo * (1 - r2v) + r2v, 0.0000001f));
    for (int c = 0; c < 3; ++c) s->fs[c] = s->D * s->F[c] * s->V;
}

/* render_equation.cu:552-663 (training forward; rand_float may be NULL when !is_training) */
void oracle_render_equation_forward(int P, int S_inc, int S_dir, int S_vis, const float* base, const float* rough,
                                    const float* metal, const float* normals, const float* viewdirs,
                                    const float* inc, const float* dir_shs, const float* vis_shs, int Ns,
                                    int is_training, const float* rand_float, float* incident_dirs, float* pbr,
                                    float* diffuse)
{
    for (int idx = 0; idx < P; ++idx) {
        float acc_p[3] = {0, 0, 0}, acc_d[3] = {0, 0, 0};
        for (int r = 0; r < Ns; ++r) {
            float d[3], coef[16];
            fib_dir(normals + 3 * idx, r, Ns, is_training ? rand_float[(size_t)idx * Ns + r] : 0.f, is_training, d);
            sh_coef3(d, coef);
            brdf_sample s;
            brdf_eval(idx, S_inc, S_dir, S_vis, base + 3 * idx, rough[idx], metal[idx], normals + 3 * idx,
                      viewdirs + 3 * idx, inc, dir_shs, vis_shs, d, coef, &s);
            float tmp = g_brdf_ref_ops ? 2.0f * PI_F * s.ndi / (float)Ns : s.ndi * (2.0f * PI_F / (float)Ns);
            for (int c = 0; c < 3; ++c) {
                float tr = s.light[c] * tmp;
                acc_p[c] += (s.fd[c] + s.fs[c]) * tr;
                acc_d[c] += tr;
            }
            for (int c = 0; c < 3; ++c) incident_dirs[((size_t)idx * Ns + r) * 3 + c] = d[c];
        }
        for (int c = 0; c < 3; ++c) { pbr[3 * idx + c] = acc_p[c]; diffuse[3 * idx + c] = acc_d[c]; }
    }
}

/* render_equation.cu:52-187 (eval forward with per-sample outputs) */
void oracle_render_equation_forward_complex(int P, int S_inc, int S_dir, int S_vis, const float* base,
                                            const float* rough, const float* metal, const float* normals,
                                            const float* viewdirs, const float* inc, const float* dir_shs,
                                            const float* vis_shs, int Ns, float* incident_dirs, float* pbr,
                                            float* lights, float* local_lights, float* global_lights, float* vis,
                                            float* diffuse, float* local_diffuse, float* accum, float* rgb_d,
                                            float* rgb_s)
{
    for (int idx = 0; idx < P; ++idx) {
        float ad[3] = {0, 0, 0}, as[3] = {0, 0, 0}, dl[3] = {0, 0, 0}, ldl[3] = {0, 0, 0};
        for (int r = 0; r < Ns; ++r) {
            float d[3], coef[16];
            fib_dir(normals + 3 * idx, r, Ns, 0.f, 0, d);
            sh_coef3(d, coef);
            brdf_sample s;
            brdf_eval(idx, S_inc, S_dir, S_vis, base + 3 * idx, rough[idx], metal[idx], normals + 3 * idx,
                      viewdirs + 3 * idx, inc, dir_shs, vis_shs, d, coef, &s);
            float tmp = g_brdf_ref_ops ? 2.0f * PI_F * s.ndi / (float)Ns : s.ndi * (2.0f * PI_F / (float)Ns);
            size_t w = (size_t)idx * Ns + r;
            for (int c = 0; c < 3; ++c) {
                float g = s.vis * s.global[c];
                float tr = s.light[c] * tmp, ltr = s.local[c] * tmp;
                dl[c] += tr;
                ldl[c] += ltr;
                ad[c] += s.fd[c] * tr;
                as[c] += s.fs[c] * tr;
                incident_dirs[w * 3 + c] = d[c];
                lights[w * 3 + c] = s.light[c];
                local_lights[w * 3 + c] = s.local[c];
                global_lights[w * 3 + c] = g;
            }
            vis[w] = s.vis;
        }
        float av[3];
        for (int c = 0; c < 3; ++c) av[c] = dl[c] * INV_PI_F + as[c];
        accum[idx] = (av[0] + av[1] + av[2]) / 3;
        for (int c = 0; c < 3; ++c) {
            pbr[3 * idx + c] = ad[c] + as[c];
            rgb_d[3 * idx + c] = ad[c];
            rgb_s[3 * idx + c] = as[c];
            diffuse[3 * idx + c] = dl[c];
            local_diffuse[3 * idx + c] = ldl[c];
        }
    }
}

/* render_equation.cu:277-460, bug-compatible except the dL_ddirect_shs race (sequential sum). */
void oracle_render_equation_backward(int P, int S_inc, int S_dir, int S_vis, const float* base, const float* rough,
                                     const float* metal, const float* normals, const float* viewdirs,
                                     const float* inc, const float* dir_shs, const float* vis_shs, int Ns,
                                     const float* incident_dirs, const float* dL_dpbr, const float* dL_ddiff,
                                     float* d_base, float* d_rough, float* d_metal, float* d_normal, float* d_view,
                                     float* d_inc, float* d_dir, float* d_vis)
{
    if (S_dir > 16 || S_inc > 16 || S_vis > 16) { /* computeSHcoef gives 16 coefficients (degree 3) */
        fprintf(stderr, "oracle_render_equation_backward: S_dir / S_inc / S_vis must be <= 16\n");
        abort();
    }
    const float K = 2.0f * PI_F / (float)Ns;
    /* dL_ddirect_shs: the reference's racy float += over every (Gaussian, sample) (:443-445) has
     * no defined value; here it is the exact sum (double accumulation, rounded once), which any
     * fixed-order float reduction approaches to its own rounding */
    double ddir_acc[16 * 3] = {0};
    for (int idx = 0; idx < P; ++idx) {
        const float* n = normals + 3 * idx;
        const float* v = viewdirs + 3 * idx;
        const float* b = base + 3 * idx;
        const float metal_i = metal[idx], rough_i = rough[idx];
        const float* gp = dL_dpbr + 3 * idx;
        const float* gdl = dL_ddiff + 3 * idx;
        for (int r = 0; r < Ns; ++r) {
            const float* d = incident_dirs + ((size_t)idx * Ns + r) * 3;
            float coef[16];
            sh_coef3(d, coef);
            brdf_sample s;
            brdf_eval(idx, S_inc, S_dir, S_vis, b, rough_i, metal_i, n, v, inc, dir_shs, vis_shs, d, coef, &s);
            float r2 = fmaxf(rough_i * rough_i, 0.0000001f);
            float amp = 1.0f / (r2 * PI_F), sharp = 2.0f / r2;
            float e_amp = g_brdf_ref_ops ? expf(sharp * (s.hdn - 1.0f)) : r3dg_expf_wide(sharp * (s.hdn - 1.0f));
            float r2v = g_brdf_ref_ops ? powf(1.0f + rough_i, 2.0f) / 8.0f
                                       : (1.0f + rough_i) * (1.0f + rough_i) / 8.0f; /* powf(1 + rough, 2) / 8 (:359) */
            float den1 = fmaxf(s.ndi * (1 - r2v) + r2v, 0.0000001f);
            float den2 = fmaxf(s.ndo * (1 - r2v) + r2v, 0.0000001f);
            float g1 = 0.5f / den1, g2 = 0.5f / den2;
            const float Tn = s.ndi * (2.0f * PI_F / (float)Ns);
            float dfd[3], dfs[3], dli[3], fsum[3];
            for (int c = 0; c < 3; ++c) {
                fsum[c] = s.fd[c] + s.fs[c];
                dfd[c] = gp[c] * s.light[c] * Tn;
                dfs[c] = gp[c] * s.light[c] * Tn;
                dli[c] = gp[c] * fsum[c] * Tn;
            }
            float dndi = (gp[0] * (fsum[0] * s.light[0]) + gp[1] * (fsum[1] * s.light[1]) + gp[2] * (fsum[2] * s.light[2])) * K;
            for (int c = 0; c < 3; ++c) dli[c] += gdl[c] * Tn;
            dndi += gdl[0] * (s.light[0] * K) + gdl[1] * (s.light[1] * K) + gdl[2] * (s.light[2] * K);
            float dbase[3];
            for (int c = 0; c < 3; ++c) dbase[c] = dfd[c] * ((1 - metal_i) / PI_F);
            float dmetal = -(dfd[0] * b[0] + dfd[1] * b[1] + dfd[2] * b[2]) * INV_PI_F;
            float dD = dfs[0] * s.V * s.F[0] + dfs[1] * s.V * s.F[1] + dfs[2] * s.V * s.F[2];
            float dF[3];
            for (int c = 0; c < 3; ++c) dF[c] = dfs[c] * s.D * s.V;
            float dV = dfs[0] * s.D * s.F[0] + dfs[1] * s.D * s.F[1] + dfs[2] * s.D * s.F[2];
            float damp = dD * e_amp, de = dD * amp;
            float dsharp = (s.hdn - 1.0f) * e_amp * de;
            float dhdn = sharp * e_amp * de;
            float dr2 = -2.0f / (r2 * r2) * dsharp - 1.0f / (r2 * r2 * PI_F) * damp;
            float drough = dr2 * 2.0f * rough_i;
            /* powf(1 - h_d_o, 5 / 4) (:394-395) as products, as brdf_eval */
            const float t1 = 1.0f - s.hdo, t2 = t1 * t1;
            float p4 = g_brdf_ref_ops ? powf(t1, 4.0f) : t2 * t2, p5 = g_brdf_ref_ops ? powf(t1, 5.0f) : p4 * t1;
            float dF0[3], dhdo = 0;
            for (int c = 0; c < 3; ++c) {
                float F0 = 0.04f * (1.0f - metal_i) + b[c] * metal_i;
                dF0[c] = (1.0f - p5) * dF[c];
                dhdo += (1.0f - F0) * dF[c];
            }
            dhdo = dhdo * -5.0f * p4;
            for (int c = 0; c < 3; ++c) dbase[c] += metal_i * dF0[c];
            dmetal += (b[0] - 0.04f) * dF0[0] + (b[1] - 0.04f) * dF0[1] + (b[2] - 0.04f) * dF0[2];
            float dg1 = dV * g2, dg2 = dV * g1;
            float dden1 = g_brdf_ref_ops ? -0.5f / (den1 * den1) * dg1 : -2.0f * (g1 * g1) * dg1; /* -0.5/den1^2 = -2 g1^2 */
            float dden2 = -0.5f / (den2 * den2) * dg2;
            dndi = dden1 * (1 - r2v); /* overwrite: render_equation.cu:403 (bug-compatible) */
            float dndo = dden2 * (1 - r2v);
            float dr2v = (1.0f - s.ndi) * dden1 + (1.0f - s.ndo) * dden2;
            drough += (1.0f + rough_i) / 4.0f * dr2v;
            float dhalf[3] = {0, 0, 0}, dn[3] = {0, 0, 0}, dv[3] = {0, 0, 0};
            if (s.hdn > 0.0f) for (int c = 0; c < 3; ++c) { dhalf[c] += n[c] * dhdn; dn[c] += s.half[c] * dhdn; }
            if (s.hdo > 0.0f) for (int c = 0; c < 3; ++c) { dhalf[c] += v[c] * dhdo; dv[c] += s.half[c] * dhdo; }
            if (s.ndi > 0.0f) for (int c = 0; c < 3; ++c) dn[c] += d[c] * dndi;
            if (s.ndo > 0.0f) for (int c = 0; c < 3; ++c) { dn[c] += v[c] * dndo; dv[c] += n[c] * dndo; }
            const float rh = 1.0f / s.half_norm;
            for (int c = 0; c < 3; ++c) dv[c] += g_brdf_ref_ops ? dhalf[c] / s.half_norm : dhalf[c] * rh;
            float dglob[3], dvis_s = 0;
            for (int c = 0; c < 3; ++c) dglob[c] = dli[c] * s.vis;
            for (int c = 0; c < 3; ++c) dvis_s += dli[c] * s.global[c];
            for (int i = 0; i < S_vis; ++i) d_vis[(size_t)idx * S_vis + i] = fmaf(dvis_s, coef[i], d_vis[(size_t)idx * S_vis + i]);
            /* clamp checks after fmaxf never fire (render_equation.cu:440-449, bug-compatible) */
            for (int i = 0; i < S_dir; ++i)
                for (int c = 0; c < 3; ++c) ddir_acc[i * 3 + c] += (double)dglob[c] * (double)coef[i];
            for (int i = 0; i < S_dir; ++i) /* loop bound S_direct, render_equation.cu:450 */
                for (int c = 0; c < 3; ++c)
                    d_inc[((size_t)idx * S_inc + i) * 3 + c] = fmaf(dli[c], coef[i], d_inc[((size_t)idx * S_inc + i) * 3 + c]);
            for (int c = 0; c < 3; ++c) {
                d_view[3 * idx + c] += dv[c];
                d_normal[3 * idx + c] += dn[c];
                d_base[3 * idx + c] += dbase[c];
            }
            d_metal[idx] += dmetal;
            d_rough[idx] += drough;
        }
    }
    for (int i = 0; i < S_dir; ++i)
        for (int c = 0; c < 3; ++c) d_dir[i * 3 + c] += (float)ddir_acc[i * 3 + c];
}

/* batch entry points for the golden-vector tests of the per-Gaussian sub-steps */
void oracle_color_from_sh_batch(int P, int deg, int M, const float* means, const float* campos, const float* shs,
                                float* rgb, uint8_t* clamped)
{
    for (int i = 0; i < P; ++i) color_from_sh(i, deg, M, means, campos, shs, clamped, rgb + 3 * i);
}

void oracle_cov3d_batch(int P, const float* scales, float mod, const float* rotations, float* cov3D)
{
    for (int i = 0; i < P; ++i) compute_cov3d(scales + 3 * i, mod, rotations + 4 * i, cov3D + 6 * i);
}
