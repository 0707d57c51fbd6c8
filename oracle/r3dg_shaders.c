/* r3dg_shaders.c -- CPU oracle for the shader library and texture sampling. TEST
 * INFRASTRUCTURE ONLY (tests/ and smoke()); never linked into the product.
 *
 * Restates r3dg-rasterization/cuda_rasterizer/ShShader.cu:62-190 (SH shaders),
 * splatShader.cu:33-52 (per-splat views), :67-269 (splat shaders), utils/shaderUtils.cu:147-155
 * (Quantize) and the CUDA texture-unit behaviour the shaders rely on through utils/texture.cu
 * (tex2D on float textures: normalized coordinates, wrap/clamp/mirror/border, bilinear weights in
 * 8-bit fixed point; point sampling for LAB/HSV). glm semantics: dot = x*x'+y*y'+z*z',
 * normalize(v) = v * (1/sqrt(dot(v,v))), length = sqrt(dot), mix(x,y,a) = x*(1-a)+y*a and the
 * bool overload of mix is a select. Parity note: the reference has no fixtures for shaders or
 * textures, and the hardware rounding of CUDA's fixed-point texture weights is not published
 * (round-to-nearest assumed): shader parity is pinned only by this restatement.
 * Post-process passes: postProcessShader.cu:13-374 with RunPostProcessShaders' double buffer
 * (forward.cu:973-1047) restated literally; helpers from shaderUtils.cu:6-161.
 * Build: oracle/Makefile (-ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846 /* the CUDA math constants the reference uses */
#endif
#ifndef M_1_PI
#define M_1_PI 0.31830988618379067154
#endif

typedef struct {
    const float* texels; /* [H, W, 4] */
    int W, H, wrap_u, wrap_v, normalized, linear;
} otex;

static int tex_index(int i, int n, int mode, int normalized, int* zero)
{
    if (mode == 3) { /* border */
        if (i < 0 || i >= n) *zero = 1;
        return i < 0 ? 0 : (i >= n ? n - 1 : i);
    }
    if (normalized && mode == 0) { /* wrap */
        i %= n;
        return i < 0 ? i + n : i;
    }
    if (normalized && mode == 2) { /* mirror */
        int p = 2 * n;
        i %= p;
        if (i < 0) i += p;
        return i < n ? i : p - 1 - i;
    }
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

static void tex_fetch(const otex* t, int i, int j, float* o)
{
    int zero = 0;
    int x = tex_index(i, t->W, t->wrap_u, t->normalized, &zero);
    int y = tex_index(j, t->H, t->wrap_v, t->normalized, &zero);
    if (zero) { o[0] = o[1] = o[2] = o[3] = 0.f; return; }
    memcpy(o, t->texels + 4 * ((size_t)y * t->W + x), 4 * sizeof(float));
}

void oracle_tex_sample(const otex* t, float x, float y, float* o)
{
    float u = t->normalized ? x * (float)t->W : x;
    float v = t->normalized ? y * (float)t->H : y;
    if (!t->linear) { tex_fetch(t, (int)floorf(u), (int)floorf(v), o); return; }
    float ub = u - 0.5f, vb = v - 0.5f;
    float fu = floorf(ub), fv = floorf(vb);
    int i = (int)fu, j = (int)fv;
    float a = rintf((ub - fu) * 256.0f) * (1.0f / 256.0f);
    float b = rintf((vb - fv) * 256.0f) * (1.0f / 256.0f);
    float t00[4], t10[4], t01[4], t11[4];
    tex_fetch(t, i, j, t00); tex_fetch(t, i + 1, j, t10);
    tex_fetch(t, i, j + 1, t01); tex_fetch(t, i + 1, j + 1, t11);
    float w00 = (1.f - a) * (1.f - b), w10 = a * (1.f - b), w01 = (1.f - a) * b, w11 = a * b;
    for (int c = 0; c < 4; ++c) o[c] = w00 * t00[c] + w10 * t10[c] + w01 * t01[c] + w11 * t11[c];
}

/* batch hook for tests */
void oracle_tex_sample_batch(const otex* t, int n, const float* xy, float* out)
{
    for (int k = 0; k < n; ++k) oracle_tex_sample(t, xy[2 * k], xy[2 * k + 1], out + 4 * k);
}

static float sat(float x) { return x != x ? 0.f : fminf(fmaxf(x, 0.f), 1.f); } /* __saturatef */
static float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static float len3(const float* a) { return sqrtf(dot3(a, a)); }

static float tri_planar(const otex* t, const float* p, int invert, int product)
{
    float o[4], a, b, c;
    oracle_tex_sample(t, p[0], p[1], o); a = o[0];
    oracle_tex_sample(t, p[0], p[2], o); b = o[0];
    oracle_tex_sample(t, p[1], p[2], o); c = o[0];
    if (invert) { a = 1 - a; b = 1 - b; c = 1 - c; }
    return product ? a * b * c : (a + b + c) / 3;
}

static float heartbeat(float t) /* ShShader.cu:109-118 (double arithmetic, M_PI) */
{
    const double k = M_PI * 4.0 / 3.0;
    double m = fmod((double)t, k);
    double up = round(sin(m) / 2 + 0.5);
    return (float)((1 + cos(m) * up + cos(m * 3) * (1 - up)) / 2);
}

enum { SH_CULLHALF = 0, SH_EXPPOS = 1, SH_GAUSSDISSOLVE = 2, SH_HEARTBEAT = 3, SH_DEFAULT = 4 };

/* One SH shader over the splat indices idx[0..n) (ExecuteSHShaderCUDA, ShShader.cu:233-249). */
void oracle_sh_shader(int id, int n, const int* idx, float time, float* pos, float* scale, float* rot,
                      float* opacity, float* sh, int M, const float* features, int S, const otex* tex0,
                      const otex* tex1)
{
    (void)rot;
    for (int k = 0; k < n; ++k) {
        int g = idx[k];
        float* p = pos + 3 * (size_t)g;
        float* s = scale + 3 * (size_t)g;
        if (id == SH_EXPPOS) { /* :67-77 */
            float posY = fabsf(p[1]);
            float ns[3] = {s[0] * posY * posY, s[1] * 2 * posY, s[2] * posY};
            float np[3] = {p[0] * posY * posY, p[1] * 2 * posY, p[2] * posY};
            memcpy(s, ns, sizeof ns);
            memcpy(p, np, sizeof np);
        } else if (id == SH_HEARTBEAT) { /* :82-138 */
            float atrial = tri_planar(tex0, p, 0, 0);
            float ventricular = tri_planar(tex1, p, 1, 0);
            float pulsePeriod = 1, distInfluence = -0.5f;
            float t = time / 1000 / pulsePeriod + len3(p) * distInfluence;
            float aG = heartbeat(t) * atrial;
            float vG = heartbeat(t - 0.9f) * ventricular;
            const float* nrm = features + (size_t)g * S + 6;
            for (int c = 0; c < 3; ++c) {
                float aP = nrm[c] * aG * 0.025f, vP = nrm[c] * vG * 0.025f;
                p[c] = p[c] + aP + vP;
                s[c] = s[c] + aG * 0.0025f + vG * 0.0025f;
            }
        } else if (id == SH_CULLHALF) { /* :141-149 */
            if (p[0] < 0) {
                opacity[g] = 0;
                s[0] = s[1] = s[2] = 0;
            }
        } else if (id == SH_GAUSSDISSOLVE) { /* :152-188 */
            float mask = tri_planar(tex0, p, 0, 1);
            mask = sat((float)(((double)mask - 0.125) * 1.5));
            float loadingSpeed = 0.25f, loopDuration = 3;
            float total = fmodf(time / 1000 * loadingSpeed, loopDuration);
            float lp = sat(total - p[2] + mask - 1);
            opacity[g] *= lp * lp * lp;
            float fade = len3(s) * 10;
            float start[3] = {p[0] + 0.f * fade, p[1] + 0.f * fade, p[2] + 1.f * fade};
            for (int c = 0; c < 3; ++c) p[c] = start[c] * (1.0f - lp) + p[c] * lp;
            float* sh0 = sh + (size_t)g * M * 3;
            const float tgt[3] = {0.6f, 0.9f, 1.0f};
            for (int c = 0; c < 3; ++c) sh0[c] = tgt[c] * (1.0f - lp) + sh0[c] * lp;
        }
    }
}

enum {
    SP_CRACK = 0, SP_CRACKNORECON = 1, SP_DISSOLVE = 2, SP_NAIVEOUTLINE = 3, SP_QUANTIZEFLATS = 4,
    SP_QUANTIZELIGHT = 5, SP_ROUGHNESSONLY = 6, SP_DEFAULT = 7, SP_STENCIL = 8, SP_WIREFRAME = 9
};

static float outline_opacity(const float* cam, const float* p, const float* n)
{
    float d[3] = {cam[0] - p[0], cam[1] - p[1], cam[2] - p[2]};
    float id = 1.0f / sqrtf(dot3(d, d)), in = 1.0f / sqrtf(dot3(n, n));
    float dn[3] = {d[0] * id, d[1] * id, d[2] * id}, nn[3] = {n[0] * in, n[1] * in, n[2] * in};
    float angle = 1 - fabsf(dot3(dn, nn));
    return angle < 0.5 ? 1 - 16 * powf(angle, 5.0f) : powf(-2 * angle + 2, 5.0f) / 2;
}

/* One splat shader over idx[0..n) (ExecuteSplatShaderCUDA, splatShader.cu:336-357). conic_opacity
 * [P,4] (opacity at .w), features [P,S] (the reference's views at +0..+20), out_rgb [P,3]. */
void oracle_splat_shader(int id, int n, const int* idx, int W, int H, float time, const float* pos,
                         const float* means2D, const float* depth_tex, const float* viewmatrix_inv,
                         const float* depths, const float* rgb, float* conic_opacity, float* features, int S,
                         float* stencils, float* stencil_opacity, float* out_rgb, const otex* tex0)
{
    const float cam[3] = {viewmatrix_inv[12], viewmatrix_inv[13], viewmatrix_inv[14]};
    for (int k = 0; k < n; ++k) {
        int g = idx[k];
        const float* p = pos + 3 * (size_t)g;
        const float* col = rgb + 3 * (size_t)g;
        float* out = out_rgb + 3 * (size_t)g;
        float* op = conic_opacity + 4 * (size_t)g + 3;
        float* F = features + (size_t)g * S;
        int mp = (int)((float)W * floorf(means2D[2 * g + 1]) + floorf(means2D[2 * g]));
        mp = mp < 0 ? 0 : (mp >= W * H ? W * H - 1 : mp);
        if (id == SP_DEFAULT) {
            memcpy(out, col, 3 * sizeof(float));
        } else if (id == SP_NAIVEOUTLINE) {
            float o = outline_opacity(cam, p, F + 6);
            for (int c = 0; c < 3; ++c) out[c] = col[c] * o;
        } else if (id == SP_WIREFRAME) {
            float o = outline_opacity(cam, p, F + 6);
            for (int c = 0; c < 3; ++c) out[c] = 1 - o;
        } else if (id == SP_DISSOLVE) {
            float mask = tri_planar(tex0, p, 0, 1);
            mask = sat((float)(((double)mask - 0.125) * 1.5));
            float period = 0.1f;
            float o = cosf((float)((double)(time * period * 4) / (M_1_PI * 2 * 1000))) + 1;
            float masked = sat(o - (1 - mask));
            *op = *op * masked;
            float fading = sat(masked * 3);
            stencils[g] = mask;
            const float tgt[3] = {0.6f, 0.9f, 1.0f};
            for (int c = 0; c < 3; ++c) out[c] = tgt[c] * (1.0f - fading) + col[c] * fading;
        } else if (id == SP_CRACK || id == SP_CRACKNORECON) {
            float texScale = 2;
            float u = (float)((double)(p[0] / texScale) - 0.5), v = (float)((double)(p[1] / texScale) - 0.5);
            float o4[4];
            oracle_tex_sample(tex0, u, v, o4);
            float ctd = 1 - o4[0];
            float maxCrackDepth = 2, projectionHeight = 2;
            float crackHeight = projectionHeight - ctd * maxCrackDepth;
            float splatHeight = p[2];
            int reaches = crackHeight < splatHeight;
            if (id == SP_CRACK) {
                *op = reaches ? 0 : *op;
                float dist = depths[g] - depth_tex[mp] + 0.3f;
                int inside = dist > 0;
                float icr = 0.1f;
                float maxPrimary = projectionHeight - (ctd + icr) * maxCrackDepth;
                int useInternal = inside && (splatHeight > maxPrimary);
                int icp = sat(dist * 10) != 0.0f;
                float internal[3];
                for (int c = 0; c < 3; ++c) internal[c] = icp ? (c < 2 ? 0.5f : 0.f) : F[9 + c];
                float dr = 0.1f;
                float maxDiscolor = maxPrimary - dr * maxCrackDepth;
                float disc = sat((splatHeight - maxDiscolor) / (dr + icr));
                for (int c = 0; c < 3; ++c) {
                    float ext = col[c] * (1.0f - disc) + internal[c] * disc;
                    out[c] = internal[c] * (float)useInternal + ext * (float)!useInternal;
                }
                *op += 0.2f * (float)useInternal * (float)!reaches;
            } else {
                float orig = *op;
                *op = reaches ? 0 : *op;
                float rel = depths[g] - depth_tex[mp] + 0.2f;
                int inside = rel > 0;
                float icr = 0.5f * ctd;
                float maxPrimary = projectionHeight - (ctd + icr) * maxCrackDepth;
                int useInternal = inside && (maxPrimary < splatHeight);
                memcpy(out, F + 9, 3 * sizeof(float));
                stencils[g] = (float)reaches;
                stencil_opacity[g] = orig;
                F[1] = (float)useInternal;
            }
        } else if (id == SP_STENCIL) {
            stencils[g] = 1;
            stencil_opacity[g] = *op;
            memcpy(out, col, 3 * sizeof(float));
        } else if (id == SP_ROUGHNESSONLY) {
            F[0] = p[0] < 0 ? 0.25f : 0.75f;
            F[1] = 0;
            F[2] = 0;
            for (int c = 0; c < 3; ++c) F[6 + c] = F[9 + c] = F[12 + c] = F[15 + c] = F[18 + c] = 0;
            out[0] = out[1] = out[2] = 0;
        } else if (id == SP_QUANTIZEFLATS) {
            memcpy(out, F + 9, 3 * sizeof(float));
        } else if (id == SP_QUANTIZELIGHT) {
            float qr = roundf(F[12] * 3) / 3, qg = roundf(F[13] * 3) / 3, qb = roundf(F[14] * 3) / 3;
            F[0] = fmaxf(qr, fmaxf(qg, qb));
            memcpy(out, F + 9, 3 * sizeof(float));
        }
    }
}

/* ---- post-process passes ------------------------------------------------------------------ */
enum {
    PP_BLURLIGHTING = 0, PP_CRACKRECON = 1, PP_INVERT = 2, PP_OUTLINE = 3, PP_QUANTIZELIGHTING = 4,
    PP_SOBEL = 5, PP_DEFAULT = 6, PP_TEXTUREDSHADOWS = 7, PP_TOON = 8
};

static void rgb_to_hsv(const float* c, float* hsv) /* shaderUtils.cu:6-37 */
{
    float mx = fmaxf(c[0], fmaxf(c[1], c[2])), mn = fminf(c[0], fminf(c[1], c[2]));
    float diff = mx - mn;
    hsv[2] = mx;
    if (hsv[2] == 0.0f) {
        hsv[0] = hsv[1] = 0.0f;
    } else {
        hsv[1] = diff / hsv[2];
        if (diff < 0.001f) {
            hsv[0] = 0.0f;
        } else if (mx == c[0]) {
            hsv[0] = (c[1] - c[2]) / diff / 6;
            if (hsv[0] < 0.0f) hsv[0] += 1.0f;
        } else if (mx == c[1]) {
            hsv[0] = (2 + (c[2] - c[0]) / diff) / 6;
        } else {
            hsv[0] = (4 + (c[0] - c[1]) / diff) / 6;
        }
    }
}

static void hsv_to_rgb(const float* hsv, float* o) /* shaderUtils.cu:41-82 */
{
    float h = hsv[0], s = hsv[1], v = hsv[2];
    float f = h * 6, hi = floorf(f);
    f = f - hi;
    float p = v * (1 - s), q = v * (1 - s * f), t = v * (1 - s * (1 - f));
    float r, g, b;
    if (hi == 0.0f || hi == 6.0f) { r = v; g = t; b = p; }
    else if (hi == 1.0f) { r = q; g = v; b = p; }
    else if (hi == 2.0f) { r = p; g = v; b = t; }
    else if (hi == 3.0f) { r = p; g = q; b = v; }
    else if (hi == 4.0f) { r = t; g = p; b = v; }
    else { r = v; g = p; b = q; }
    o[0] = r; o[1] = g; o[2] = b;
}

static const float kBlend[5][5] = {{0.009375f, 0.01875f, 0.028125f, 0.01875f, 0.009375f},
                                   {0.01875f, 0.0375f, 0.045f, 0.0375f, 0.01875f},
                                   {0.028125f, 0.045f, 0.3f, 0.045f, 0.028125f},
                                   {0.01875f, 0.0375f, 0.045f, 0.0375f, 0.01875f},
                                   {0.009375f, 0.01875f, 0.028125f, 0.01875f, 0.009375f}};

/* PostProcessShaderBuffer views (postProcessShader.cu:13-105) */
typedef struct {
    float *features, *metallic, *incident, *base, *opacity, *depth, *stencil, *xyz, *normal, *shader, *sh;
} pp_buf;

static pp_buf pp_views(float* features, float* opacity, float* depth, float* stencil, float* xyz, float* normal,
                       float* shader, float* sh, long HW)
{
    pp_buf b;
    b.features = features;
    b.metallic = features ? features + HW : NULL;
    b.base = features ? features + 9 * HW : NULL;
    b.incident = features ? features + 12 * HW : NULL;
    b.opacity = opacity; b.depth = depth; b.stencil = stencil; b.xyz = xyz; b.normal = normal;
    b.shader = shader; b.sh = sh;
    return b;
}

static void pp_color_correction(const pp_buf* in, const pp_buf* out, long p) /* :276-289 */
{
    float hsv[3], color[3];
    rgb_to_hsv(in->base + 3 * p, hsv);
    hsv[0] = roundf(hsv[0] * 24) / 24;
    hsv_to_rgb(hsv, color);
    float intensity = in->incident[3 * p];
    float reduced = sat(intensity + 0.25f);
    for (int c = 0; c < 3; ++c) out->shader[3 * p + c] = color[c] * reduced;
}

static void pp_textured_shadows(const pp_buf* in, const pp_buf* out, long p, int x, int y, int W, int H,
                                const otex* shadow) /* :238-274 */
{
    if (in->stencil[p] < 0.01f) {
        for (int c = 0; c < 3; ++c) out->shader[3 * p + c] = 1.0f;
        return;
    }
    float uvScale = 10;
    float u = (float)x / (float)W * uvScale, v = (float)y / (float)H * uvScale;
    float t[4];
    oracle_tex_sample(shadow, u, v, t);
    float lightShadow = 1 - t[0], mediumShadow = 1 - t[2], heavyShadow = 1 - t[1];
    const float* L = in->incident + 3 * p;
    float m = L[1] > L[2] ? L[1] : L[2]; /* __max */
    float intensity = L[0] > m ? L[0] : m;
    intensity = roundf(intensity * 4);
    heavyShadow = sat(heavyShadow + intensity);
    intensity = 0 > intensity - 1.0f ? 0 : intensity - 1.0f;
    mediumShadow = sat(mediumShadow + intensity);
    intensity = 0 > intensity - 1.0f ? 0 : intensity - 1.0f;
    lightShadow = sat(lightShadow + intensity);
    for (int c = 0; c < 3; ++c) out->shader[3 * p + c] = out->shader[3 * p + c] * lightShadow * mediumShadow * heavyShadow;
}

static void pp_sobel(const pp_buf* in, const pp_buf* out, long p, int W) /* :304-331 */
{
    const float SH[3][3] = {{-1, 0, 1}, {-2, 0, 2}, {-1, 0, 1}};
    const float SV[3][3] = {{-1, -2, -1}, {0, 0, 0}, {1, 2, 1}};
    float outlineStrength = 2, hori = 0, vert = 0;
    for (int x = -1; x < 2; x++)
        for (int y = -1; y < 2; y++) {
            long sp = p + x + (long)y * W;
            float d = in->depth[sp]; /* unclamped: neighbouring planes of the input buffer */
            hori += SH[x + 1][y + 1] * d * outlineStrength;
            vert += SV[x + 1][y + 1] * d * outlineStrength;
        }
    int depthChange = (int)sqrtf(powf(hori, 2) + powf(vert, 2));
    float k = sat((float)(1 - abs(depthChange)));
    for (int c = 0; c < 3; ++c) out->shader[3 * p + c] = out->shader[3 * p + c] * k;
}

static void pp_run(int id, const pp_buf* in, const pp_buf* out, long p, int x, int y, int W, int H,
                   const float* view, const otex* shadow)
{
    (void)view;
    long HW = (long)W * H;
    float* sc = out->shader + 3 * p;
    switch (id) {
    case PP_INVERT: /* :187-189 */
        for (int c = 0; c < 3; ++c) sc[c] = 1 - in->shader[3 * p + c];
        break;
    case PP_OUTLINE: { /* :212-232 (every sample tests in.pixel itself) */
        long idx = p;
        int inside = !(idx < 0 || idx > HW) && in->stencil[idx] >= 0.9f;
        int outside = !inside, near = 0;
        for (float radius = 1; radius < 5 + 1; radius++)
            for (float direction = 0; direction <= 1; direction += 1.0f / (float)5) near |= inside;
        float o = (float)(outside && near);
        const float red[3] = {1, 0, 0};
        for (int c = 0; c < 3; ++c) sc[c] = in->base[3 * p + c] * (1.0f - o) + red[c] * o;
        break;
    }
    case PP_CRACKRECON: { /* :234-261 */
        float mask = in->stencil[p] * in->metallic[p];
        if (mask <= 0.01f) break;
        const float* n = in->normal + 3 * p;
        float ld[3] = {0, -0.2f, 1};
        float inv = 1.0f / sqrtf(dot3(ld, ld));
        for (int c = 0; c < 3; ++c) ld[c] = ld[c] * inv;
        float internal[3] = {0.83f, 0.64f, 0.2f};
        float k = sat(sat(dot3(ld, n) * 0.1f) + 0.9f);
        for (int c = 0; c < 3; ++c) {
            internal[c] *= k;
            sc[c] = internal[c] * mask + in->shader[3 * p + c] * (1 - mask);
        }
        break;
    }
    case PP_TEXTUREDSHADOWS: pp_textured_shadows(in, out, p, x, y, W, H, shadow); break;
    case PP_QUANTIZELIGHTING: { /* :291-297 */
        const float* L = in->incident + 3 * p;
        float white = fmaxf(L[0], fmaxf(L[1], L[2]));
        float q = roundf(white * 4) / 4;
        for (int c = 0; c < 3; ++c) out->incident[3 * p + c] = q;
        break;
    }
    case PP_BLURLIGHTING: { /* :299-309, GaussianBlur shaderUtils.cu:104-123 */
        const float* pix = in->incident + 3 * p;
        if (pix[0] == 0 && pix[1] == 0 && pix[2] == 0) break;
        float acc[3] = {0, 0, 0};
        for (int dx = -2; dx < 3; dx++)
            for (int dy = -2; dy < 3; dy++) {
                long sp = p + dx + (long)dy * W;
                sp = sp < 0 ? 0 : (sp > HW - 1 ? HW - 1 : sp);
                for (int c = 0; c < 3; ++c) acc[c] += kBlend[dx + 2][dy + 2] * in->incident[3 * sp + c];
            }
        for (int c = 0; c < 3; ++c) out->incident[3 * p + c] = acc[c];
        break;
    }
    case PP_SOBEL: pp_sobel(in, out, p, W); break;
    case PP_TOON: /* :333-337 */
        pp_color_correction(in, out, p);
        pp_textured_shadows(in, out, p, x, y, W, H, shadow);
        pp_sobel(in, out, p, W);
        break;
    default: break; /* DefaultPostProcess */
    }
}

/* RunPostProcessShaders (forward.cu:973-1047). `features` is out_feature in the reference's
 * 21-channel block layout (NULL when S != 21: the feature planes of the copy stay zero). The
 * thread -> pixel mapping is x = idx % W, y = idx / W (the reference divides by H, which only
 * agrees for square images). */
void oracle_post_passes(const int* ids, int n, int W, int H, const float* view, float* color, float* opacity,
                        float* depth, float* stencil, float* xyz, float* normal, float* features, float* shader,
                        const otex* shadow)
{
    long HW = (long)W * H;
    if (n <= 0 || HW == 0) return;
    /* CreateDeepBuffer: one allocation, 21 feature planes + 15 scene planes */
    float* buf = (float*)calloc((size_t)36 * HW, sizeof(float));
    pp_buf out = pp_views(features, opacity, depth, stencil, xyz, normal, shader, color, HW);
    pp_buf in = pp_views(buf, buf + 21 * HW, buf + 22 * HW, buf + 23 * HW, buf + 24 * HW, buf + 27 * HW,
                         buf + 30 * HW, buf + 33 * HW, HW);
    float* planes_out[8] = {features, opacity, depth, stencil, xyz, normal, shader, color};
    const long sizes[8] = {21 * HW, HW, HW, HW, 3 * HW, 3 * HW, 3 * HW, 3 * HW};
    const long offs[8] = {0, 21 * HW, 22 * HW, 23 * HW, 24 * HW, 27 * HW, 30 * HW, 33 * HW};
    for (int i = 0; i < n; ++i) {
        /* DeepCopy (before the first pass, then between passes) */
        for (int k = 0; k < 8; ++k)
            if (planes_out[k]) memcpy(buf + offs[k], planes_out[k], sizeof(float) * (size_t)sizes[k]);
        for (long p = 0; p < HW; ++p) pp_run(ids[i], &in, &out, p, (int)(p % W), (int)(p / W), W, H, view, shadow);
    }
    free(buf);
}
