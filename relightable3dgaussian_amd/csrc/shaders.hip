// shaders.hip -- SH / splat shader library, texture objects and texture manager (gfx950).
//
// Restates cuda_rasterizer/ShShader.cu:62-190 (SH shaders: run before preprocessing on working
// copies of positions / scales / rotations / opacity / SH), splatShader.cu:67-269 (splat
// shaders: run after the intermediate depth/stencil pass, edit opacity, stencil, features and
// write the shader colour), utils/shaderUtils.cu:147-161 (Quantize) and utils/texture.cu
// (texture objects, TextureManager). Plain IEEE ops with contraction off; the reference's double
// promotions (M_PI, 0.125, 1.5, M_1_PI literals) are kept.
#pragma clang fp contract(off)

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "r3dg_hip.h"
#include "shaders.h"

namespace r3dg {

__device__ inline float3 f3(const float* p) { return make_float3(p[0], p[1], p[2]); }
__device__ inline void st3(float* p, float3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
__device__ inline float3 add3(float3 a, float3 b) { return make_float3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ inline float3 sub3(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ inline float3 mul3(float3 a, float s) { return make_float3(a.x * s, a.y * s, a.z * s); }
// glm::dot (func_geometric.inl: tmp = a * b; tmp.x + tmp.y + tmp.z)
__device__ inline float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ inline float len3(float3 a) { return sqrtf(dot3(a, a)); }
// glm::normalize: x * inversesqrt(dot(x, x)), inversesqrt = 1 / sqrt
__device__ inline float3 norm3(float3 a) { return mul3(a, 1.0f / sqrtf(dot3(a, a))); }
// glm::mix(x, y, a) = x * (1 - a) + y * a
__device__ inline float3 mix3(float3 x, float3 y, float a) { return add3(mul3(x, 1.0f - a), mul3(y, a)); }
__device__ inline float sat(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }  // __saturatef (NaN -> 0 below)
__device__ inline float satf(float x) { return x != x ? 0.0f : sat(x); }

// Heartbeat volume curve (ShShader.cu:109-118): evaluated in double (M_PI literal), cast to float
__device__ inline float heartbeat(float t) {
    const double k = M_PI * 4.0 / 3.0;
    const double m = fmod((double)t, k);
    const double up = round(sin(m) / 2 + 0.5);
    return (float)((1 + cos(m) * up + cos(m * 3) * (1 - up)) / 2);
}

// three-plane texture mask (ShShader.cu:84-95,151-158; splatShader.cu:104-111)
__device__ inline float tri_planar(const TexDesc& t, float3 p, bool invert, bool product) {
    float a = tex_sample(t, p.x, p.y).x, b = tex_sample(t, p.x, p.z).x, c = tex_sample(t, p.y, p.z).x;
    if (invert) {
        a = 1 - a;
        b = 1 - b;
        c = 1 - c;
    }
    return product ? a * b * c : (a + b + c) / 3;
}

template <int ID>
__global__ void __launch_bounds__(256) sh_shader_kernel(ShShaderArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int g = a.idx[i];
    float* pos = a.pos + 3 * (size_t)g;
    float* scale = a.scale + 3 * (size_t)g;
    if constexpr (ID == kShExpPos) {  // ShShader.cu:67-77
        const float3 p = f3(pos), s = f3(scale);
        const float posY = fabsf(p.y);
        st3(scale, mul3(make_float3(s.x * posY, s.y * 2, s.z), posY));
        st3(pos, mul3(make_float3(p.x * posY, p.y * 2, p.z), posY));
    } else if constexpr (ID == kShHeartbeat) {  // ShShader.cu:82-138
        const float3 p = f3(pos);
        const float atrial = tri_planar(a.tex0, p, false, false);     // "Turbulence"
        const float ventricular = tri_planar(a.tex1, p, true, false); // "Craters"
        const float pulsePeriod = 1, distInfluence = -0.5f;
        const float time = a.time / 1000 / pulsePeriod + len3(p) * distInfluence;
        const float atrialGrowth = heartbeat(time) * atrial;
        const float ventricularGrowth = heartbeat(time - 0.9f) * ventricular;
        const float3 n = f3(a.features + (size_t)g * a.S + 6);
        const float3 aPos = mul3(mul3(n, atrialGrowth), 0.025f), vPos = mul3(mul3(n, ventricularGrowth), 0.025f);
        const float3 aSc = mul3(make_float3(atrialGrowth, atrialGrowth, atrialGrowth), 0.0025f);
        const float3 vSc = mul3(make_float3(ventricularGrowth, ventricularGrowth, ventricularGrowth), 0.0025f);
        st3(pos, add3(add3(p, aPos), vPos));
        st3(scale, add3(add3(f3(scale), aSc), vSc));
    } else if constexpr (ID == kShCullHalf) {  // ShShader.cu:141-149
        if (pos[0] < 0) {
            a.opacity[g] = 0;
            st3(scale, make_float3(0.f, 0.f, 0.f));
        }
    } else if constexpr (ID == kShGaussDissolve) {  // ShShader.cu:152-188
        const float3 p = f3(pos);
        float mask = tri_planar(a.tex0, p, false, true);  // "Cracks"
        mask = satf((float)(((double)mask - 0.125) * 1.5));
        const float loadingSpeed = 0.25f, loopDuration = 3;
        const float total = fmodf(a.time / 1000 * loadingSpeed, loopDuration);
        const float lp = satf(total - p.z + mask - 1);
        a.opacity[g] *= lp * lp * lp;
        const float fadeDistance = len3(f3(scale)) * 10;
        const float3 startPos = add3(p, mul3(make_float3(0.f, 0.f, 1.f), fadeDistance));
        st3(pos, mix3(startPos, p, lp));
        float* sh0 = a.sh + (size_t)g * a.M * 3;
        st3(sh0, mix3(make_float3(0.6f, 0.9f, 1.0f), f3(sh0), lp));
    }
}

// splat shader helpers: the reference's per-splat feature views (splatShader.cu:44-52)
struct SplatFeatures {
    float* f;
    __device__ float& roughness() { return f[0]; }
    __device__ float& metallic() { return f[1]; }
    __device__ float& visibility() { return f[2]; }
    __device__ float* normal() { return f + 6; }
    __device__ float* color_base() { return f + 9; }
    __device__ float* incident() { return f + 12; }
    __device__ float* local() { return f + 15; }
    __device__ float* global() { return f + 18; }
};

__device__ inline float outline_opacity(float3 cam, float3 p, float3 n) {  // splatShader.cu:76-83
    const float angle = 1 - fabsf(dot3(norm3(sub3(cam, p)), norm3(n)));
    return angle < 0.5 ? 1 - 16 * powf(angle, 5.0f) : powf(-2 * angle + 2, 5.0f) / 2;
}

template <int ID>
__global__ void __launch_bounds__(256) splat_shader_kernel(SplatShaderArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int g = a.idx[i];
    const float3 p = f3(a.pos + 3 * (size_t)g);
    const float3 colSH = f3(a.rgb + 3 * (size_t)g);
    float* out = a.out_rgb + 3 * (size_t)g;
    float& opacity = a.conic_opacity[g].w;
    SplatFeatures F{a.features + (size_t)g * a.S};
    const float3 cam = make_float3(a.viewmatrix_inv[12], a.viewmatrix_inv[13], a.viewmatrix_inv[14]);
    auto mean_pixel = [&]() {  // splatShader.cu:33: W * floor(y) + floor(x) (clamped: see DESIGN)
        const float2 s = a.means2D[g];
        const int id = (int)((float)a.W * floorf(s.y) + floorf(s.x));
        return id < 0 ? 0 : (id >= a.W * a.H ? a.W * a.H - 1 : id);
    };
    if constexpr (ID == kSpDefault) {  // :66-70
        st3(out, colSH);
    } else if constexpr (ID == kSpNaiveOutline) {  // :73-84
        st3(out, mul3(colSH, outline_opacity(cam, p, f3(F.normal()))));
    } else if constexpr (ID == kSpWireframe) {  // :86-97
        const float o = outline_opacity(cam, p, f3(F.normal()));
        st3(out, make_float3(1 - o, 1 - o, 1 - o));
    } else if constexpr (ID == kSpDissolve) {  // :101-136
        float mask = tri_planar(a.tex0, p, false, true);  // "Cracks"
        mask = satf((float)(((double)mask - 0.125) * 1.5));
        const float period = 0.1f;
        const float o = cosf((float)((double)(a.time * period * 4) / (M_1_PI * 2 * 1000))) + 1;
        const float masked = satf(o - (1 - mask));
        opacity = opacity * masked;
        const float fading = satf(masked * 3);
        a.stencils[g] = mask;
        st3(out, mix3(make_float3(0.6f, 0.9f, 1.0f), colSH, fading));
    } else if constexpr (ID == kSpCrack) {  // :138-183
        const float texScale = 2;
        const float u = (float)((double)(p.x / texScale) - 0.5), v = (float)((double)(p.y / texScale) - 0.5);
        const float crackTexDepth = 1 - tex_sample(a.tex0, u, v).x;  // "Depth cracks"
        const float maxCrackDepth = 2, projectionHeight = 2;
        const float crackHeight = projectionHeight - crackTexDepth * maxCrackDepth;
        const float splatHeight = p.z;
        const bool reaches = crackHeight < splatHeight;
        opacity = reaches ? 0 : opacity;
        const float depthTolerance = 0.3f;
        const float distToSurface = a.depths[g] - a.depth_tex[mean_pixel()] + depthTolerance;
        const bool inside = distToSurface > 0;
        const float internalColorReach = 0.1f;
        const float maxPrimary = projectionHeight - (crackTexDepth + internalColorReach) * maxCrackDepth;
        const bool inReach = splatHeight > maxPrimary;
        const bool useInternal = inside && inReach;
        const bool internalColorPercent = satf(distToSurface * 10) != 0.0f;  // a bool in the reference
        const float3 internalColor = internalColorPercent ? make_float3(0.5f, 0.5f, 0.f) : f3(F.color_base());
        const float discolorReach = 0.1f;
        const float maxDiscolor = maxPrimary - discolorReach * maxCrackDepth;
        const float discolor = satf((splatHeight - maxDiscolor) / (discolorReach + internalColorReach));
        const float3 externalColor = mix3(colSH, internalColor, discolor);
        const float3 finalColor =
            add3(mul3(internalColor, (float)useInternal), mul3(externalColor, (float)!useInternal));
        opacity += 0.2f * (float)useInternal * (float)!reaches;
        st3(out, finalColor);
    } else if constexpr (ID == kSpCrackNoRecon) {  // :185-227
        const float texScale = 2;
        const float u = (float)((double)(p.x / texScale) - 0.5), v = (float)((double)(p.y / texScale) - 0.5);
        const float crackTexDepth = 1 - tex_sample(a.tex0, u, v).x;  // "Bulge"
        const float maxCrackDepth = 2, projectionHeight = 2;
        const float crackHeight = projectionHeight - crackTexDepth * maxCrackDepth;
        const float splatHeight = p.z;
        const bool reaches = crackHeight < splatHeight;
        const float originalOpacity = opacity;
        opacity = reaches ? 0 : opacity;
        const float depthTolerance = 0.2f;
        const float rel = a.depths[g] - a.depth_tex[mean_pixel()] + depthTolerance;
        const bool inside = rel > 0;
        const float internalColorReach = 0.5f * crackTexDepth;
        const float maxPrimary = projectionHeight - (crackTexDepth + internalColorReach) * maxCrackDepth;
        const bool inReach = maxPrimary < splatHeight;
        const bool useInternal = inside && inReach;
        st3(out, f3(F.color_base()));
        a.stencils[g] = (float)reaches;
        a.stencil_opacity[g] = originalOpacity;
        F.metallic() = (float)useInternal;
    } else if constexpr (ID == kSpStencil) {  // :229-233
        a.stencils[g] = 1;
        a.stencil_opacity[g] = opacity;
        st3(out, colSH);
    } else if constexpr (ID == kSpRoughnessOnly) {  // :235-252
        F.roughness() = p.x < 0 ? 0.25f : 0.75f;
        F.metallic() = 0;
        F.visibility() = 0;
        st3(F.normal(), make_float3(0.f, 0.f, 0.f));
        st3(F.color_base(), make_float3(0.f, 0.f, 0.f));
        st3(F.incident(), make_float3(0.f, 0.f, 0.f));
        st3(F.local(), make_float3(0.f, 0.f, 0.f));
        st3(F.global(), make_float3(0.f, 0.f, 0.f));
        st3(out, make_float3(0.f, 0.f, 0.f));
    } else if constexpr (ID == kSpQuantizeFlats) {  // :254-258
        st3(out, f3(F.color_base()));
    } else if constexpr (ID == kSpQuantizeLight) {  // :260-269, Quantize (shaderUtils.cu:147-155)
        const float* L = F.incident();
        const float qr = roundf(L[0] * 3) / 3, qg = roundf(L[1] * 3) / 3, qb = roundf(L[2] * 3) / 3;
        F.roughness() = fmaxf(qr, fmaxf(qg, qb));
        st3(out, f3(F.color_base()));
    }
}

template <int ID>
static hipError_t sh_launch(const ShShaderArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(sh_shader_kernel<ID>, dim3((a.n + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_sh_shader(int id, const ShShaderArgs& a, hipStream_t st) {
    if (a.n == 0 || id == kShDefault) return hipSuccess;  // DefaultShShaderCUDA does nothing
    switch (id) {
        case kShCullHalf: return sh_launch<kShCullHalf>(a, st);
        case kShExpPos: return sh_launch<kShExpPos>(a, st);
        case kShGaussDissolve: return sh_launch<kShGaussDissolve>(a, st);
        case kShHeartbeat: return sh_launch<kShHeartbeat>(a, st);
    }
    return hipErrorInvalidValue;
}

template <int ID>
static hipError_t sp_launch(const SplatShaderArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(splat_shader_kernel<ID>, dim3((a.n + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_splat_shader(int id, const SplatShaderArgs& a, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    switch (id) {
        case kSpCrack: return sp_launch<kSpCrack>(a, st);
        case kSpCrackNoRecon: return sp_launch<kSpCrackNoRecon>(a, st);
        case kSpDissolve: return sp_launch<kSpDissolve>(a, st);
        case kSpNaiveOutline: return sp_launch<kSpNaiveOutline>(a, st);
        case kSpQuantizeFlats: return sp_launch<kSpQuantizeFlats>(a, st);
        case kSpQuantizeLight: return sp_launch<kSpQuantizeLight>(a, st);
        case kSpRoughnessOnly: return sp_launch<kSpRoughnessOnly>(a, st);
        case kSpDefault: return sp_launch<kSpDefault>(a, st);
        case kSpStencil: return sp_launch<kSpStencil>(a, st);
        case kSpWireframe: return sp_launch<kSpWireframe>(a, st);
    }
    return hipErrorInvalidValue;
}

const char* sh_shader_texture(int id, int k) {
    if (id == kShHeartbeat) return k == 0 ? "Turbulence" : "Craters";
    if (id == kShGaussDissolve && k == 0) return "Cracks";
    return nullptr;
}
const char* splat_shader_texture(int id) {
    switch (id) {
        case kSpDissolve: return "Cracks";
        case kSpCrack: return "Depth cracks";
        case kSpCrackNoRecon: return "Bulge";
    }
    return nullptr;
}
bool sh_shader_needs_features(int id) { return id == kShHeartbeat; }
bool splat_shader_needs_features(int id) {
    return id == kSpNaiveOutline || id == kSpWireframe || id == kSpCrack || id == kSpCrackNoRecon ||
           id == kSpRoughnessOnly || id == kSpQuantizeFlats || id == kSpQuantizeLight;
}

// ---- post-process passes (postProcessShader.cu:177-374, shaderUtils.cu) ----------------------
bool post_pass_needs_features(int id) {
    return id == kPpBlurLighting || id == kPpCrackReconstruction || id == kPpOutline || id == kPpQuantizeLighting ||
           id == kPpTexturedShadows || id == kPpToon;
}
bool post_pass_needs_shadow(int id) { return id == kPpTexturedShadows || id == kPpToon; }

// RgbToHsv / HsvToRgb (shaderUtils.cu:6-82)
__device__ inline float3 rgb_to_hsv(float3 c) {
    const float mx = fmaxf(c.x, fmaxf(c.y, c.z)), mn = fminf(c.x, fminf(c.y, c.z));
    const float diff = mx - mn;
    float h = 0.f, s = 0.f;
    if (mx != 0.0f) {
        s = diff / mx;
        if (!(diff < 0.001f)) {
            if (mx == c.x) {
                h = (c.y - c.z) / diff / 6;
                if (h < 0.0f) h += 1.0f;
            } else if (mx == c.y) {
                h = (2 + (c.z - c.x) / diff) / 6;
            } else {
                h = (4 + (c.x - c.y) / diff) / 6;
            }
        }
    }
    return make_float3(h, s, mx);
}
__device__ inline float3 hsv_to_rgb(float3 hsv) {
    const float h = hsv.x, s = hsv.y, v = hsv.z;
    float f = h * 6;
    const float hi = floorf(f);
    f = f - hi;
    const float p = v * (1 - s), q = v * (1 - s * f), t = v * (1 - s * (1 - f));
    if (hi == 0.0f || hi == 6.0f) return make_float3(v, t, p);
    if (hi == 1.0f) return make_float3(q, v, p);
    if (hi == 2.0f) return make_float3(p, v, t);
    if (hi == 3.0f) return make_float3(p, q, v);
    if (hi == 4.0f) return make_float3(t, p, v);
    return make_float3(v, p, q);
}

// Sobel's unclamped depth reads (postProcessShader.cu:317-323): the reference's input buffer is
// one allocation [21 feature planes | opacity | depth | stencil | xyz | ...]
// (postProcessShader.cu:76-103), so reads above the first / below the last row land in the
// opacity / stencil planes. None of those planes is written by a pass, so the live buffers hold
// the same values as the reference's copy.
__device__ inline float depth_in_buffer(const PostArgs& a, long long sp) {
    const long long HW = (long long)a.W * a.H;
    const long long k = 22 * HW + sp;
    if (k >= 24 * HW) return k - 24 * HW < 3 * HW ? a.surface_xyz[k - 24 * HW] : 0.f;
    if (k >= 23 * HW) return a.stencil[k - 23 * HW];
    if (k >= 22 * HW) return a.depth[k - 22 * HW];
    if (k >= 21 * HW) return a.opacity[k - 21 * HW];
    return (a.features && k >= 0) ? a.features[k] : 0.f;
}

__device__ inline void pp_color_correction(const PostArgs& a, int p, float3 inc_in, float3& sc) {  // :276-289
    const long long HW = (long long)a.W * a.H;
    float3 hsv = rgb_to_hsv(f3(a.features + 9 * HW + 3 * (long long)p));
    hsv.x = roundf(hsv.x * 24) / 24;  // Quantize(hue, 24)
    const float3 color = hsv_to_rgb(hsv);
    const float reduced = satf(inc_in.x + 0.25f);
    sc = mul3(color, reduced);
}

__device__ inline void pp_textured_shadows(const PostArgs& a, int p, int x, int y, float3 inc_in, float3& sc) {  // :238-274
    if (a.stencil[p] < 0.01f) {
        sc = make_float3(1.f, 1.f, 1.f);
        return;
    }
    const float uvScale = 10;
    const float u = (float)x / (float)a.W * uvScale, v = (float)y / (float)a.H * uvScale;
    const float4 t = tex_sample(a.shadow, u, v);
    float lightShadow = 1 - t.x, mediumShadow = 1 - t.z, heavyShadow = 1 - t.y;
    float intensity = inc_in.x > fmaxf(inc_in.y, inc_in.z) ? inc_in.x : fmaxf(inc_in.y, inc_in.z);  // __max
    intensity = roundf(intensity * 4);
    heavyShadow = satf(heavyShadow + intensity);
    intensity = 0.f > intensity - 1.0f ? 0.f : intensity - 1.0f;
    mediumShadow = satf(mediumShadow + intensity);
    intensity = 0.f > intensity - 1.0f ? 0.f : intensity - 1.0f;
    lightShadow = satf(lightShadow + intensity);
    sc = mul3(mul3(mul3(sc, lightShadow), mediumShadow), heavyShadow);
}

__device__ inline void pp_sobel(const PostArgs& a, int p, float3& sc) {  // :304-331
    const float SobelHorizontal[3][3] = {{-1, 0, 1}, {-2, 0, 2}, {-1, 0, 1}};
    const float SobelVertical[3][3] = {{-1, -2, -1}, {0, 0, 0}, {1, 2, 1}};
    const float outlineStrength = 2;
    float hori = 0, vert = 0;
    for (int x = -1; x < 2; x++)
        for (int y = -1; y < 2; y++) {
            const float d = depth_in_buffer(a, (long long)p + x + (long long)y * a.W);
            hori += SobelHorizontal[x + 1][y + 1] * d * outlineStrength;
            vert += SobelVertical[x + 1][y + 1] * d * outlineStrength;
        }
    const int depthChange = (int)sqrtf(powf(hori, 2.0f) + powf(vert, 2.0f));
    sc = mul3(sc, satf((float)(1 - abs(depthChange))));
}

// One thread per pixel (the intended x + y * W mapping), every pass of a
// pixel-local run in order. `in.*` reads of the pixel's own values are the live values at the
// pass start: no other thread writes this pixel.
__global__ void __launch_bounds__(256) post_pixel_kernel(PostArgs a) {
    const long long HW = (long long)a.W * a.H;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    const int x = p % a.W, y = p / a.W;
    float3 sc = f3(a.shader_color + 3 * (long long)p);
    float* inc_ptr = a.features ? a.features + 12 * HW + 3 * (long long)p : nullptr;
    float3 inc = inc_ptr ? f3(inc_ptr) : make_float3(0.f, 0.f, 0.f);
    for (int i = 0; i < a.n_pass; ++i) {
        const float3 sc_in = sc, inc_in = inc;
        switch (a.pass[i]) {
            case kPpInvert:  // :187-189
                sc = sub3(make_float3(1.f, 1.f, 1.f), sc_in);
                break;
            case kPpOutline: {  // :212-232: the samples test in.pixel itself, so "near" == "inside"
                const bool inside = a.stencil[p] >= 0.9f;
                const bool near = inside;
                const float o = (float)(!inside && near);
                const float3 base = f3(a.features + 9 * HW + 3 * (long long)p);
                sc = add3(mul3(base, 1.0f - o), mul3(make_float3(1.f, 0.f, 0.f), o));
                break;
            }
            case kPpCrackReconstruction: {  // :234-261
                const float mask = a.stencil[p] * a.features[HW + p];
                if (mask <= 0.01f) break;
                const float3 normal = f3(a.pseudonormal + 3 * (long long)p);
                const float3 lightDir = norm3(make_float3(0.f, -0.2f, 1.f));
                const float lightIntensity = 0.1f, ambientLight = 0.9f;
                float3 internal = make_float3(0.83f, 0.64f, 0.2f);
                internal = mul3(internal, satf(satf(dot3(lightDir, normal) * lightIntensity) + ambientLight));
                sc = add3(mul3(internal, mask), mul3(sc_in, 1 - mask));
                break;
            }
            case kPpTexturedShadows:
                pp_textured_shadows(a, p, x, y, inc_in, sc);
                break;
            case kPpQuantizeLighting: {  // :291-297
                const float white = fmaxf(inc_in.x, fmaxf(inc_in.y, inc_in.z));
                const float q = roundf(white * 4) / 4;
                inc = make_float3(q, q, q);
                break;
            }
            case kPpSobelFilter:
                pp_sobel(a, p, sc);
                break;
            case kPpToon:  // :333-337
                pp_color_correction(a, p, inc_in, sc);
                pp_textured_shadows(a, p, x, y, inc_in, sc);
                pp_sobel(a, p, sc);
                break;
            default:
                break;
        }
    }
    st3(a.shader_color + 3 * (long long)p, sc);
    if (inc_ptr) st3(inc_ptr, inc);
}

// BlurLighting (:299-309) with GaussianBlur's clamped 1-D neighbourhood (shaderUtils.cu:104-123)
__constant__ float kBlend[5][5] = {{0.009375f, 0.01875f, 0.028125f, 0.01875f, 0.009375f},
                                   {0.01875f, 0.0375f, 0.045f, 0.0375f, 0.01875f},
                                   {0.028125f, 0.045f, 0.3f, 0.045f, 0.028125f},
                                   {0.01875f, 0.0375f, 0.045f, 0.0375f, 0.01875f},
                                   {0.009375f, 0.01875f, 0.028125f, 0.01875f, 0.009375f}};
__global__ void __launch_bounds__(256) post_blur_kernel(PostArgs a) {
    const int HW = a.W * a.H;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    const float3 pix = f3(a.incident_in + 3 * (size_t)p);
    if (pix.x == 0 && pix.y == 0 && pix.z == 0) return;
    float3 acc = make_float3(0.f, 0.f, 0.f);
    for (int x = -2; x < 3; x++)
        for (int y = -2; y < 3; y++) {
            int sp = p + x + y * a.W;
            sp = max(0, min(HW - 1, sp));
            acc = add3(acc, mul3(f3(a.incident_in + 3 * (size_t)sp), kBlend[x + 2][y + 2]));
        }
    st3(a.features + 12 * (size_t)HW + 3 * (size_t)p, acc);
}

hipError_t launch_post_passes(const int* ids, int n, const PostArgs& base, float* scratch, hipStream_t st) {
    const int HW = base.W * base.H;
    if (HW == 0) return hipSuccess;
    const dim3 grid((HW + 255) / 256), block(256);
    PostArgs a = base;
    a.n_pass = 0;
    auto flush = [&]() -> hipError_t {
        if (a.n_pass == 0) return hipSuccess;
        hipLaunchKernelGGL(post_pixel_kernel, grid, block, 0, st, a);
        a.n_pass = 0;
        return hipGetLastError();
    };
    for (int i = 0; i < n; ++i) {
        const int id = ids[i];
        if (id == kPpDefault) continue;  // DefaultPostProcess does nothing
        if (id == kPpBlurLighting) {
            hipError_t e = flush();
            if (e != hipSuccess) return e;
            e = hipMemcpyAsync(scratch, a.features + 12 * (size_t)HW, sizeof(float) * 3 * (size_t)HW,
                               hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
            a.incident_in = scratch;
            hipLaunchKernelGGL(post_blur_kernel, grid, block, 0, st, a);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            continue;
        }
        if (a.n_pass == kMaxFusedPasses) {
            const hipError_t e = flush();
            if (e != hipSuccess) return e;
        }
        a.pass[a.n_pass++] = id;
    }
    return flush();
}

// ---- texture objects (texture.cu:86-262) ----------------------------------------------------
// Texel expansion: 1-channel modes go to .x (alpha 1), 3-channel modes get alpha 1
// (CreatPaddedArrayFromBase), 4-channel modes are copied.
__global__ void __launch_bounds__(256) expand_texels_kernel(const float* __restrict__ src, int n, int C,
                                                            float4* __restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* s = src + (size_t)i * C;
    dst[i] = C == 1 ? make_float4(s[0], 0.f, 0.f, 1.f)
                    : (C == 3 ? make_float4(s[0], s[1], s[2], 1.f) : make_float4(s[0], s[1], s[2], s[3]));
}

struct TextureObj {
    TexDesc desc;
    float4* texels;
};
struct TextureManagerObj {
    std::map<std::string, TexDesc> by_name;
    TexDesc error;
};
static std::mutex g_tex_mu;
static std::map<int64_t, TextureObj*> g_textures;
static std::map<int64_t, TextureManagerObj*> g_tex_managers;
static int64_t g_next_tex = 1;

int texture_mode_channels(int mode) {  // texture.h TextureMode order = r3dg_encode_texture_mode
    switch (mode) {
        case 0: case 1: case 2: case 9: case 10: return 1;  // 1, L, P, I, F
        case 3: case 6: case 7: case 8: return 3;           // RGB, YCbCr, LAB, HSV
        case 4: case 5: return 4;                           // RGBA, CMYK
    }
    return 0;
}

bool lookup_texture_manager(int64_t h, const std::map<std::string, TexDesc>** names, TexDesc* error) {
    std::lock_guard<std::mutex> lk(g_tex_mu);
    auto it = g_tex_managers.find(h);
    if (it == g_tex_managers.end()) return false;
    *names = &it->second->by_name;
    *error = it->second->error;
    return true;
}

}  // namespace r3dg

using namespace r3dg;

extern "C" int r3dg_texture_create(const float* pixels, int width, int height, int mode, int wrap_u, int wrap_v,
                                   int normalized, int64_t* texture, r3dg_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    const int C = texture_mode_channels(mode);
    R3DG_REQUIRE(texture && pixels && width > 0 && height > 0, "AllocateTexture: invalid arguments");
    R3DG_REQUIRE(C > 0, "AllocateTexture: unknown texture encoding mode");
    R3DG_REQUIRE(wrap_u >= 0 && wrap_u <= 3 && wrap_v >= 0 && wrap_v <= 3, "AllocateTexture: invalid wrap mode");
    const int n = width * height;
    float4* texels = nullptr;
    R3DG_CHECK_HIP(hipMalloc(&texels, sizeof(float4) * (size_t)n));
    hipLaunchKernelGGL(expand_texels_kernel, dim3((n + 255) / 256), dim3(256), 0, st, pixels, n, C, texels);
    R3DG_CHECK_HIP(hipGetLastError());
    R3DG_CHECK_HIP(hipStreamSynchronize(st));
    auto* t = new TextureObj();
    // LAB / HSV: point sampling (the reference's unsigned normalized-float read mode, texture.cu:162-168)
    t->desc = TexDesc{texels, width, height, wrap_u, wrap_v, normalized ? 1 : 0, (mode == 7 || mode == 8) ? 0 : 1};
    t->texels = texels;
    std::lock_guard<std::mutex> lk(g_tex_mu);
    const int64_t h = (int64_t)0x5454000000000000ll | g_next_tex++;
    g_textures[h] = t;
    *texture = h;
    return R3DG_OK;
}

extern "C" int r3dg_texture_manager_create(int n, const char* const* names, const int64_t* textures,
                                           int64_t error_texture, int64_t* manager) {
    R3DG_REQUIRE(manager && n >= 0 && (n == 0 || (names && textures)), "UploadTexturesToDevice: invalid arguments");
    std::lock_guard<std::mutex> lk(g_tex_mu);
    auto err = g_textures.find(error_texture);
    R3DG_REQUIRE(err != g_textures.end(), "UploadTexturesToDevice: unknown error texture");
    auto* m = new TextureManagerObj();
    m->error = err->second->desc;
    for (int i = 0; i < n; ++i) {
        auto it = g_textures.find(textures[i]);
        if (it == g_textures.end()) {
            delete m;
            set_error("UploadTexturesToDevice: unknown texture handle");
            return R3DG_ERR_ARG;
        }
        m->by_name.emplace(names[i], it->second->desc);  // first entry of a name wins, as the linear lookup
    }
    const int64_t h = (int64_t)0x544d000000000000ll | g_next_tex++;
    g_tex_managers[h] = m;
    *manager = h;
    return R3DG_OK;
}
