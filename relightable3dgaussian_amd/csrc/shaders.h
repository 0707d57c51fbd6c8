// shaders.h -- SH / splat shader library and software texture sampling (gfx950).
//
// Restates the reference's shader library (cuda_rasterizer/ShShader.cu:62-190,
// splatShader.cu:67-269, utils/shaderUtils.cu) and texture objects (utils/texture.cu:86-262).
// Shaders are selected by registry id (rasterizer.hip shader_names), not device function
// pointers: every non-empty per-shader bucket of a shader manager launches the kernel
// instantiated for that shader. Textures are float4 texel arrays in HBM sampled in software with
// the CUDA texture-unit rules the reference relies on (normalized coordinates, wrap / clamp /
// mirror / border addressing, bilinear filtering with 8-bit fractional weights, point sampling
// for LAB/HSV), so the oracle can restate them exactly.
#pragma once
#include <map>
#include <string>

#include "r3dg_common.h"

namespace r3dg {

// hipTextureAddressMode values (== cudaTextureAddressMode, texture.cu:64-76)
enum { kAddrWrap = 0, kAddrClamp = 1, kAddrMirror = 2, kAddrBorder = 3 };

struct TexDesc {
    const float4* texels;  // [H, W] row-major
    int W, H;
    int wrap_u, wrap_v;
    int normalized;  // coordinates in [0, 1) per texture extent
    int linear;      // bilinear (float modes) or point (LAB / HSV)
};

__host__ __device__ inline int tex_index(int i, int n, int mode, int normalized, bool& zero) {
    if (mode == kAddrBorder) {
        if (i < 0 || i >= n) zero = true;
        return i < 0 ? 0 : (i >= n ? n - 1 : i);
    }
    if (normalized && mode == kAddrWrap) {
        i %= n;
        return i < 0 ? i + n : i;
    }
    if (normalized && mode == kAddrMirror) {
        const int p = 2 * n;
        i %= p;
        if (i < 0) i += p;
        return i < n ? i : p - 1 - i;
    }
    return i < 0 ? 0 : (i >= n ? n - 1 : i);  // clamp (also wrap / mirror on texel coordinates)
}

__host__ __device__ inline float4 tex_fetch(const TexDesc& t, int i, int j) {
    bool zero = false;
    const int x = tex_index(i, t.W, t.wrap_u, t.normalized, zero);
    const int y = tex_index(j, t.H, t.wrap_v, t.normalized, zero);
    if (zero) return make_float4(0.f, 0.f, 0.f, 0.f);
    return t.texels[(size_t)y * t.W + x];
}

// tex2D<float4>(tex, x, y)
__host__ __device__ inline float4 tex_sample(const TexDesc& t, float x, float y) {
    const float u = t.normalized ? x * (float)t.W : x;
    const float v = t.normalized ? y * (float)t.H : y;
    if (!t.linear) return tex_fetch(t, (int)floorf(u), (int)floorf(v));
    const float ub = u - 0.5f, vb = v - 0.5f;
    const float fu = floorf(ub), fv = floorf(vb);
    const int i = (int)fu, j = (int)fv;
    // the texture unit keeps the interpolation weights in 9-bit fixed point, 8 fractional bits
    const float a = rintf((ub - fu) * 256.0f) * (1.0f / 256.0f);
    const float b = rintf((vb - fv) * 256.0f) * (1.0f / 256.0f);
    const float4 t00 = tex_fetch(t, i, j), t10 = tex_fetch(t, i + 1, j);
    const float4 t01 = tex_fetch(t, i, j + 1), t11 = tex_fetch(t, i + 1, j + 1);
    const float w00 = (1.f - a) * (1.f - b), w10 = a * (1.f - b), w01 = (1.f - a) * b, w11 = a * b;
    return make_float4(w00 * t00.x + w10 * t10.x + w01 * t01.x + w11 * t11.x,
                       w00 * t00.y + w10 * t10.y + w01 * t01.y + w11 * t11.y,
                       w00 * t00.z + w10 * t10.z + w01 * t01.z + w11 * t11.z,
                       w00 * t00.w + w10 * t10.w + w01 * t01.w + w11 * t11.w);
}

// Registry ids (alphabetical, rasterizer.hip shader_names)
enum ShShaderId { kShCullHalf = 0, kShExpPos = 1, kShGaussDissolve = 2, kShHeartbeat = 3, kShDefault = 4 };
enum SplatShaderId {
    kSpCrack = 0, kSpCrackNoRecon = 1, kSpDissolve = 2, kSpNaiveOutline = 3, kSpQuantizeFlats = 4,
    kSpQuantizeLight = 5, kSpRoughnessOnly = 6, kSpDefault = 7, kSpStencil = 8, kSpWireframe = 9
};

struct ShShaderArgs {
    const int* idx;  // bucket: splat indices
    int n;
    float time, dt;
    float* pos;      // [P,3] working copies (the reference shades clones, rasterize_points.cu:117-122)
    float* scale;    // [P,3]
    float* rot;      // [P,4]
    float* opacity;  // [P]
    float* sh;       // [P,M,3]
    int M;
    const float* features;  // [P,S]
    int S;
    TexDesc tex0, tex1;
};

struct SplatShaderArgs {
    const int* idx;
    int n;
    int W, H;
    float time, dt;
    const float* pos;        // [P,3] (after the SH shaders)
    const float2* means2D;
    const float* depth_tex;  // [H*W] intermediate depth
    const float* stencil_tex;
    const float* viewmatrix_inv;
    const float* depths;
    const float* rgb;        // SH colour
    float4* conic_opacity;   // opacity is .w (modifiable)
    float* features;         // [P,S] working copy
    int S;
    float* stencils;
    float* stencil_opacity;
    float* out_rgb;          // shader colour
    TexDesc tex0;
};

// Post-process passes (postProcessShader.cu:177-374), registry ids in name order
enum PostShaderId {
    kPpBlurLighting = 0, kPpCrackReconstruction = 1, kPpInvert = 2, kPpOutline = 3, kPpQuantizeLighting = 4,
    kPpSobelFilter = 5, kPpDefault = 6, kPpTexturedShadows = 7, kPpToon = 8
};
constexpr int kMaxFusedPasses = 16;

// Screen buffers the passes read and write (the reference's PostProcessShaderBuffer views,
// postProcessShader.cu:13-39). Writes go to the live outputs as in the reference; the only pass
// that reads neighbours of a channel a pass writes (BlurLighting: incident light) reads a
// snapshot of that block instead of the reference's full 36-channel double buffer.
struct PostArgs {
    int W, H;
    const float* sh_color;      // out_color [H,W,3]
    const float* opacity;       // out_opacity [H,W]
    const float* depth;         // intermediate depth, re-rendered before the passes
    const float* stencil;       // intermediate stencil
    const float* surface_xyz;   // [H,W,3]
    const float* pseudonormal;  // [H,W,3]
    float* shader_color;        // [H,W,3]
    float* features;            // out_feature in the reference's 21-channel block layout, or null
    const float* incident_in;   // BlurLighting: snapshot of the incident-light block [H*W,3]
    TexDesc shadow;             // "shadow" (TexturedShadows / ToonShader)
    int n_pass;
    int pass[kMaxFusedPasses];
};

hipError_t launch_sh_shader(int id, const ShShaderArgs& a, hipStream_t st);
// Runs the passes ids[0..n) in order. Runs of pixel-local passes fuse into one launch; a
// BlurLighting pass snapshots the incident-light block into scratch (3*W*H floats) first.
hipError_t launch_post_passes(const int* ids, int n, const PostArgs& a, float* scratch, hipStream_t st);
bool post_pass_needs_features(int id);
bool post_pass_needs_shadow(int id);
hipError_t launch_splat_shader(int id, const SplatShaderArgs& a, hipStream_t st);
// texture names each shader samples (resolved by the host against the texture manager)
const char* sh_shader_texture(int id, int k);
const char* splat_shader_texture(int id);
// shaders that address the reference's 21-channel feature layout (ShShader.h / splatShader.h)
bool sh_shader_needs_features(int id);
bool splat_shader_needs_features(int id);
// texture manager registry (shaders.hip): name -> texture, plus the error texture
bool lookup_texture_manager(int64_t handle, const std::map<std::string, TexDesc>** names, TexDesc* error);
int texture_mode_channels(int mode);

}  // namespace r3dg
