/*
 * r3dg_hip.h -- C ABI of the MI355X-native relightable Gaussian-splat rasterizer.
 *
 * This is the drop-in boundary. Every entry point here is the plain-pointer form of one
 * function of the reference's pybind module `r3dg_rasterization._C`
 * (reference: r3dg-rasterization/ext.cu:21-35). The torch binding
 * relightable3dgaussian_amd/csrc/torch_ext.cpp re-exports them under the reference's names
 * with the reference's argument order and return tuples. No torch types appear here: device
 * buffers are raw pointers, the stream is a hipStream_t passed as void*, and the three opaque
 * state buffers of the reference (geomBuffer / binningBuffer / imgBuffer,
 * rasterize_points.cu:104-111) are obtained through caller-supplied allocation callbacks, the
 * C form of the reference's std::function<char*(size_t)> resize functors
 * (rasterize_points.cu:31-37).
 *
 * Conventions (as in the reference):
 *   - all float data is fp32, contiguous, on the current device;
 *   - an absent optional tensor (reference: empty tensor -> nullptr) is passed as NULL;
 *   - view/proj matrices are the transposed 4x4 torch matrices of scene/cameras.py:63-79
 *     (element m[4*c + r] multiplies coordinate c for output r);
 *   - image outputs are HWC (rasterize_points.cu:94-101); the feature output uses the layout
 *     documented at r3dg_feature_groups().
 * All functions return R3DG_OK (0) or a negative error code; r3dg_last_error() has the text.
 */
#ifndef R3DG_HIP_H
#define R3DG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: r3dg_raster_settings and r3dg_backward_outputs start with struct_size; r3dg_options */
#define R3DG_ABI_VERSION 2

enum {
    R3DG_OK = 0,
    R3DG_ERR_ARG = -1,         /* shape / argument error (reference: AT_ERROR -> RuntimeError) */
    R3DG_ERR_HIP = -2,         /* HIP runtime or kernel launch failure */
    R3DG_ERR_UNSUPPORTED = -3, /* feature outside this build's scope (DESIGN.md "Scope") */
    R3DG_ERR_ALLOC = -4        /* an allocation callback returned NULL */
};

typedef void* r3dg_stream_t;                                 /* hipStream_t */
typedef void* (*r3dg_alloc_fn)(void* ctx, size_t nbytes);    /* returns device memory, >= 256-B aligned */

int r3dg_abi_version(void);
const char* r3dg_last_error(void);

/* ---- library options (process-wide) ----------------------------------------------------------
 * Extensible structs carry their own size as the first field: a caller sets
 * struct_size = sizeof(the struct) as its header declares it, and the library rejects (R3DG_ERR_ARG)
 * a struct_size it does not know, so a binding built against another version of this header, or one
 * that forgot to zero-initialise the struct, fails loudly instead of reading garbage.
 *
 * No option is read from the environment on a launch. The one supported runtime option, the
 * backward's second reduction stage, starts from R3DG_BWD_REDUCE=rows|atomic, read once when the
 * library is loaded (default atomic); every field can be changed with r3dg_set_options. The test_*
 * fields select cross-check, negative-test and experiment variants for the test suite and the
 * measurement tools; production callers leave them 0. */
enum { R3DG_REDUCE_ATOMIC = 0, R3DG_REDUCE_ROWS = 1 };
typedef struct r3dg_options {
    size_t struct_size;       /* sizeof(r3dg_options) */
    int bwd_reduce;           /* R3DG_REDUCE_ATOMIC: (instance, wave) rows added into per-Gaussian sums with
                                 atomics (default, fastest; last bits depend on arrival order, as the
                                 reference's per-pixel atomicAdd); R3DG_REDUCE_ROWS: partial rows summed in a
                                 fixed order, bitwise reproducible */
    int prof_sort_markers;    /* r3dg_profile_*: also time the binning / sort stages (marker events) */
    int test_bwd_dpp;         /* backward blend by the DPP-reduction cross-check kernel (rows reduction) */
    int test_bwd_wterms;      /* 0 default (w in two bf16 terms); 1 / 3 (S 9..11, atomic): one term, the
                                 inexact reduction the gradient bar must reject, or three (exact) */
    int test_no_cull;         /* blends without the exact per-quadrant cull (same results) */
    int test_bin_atomic;      /* the global-atomic binning (the fallback above the LDS binning's tiles) */
    int test_bin_blocks;      /* > 0: cap on the LDS binning's workgroups (experiments) */
    int test_tile_order_spatial; /* backward tiles in the XCD-aware spatial order, not longest first */
    int test_bwd_srs;         /* > 0: row stride (floats) of the atomic per-Gaussian sums, rounded up to a
                                 multiple of 8 and to at least the X part + the six f64 moments */
    int test_bvh_lanes;       /* > 0: lanes per ray of the BVH opacity tracer (1, 2, 4, .. 64) */
    int test_bvh_sort;        /* 0 auto (Morton-sorted rays from 256k); 1 off; 2 on */
    int test_bvh_split;       /* 1: the static subtree-split tracer instead of the shared-stack groups */
    int test_bin_one_pass;    /* 1: the one-pass binning scatter (per-(workgroup, tile) runs) instead of the
                                 two passes through tile buckets (same results after the depth sort) */
} r3dg_options;
int r3dg_get_options(r3dg_options* out);   /* out->struct_size must be set */
int r3dg_set_options(const r3dg_options* in);

/* Feature output layout (replaces forward.cu:537-558, DESIGN.md "Feature layout").
 * Writes the channel-group sizes for S channels into groups[] and returns their count.
 * A group of size n starting at channel c0 is stored as a [H*W, n] block at offset c0*H*W
 * of the flat feature output. S=21 reproduces the reference's 3 scalar planes + six [HW,3]
 * blocks exactly; S=11 (training) uses [1,1,3,3,3]; any other S is planar [S,H,W]. */
int r3dg_feature_groups(int S, int* groups);

/* ---- rasterizer (rasterize_points.cu:39-181, rasterizer_impl.cu:213-529) ------------------- */

typedef struct r3dg_raster_settings {
    size_t struct_size; /* sizeof(r3dg_raster_settings) (ABI 2; checked) */
    int P;  /* number of Gaussians (means3D.size(0)) */
    int S;  /* feature channels (features.size(1)) */
    int D;  /* active SH degree */
    int M;  /* SH coefficients per Gaussian (sh.size(1)), 0 if sh absent */
    int W, H;
    float tan_fovx, tan_fovy, cx, cy;
    float scale_modifier;
    float time, dt;
    int prefiltered;
    int compute_pseudo_normal; /* reference spelling: computer_pseudo_normal */
    int debug;                 /* synchronise and check after every launch */
    const float* bg;           /* [3] */
    const float* viewmatrix;   /* [16] */
    const float* viewmatrix_inv;
    const float* projmatrix;
    const float* projmatrix_inv;
    const float* campos;       /* [3] */
    int64_t sh_shader_manager;    /* handle from r3dg_preprocess_model, 0 = all ShDefault */
    int64_t splat_shader_manager; /* handle from r3dg_preprocess_model, 0 = all SplatDefault */
    int64_t texture_manager;      /* 0 = none */
    const int64_t* post_passes;   /* host array of post-process pass handles, run in order after the
                                     blend (FORWARD::RunPostProcessShaders, forward.cu:973-1047);
                                     a non-empty list re-renders depth + stencil first
                                     (rasterizer_impl.cu:485-502) */
    int n_post_passes;
} r3dg_raster_settings;

typedef struct r3dg_gaussians {
    const float* means3D;        /* [P,3] */
    const float* features;       /* [P,S] or NULL when S == 0 */
    const float* colors_precomp; /* [P,3] or NULL (exactly one of colors_precomp / sh) */
    const float* opacity;        /* [P,1] */
    const float* scales;         /* [P,3] or NULL (exactly one of scales+rotations / cov3D_precomp) */
    const float* rotations;      /* [P,4] or NULL */
    const float* cov3D_precomp;  /* [P,6] or NULL */
    const float* sh;             /* [P,M,3] or NULL */
} r3dg_gaussians;

typedef struct r3dg_forward_outputs {
    float* color;        /* [H,W,3] */
    float* opacity;      /* [H,W,1] */
    float* depth;        /* [H,W,1] */
    float* stencil;      /* [H,W,1] */
    float* feature;      /* [H,W,S] storage, layout per r3dg_feature_groups */
    float* shader_color; /* [H,W,3] */
    float* normal;       /* [H,W,3] pseudo normal (zero where undefined) */
    float* surface_xyz;  /* [H,W,3] */
    int* radii;          /* [P] */
} r3dg_forward_outputs;

/* RasterizeGaussiansCUDA (rasterize_points.cu:39-181). The image state buffer holds n_contrib
 * (int32 [H,W]) at byte offset r3dg_image_state_n_contrib_offset(H, W). */
int r3dg_rasterize_gaussians(const r3dg_raster_settings* settings, const r3dg_gaussians* g,
                             const r3dg_forward_outputs* out, r3dg_alloc_fn geom_alloc, void* geom_ctx,
                             r3dg_alloc_fn binning_alloc, void* binning_ctx, r3dg_alloc_fn image_alloc,
                             void* image_ctx, int* num_rendered, r3dg_stream_t stream);

/* r3dg_rasterize_gaussians with a scratch allocator, called once per call: the forward-only
 * transients -- the binning's per-workgroup tile counts (up to 8 MiB, [workgroups, tiles] u32, used
 * only until the instances are scattered) and, with non-default splat shaders or post passes, the
 * shader colour / intermediate-pass records (16 B * P * (record float4s - 2) + 16 B * P) -- come
 * from scratch_alloc, which may hand out stream-ordered memory the caller frees as soon as the call
 * returns (the torch binding passes the caching allocator), instead of the tails of the image and
 * geometry states, which live as long as the autograd context. scratch_alloc NULL =
 * r3dg_rasterize_gaussians. */
int r3dg_rasterize_gaussians_ex(const r3dg_raster_settings* settings, const r3dg_gaussians* g,
                                const r3dg_forward_outputs* out, r3dg_alloc_fn geom_alloc, void* geom_ctx,
                                r3dg_alloc_fn binning_alloc, void* binning_ctx, r3dg_alloc_fn image_alloc,
                                void* image_ctx, r3dg_alloc_fn scratch_alloc, void* scratch_ctx, int* num_rendered,
                                r3dg_stream_t stream);

size_t r3dg_image_state_n_contrib_offset(int H, int W);

/* Bytes of the geometry state buffer for P Gaussians with S features (S < 0: the S-independent
 * part every per-Gaussian accessor reads, i.e. without the render records). Lets a binding check
 * a caller-supplied geomBuffer before handing it to r3dg_sh_color_grads. */
size_t r3dg_geom_state_bytes(int P, int S);

/* Debug / parity accessors into the opaque state buffers (tile keys, sort order, ranges). */
typedef struct r3dg_binning_view {
    const uint32_t* point_list;   /* [L] Gaussian ids in sorted order (reference point_list); the
                                     reference's sort key of position i is tile << 32 | depth bits
                                     of point_list[i], with the tile given by ranges */
    const uint32_t* ranges;       /* [tiles,2] from the image buffer */
    const uint32_t* point_offsets;/* [P] inclusive scan of tiles touched */
    const float* depths;          /* [P] */
    const float* means2D;         /* [P,2] */
    const float* conic_opacity;   /* [P,4] */
    const float* rgb;             /* [P,3] */
    const float* cov3D;           /* [P,6] */
    const uint8_t* clamped;       /* [P] bit c = channel c clamped */
} r3dg_binning_view;
int r3dg_state_view(int P, int H, int W, int L, void* geom, void* binning, void* image, r3dg_binning_view* view);

typedef struct r3dg_backward_grads {
    const float* dL_dout_color;   /* colour gradient */
    int color_hwc;                /* 0: [3,H,W] planar (reference contract, rasterize_points.cu:214-215); 1: [H,W,3] */
    const float* dL_dout_opacity; /* [H*W] */
    const float* dL_dout_depth;   /* [H*W] */
    const float* dL_dout_feature; /* feature gradient */
    int feature_native;           /* 0: [S,H,W] planar (reference, backward.cu:470-471); 1: forward output layout */
} r3dg_backward_grads;

typedef struct r3dg_backward_outputs {
    size_t struct_size;   /* sizeof(r3dg_backward_outputs) (ABI 2; checked) */
    float* dL_dmeans2D;   /* [P,3] (x, y, depth) */
    float* dL_dcolors;    /* [P,3] */
    float* dL_dopacity;   /* [P,1] */
    float* dL_dmeans3D;   /* [P,3] */
    float* dL_dfeatures;  /* [P,S] */
    float* dL_dcov3D;     /* [P,6] */
    float* dL_dsh;        /* [P,M,3] (may be NULL when M == 0) */
    float* dL_dscales;    /* [P,3] */
    float* dL_drotations; /* [P,4] */
    /* Optional chunked delivery (zero-initialised: one chunk, no callback). The per-Gaussian phase
     * (partial-row sums, cov2D / projection / SH / cov3D backward) runs over n_chunks contiguous
     * Gaussian ranges, 256-aligned, in order; after the kernels of [g_begin, g_end) are enqueued
     * on the stream, chunk_done(chunk_ctx, chunk, g_begin, g_end) is called on the host, so the
     * caller can start exchanging that range's gradients (an RCCL all-reduce on another stream)
     * while the next range computes. Results do not depend on n_chunks. */
    int n_chunks;
    void (*chunk_done)(void* ctx, int chunk, int g_begin, int g_end);
    void* chunk_ctx;
    /* Optional packed layout of the dense per-Gaussian gradients (0: dL_dmeans3D [P,3],
     * dL_dopacity [P,1], dL_dscales [P,3], dL_drotations [P,4], dL_dfeatures [P,S] as above). The
     * value 11 + S (the only other one accepted) is the row stride, in floats, of all five: the
     * caller points them at the columns 0, 3, 4, 7 and 11 of one [P, 11 + S] array, so a Gaussian
     * range of the five is one contiguous span -- one collective per chunk for the view-parallel
     * exchange (relightable3dgaussian_amd/view_parallel.py). */
    int dense_stride;
} r3dg_backward_outputs;

/* RasterizeGaussiansBackwardCUDA (rasterize_points.cu:183-275). Every output element is written
 * (no pre-zeroing needed). Deterministic: per-Gaussian sums have a fixed order. */
int r3dg_rasterize_gaussians_backward(const r3dg_raster_settings* settings, const r3dg_gaussians* g,
                                      const int* radii, const r3dg_backward_grads* grads, void* geom,
                                      void* binning, void* image, int num_rendered, int backward_geometry,
                                      r3dg_alloc_fn scratch_alloc, void* scratch_ctx,
                                      const r3dg_backward_outputs* out, r3dg_stream_t stream);

/* View-parallel SH-gradient exchange (relightable3dgaussian_amd/view_parallel.py). The SH part of
 * a view's gradient is rank-1 per Gaussian: dL/dsh[k][c] = Y_k(dir) * dRGB[c] with dir =
 * normalize(mean - campos) and dRGB the clamp-masked colour gradient (backward.cu:20-139). So
 * instead of all-reducing 3*M floats per Gaussian, ranks all-gather dRGB (3 floats) and every
 * rank rebuilds the sum over views.
 *   r3dg_sh_color_grads: dRGB of Gaussians [g0, g0 + n) of this view: dL_dcolors (the backward's
 *     output) with the channels whose SH colour the forward clamped at 0 zeroed (geom state).
 *   r3dg_sh_grad_from_views: dL_dsh rows [g0, g0 + n) = sum over the N views, in view order, of
 *     Y_k(normalize(mean - campos[v])) * drgb[v][i][c] for k < (degree+1)^2, 0 for k < M beyond;
 *     drgb is [N][n][3] (the views' dRGB of these Gaussians), campos [N][3]. */
int r3dg_sh_color_grads(int P, int g0, int n, void* geom, const float* dL_dcolors, float* drgb, r3dg_stream_t stream);
int r3dg_sh_grad_from_views(int g0, int n, int degree, int M, int N, const float* means3D, const float* campos,
                            const float* drgb, float* dL_dsh, r3dg_stream_t stream);

/* markVisible (rasterize_points.cu:277-295): present[i] = view-space z > 0.2 */
int r3dg_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                      uint8_t* present, r3dg_stream_t stream);

/* ---- render equation (render_equation.cu) ---------------------------------------------- */

typedef struct r3dg_brdf_inputs {
    int P, S_incident, S_direct, S_visibility, sample_num;
    const float* base_color;     /* [P,3] */
    const float* roughness;      /* [P,1] */
    const float* metallic;       /* [P,1] */
    const float* normals;        /* [P,3] */
    const float* viewdirs;       /* [P,3] */
    const float* incidents_shs;  /* [P,S_incident,3] */
    const float* direct_shs;     /* [1,S_direct,3] */
    const float* visibility_shs; /* [P,S_visibility,1] */
} r3dg_brdf_inputs;

/* RenderEquationForwardCUDA (render_equation.cu:688-726). rand_float [P,sample_num] is read
 * only when is_training (reference draws it with torch::rand at :708). */
int r3dg_render_equation_forward(const r3dg_brdf_inputs* in, int is_training, const float* rand_float,
                                 float* pbr, float* incident_dirs, float* diffuse_light, r3dg_stream_t stream);

/* RenderEquationForwardCUDA_complex (render_equation.cu:220-274), outputs in reference order. */
typedef struct r3dg_brdf_complex_outputs {
    float* pbr;                    /* [P,3] */
    float* incident_dirs;          /* [P,Ns,3] */
    float* incident_lights;        /* [P,Ns,3] */
    float* local_incident_lights;  /* [P,Ns,3] */
    float* global_incident_lights; /* [P,Ns,3] */
    float* incident_visibility;    /* [P,Ns,1] */
    float* diffuse_light;          /* [P,3] */
    float* local_diffuse_light;    /* [P,3] */
    float* accum;                  /* [P,1] */
    float* rgb_d;                  /* [P,3] */
    float* rgb_s;                  /* [P,3] */
} r3dg_brdf_complex_outputs;
int r3dg_render_equation_forward_complex(const r3dg_brdf_inputs* in, const r3dg_brdf_complex_outputs* out,
                                         r3dg_stream_t stream);

/* RenderEquationBackwardCUDA (render_equation.cu:494-547). Bug-compatible with the reference
 * kernel except that dL_ddirect_shs is reduced deterministically (the reference races). */
typedef struct r3dg_brdf_grads {
    float* dL_dbase_color;     /* [P,3] */
    float* dL_droughness;      /* [P,1] */
    float* dL_dmetallic;       /* [P,1] */
    float* dL_dnormals;        /* [P,3] */
    float* dL_dviewdirs;       /* [P,3] */
    float* dL_dincidents_shs;  /* [P,S_incident,3] */
    float* dL_ddirect_shs;     /* [1,S_direct,3] */
    float* dL_dvisibility_shs; /* [P,S_visibility,1] */
} r3dg_brdf_grads;
int r3dg_render_equation_backward(const r3dg_brdf_inputs* in, const float* incident_dirs, const float* dL_dpbr,
                                  const float* dL_ddiffuse_light, r3dg_alloc_fn scratch_alloc, void* scratch_ctx,
                                  const r3dg_brdf_grads* out, r3dg_stream_t stream);

/* ---- shader manager (shaderManager.cu, preprocessModel.cu, ShShader.cu, splatShader.cu) ---- */

enum { R3DG_SHADER_SH = 0, R3DG_SHADER_SPLAT = 1, R3DG_SHADER_POST = 2 };
/* Name -> handle maps (GetShShaderAddressMap & co., ShShader.cu:196-230, splatShader.cu:283-333,
 * postProcessShader.cu). Handles are opaque shader ids, not device function pointers. */
int r3dg_shader_count(int kind);
const char* r3dg_shader_name(int kind, int index);
int64_t r3dg_shader_handle(int kind, int index);

/* PreprocessModel (preprocessModel.cu:156-213): assigns SH and splat shaders by position
 * (SelectShadersCUDA, :17-59) and buckets splat indices per shader. Returns two manager
 * handles (host objects owning device index lists). */
int r3dg_preprocess_model(int P, const float* xyz, int64_t* sh_manager, int64_t* splat_manager,
                          r3dg_stream_t stream);
/* Build a manager from explicit per-splat shader handles (host array [P]); the GPU-bucketing
 * half of PreprocessModel without the position rules. */
int r3dg_create_shader_manager(int kind, int P, const int64_t* shader_handles_host, int64_t* manager,
                               r3dg_stream_t stream);
int r3dg_shader_manager_info(int64_t manager, int* n_shaders, int64_t* handles, int* instance_counts);

/* ---- profiling ------------------------------------------------------------------------------ */
/* When enabled, HIP events are recorded on the caller's stream immediately before and after the
 * tile-blend kernels (the roofline kernels of DESIGN.md), up to max_records launches each.
 * r3dg_profile_read synchronises on the recorded events, returns the launch count and summed
 * device time in ms for one kernel, and resets that kernel's records. */
enum { R3DG_PROF_RENDER_FWD = 0, R3DG_PROF_RENDER_BWD = 1, R3DG_PROF_GATHER_BWD = 2, R3DG_PROF_SORT = 3,
       R3DG_PROF_PREPROCESS = 4, R3DG_PROF_ROW_SUM = 5, R3DG_PROF_KINDS = 6 };
int r3dg_profile_enable(int max_records);
int r3dg_profile_read(int kernel, int* count, float* total_ms);

/* Texture mode helpers (utils/texture.cu EncodeTextureMode / EncodeWrapMode). */
/* ---- textures (utils/texture.cu, asset_processing/textureImport.py) ----------------------- */
/* AllocateTexture (texture.cu:86-101,103-226): a texture from a device pixel array [H, W, C],
 * C the channel count of the PIL mode `mode` (r3dg_encode_texture_mode: 1 for 1/L/P/I/F, 3 for
 * RGB/YCbCr/LAB/HSV, 4 for RGBA/CMYK). Stored as float4 texels (3-channel modes get alpha 1 as
 * CreatPaddedArrayFromBase does) and sampled in software with the CUDA texture rules: wrap_u/v
 * from r3dg_encode_wrap_mode, normalized or texel coordinates, bilinear filtering with 8-bit
 * fractional weights (point sampling for LAB/HSV). Returns an opaque handle. */
int r3dg_texture_create(const float* pixels, int width, int height, int mode, int wrap_u, int wrap_v,
                        int normalized, int64_t* texture, r3dg_stream_t stream);
/* UploadTexturesToDevice (texture.cu:237-246): named textures + the error texture a shader gets
 * for a missing name (TextureManager::GetTexture, texture.cu:298-314). Shaders resolve their
 * texture names against it at launch. */
int r3dg_texture_manager_create(int n, const char* const* names, const int64_t* textures, int64_t error_texture,
                                int64_t* manager);
int r3dg_encode_texture_mode(const char* mode);
int r3dg_encode_wrap_mode(const char* mode);

/* ---- training step on the device -------------------------------------
 * The reference keeps one nn.Parameter per attribute group and steps them with torch.optim.Adam
 * (scene/gaussian_model.py:581-620); densification edits every group and the Adam states with
 * boolean-mask indexing and torch.cat (gaussian_model.py:795-1062). Here all groups of one model
 * live in ONE flat fp32 buffer: group g is a [P, width[g]] block starting at P * sum(width[<g])
 * (the layout below), with exp_avg / exp_avg_sq buffers of the same layout. */
#define R3DG_MAX_GROUPS 16
typedef struct r3dg_param_layout {
    int P;                        /* Gaussians */
    int n_groups;                 /* <= R3DG_MAX_GROUPS */
    int width[R3DG_MAX_GROUPS];   /* floats per Gaussian of each group */
    int xyz, scaling, rotation, opacity; /* group index of these roles (scaling / opacity raw,
                                             i.e. before exp / sigmoid as the reference stores them) */
} r3dg_param_layout;

/* One torch.optim.Adam step (gaussian_model.py:615-620 `step`, lr per param group) over the
 * flat elements [lo, hi) of `param` (global indices; a rank of the sharded optimizer passes its
 * shard). grad, exp_avg, exp_avg_sq are shard-local arrays of hi - lo floats. lr_host[g] is group
 * g's learning rate; step is Adam's 1-based step count. Arithmetic as torch's Adam:
 * m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2; p += -(lr / (1 - b1^t)) m / (sqrt(v) /
 * sqrt(1 - b2^t) + eps), the bias corrections in double on the host. */
int r3dg_adam_step(const r3dg_param_layout* layout, float* param, const float* grad, float* exp_avg,
                   float* exp_avg_sq, int64_t lo, int64_t hi, const float* lr_host, double beta1, double beta2,
                   double eps, int step, r3dg_stream_t stream);

/* r3dg_adam_step with one Adam step count per group (torch keeps `state['step']` per parameter):
 * steps_host[g] is group g's 1-based count for this step, or <= 0 when the group has no gradient
 * this iteration -- torch.optim.Adam skips a parameter whose .grad is None (gaussian_model.py:615-617
 * zero_grad(set_to_none=True)), so its param, exp_avg and exp_avg_sq stay untouched. */
int r3dg_adam_step_groups(const r3dg_param_layout* layout, float* param, const float* grad, float* exp_avg,
                          float* exp_avg_sq, int64_t lo, int64_t hi, const float* lr_host, const int* steps_host,
                          double beta1, double beta2, double eps, r3dg_stream_t stream);

/* train.py:172-176 + add_densification_stats (gaussian_model.py:1055-1062) for the Gaussians
 * with radii > 0 (visibility_filter): max_radii2D = max(max_radii2D, radii); xyz_accum +=
 * |dL/dmeans2D[:, :2]| (rows of stride2d floats); normal_accum += |normalize(normal_grad, eps=1e-3)|
 * (skipped when normal_grad is NULL); denom += 1. */
int r3dg_densification_stats(int P, const float* dL_dmeans2D, int stride2d, const float* normal_grad,
                             const int* radii, float* xyz_accum, float* normal_accum, float* denom,
                             float* max_radii2D, r3dg_stream_t stream);

typedef struct r3dg_densify_args {
    float grad_threshold, grad_normal_threshold, percent_dense, extent, min_opacity;
    float max_screen_size; /* 0 = no screen/world size pruning (the reference's None) */
    int N;                 /* split children per Gaussian (2) */
    int prune_only;        /* 1: `prune` (gaussian_model.py:1045-1053), no clone / split */
} r3dg_densify_args;

/* densify_and_prune (gaussian_model.py:1025-1043; densify_and_clone :982-1023, densify_and_split
 * :926-980, prune_points :822-848, densification_postfix :880-924) or `prune` in one device pass
 * over the flat buffers. Result order is the reference's: surviving originals, then the clones,
 * then the split children (child k of every split Gaussian, k = 0..N-1). max_radii2D may be
 * NULL; as in the reference densify_and_prune's screen-size test never fires (the postfix has
 * zeroed max_radii2D), `prune` uses it. The split samples come from `randn`: called once with
 * n = 3 * N * n_split, it returns n standard-normal floats on the device (the reference draws
 * torch.normal(0, std)); the new buffers come from `alloc` (param, exp_avg, exp_avg_sq, each
 * P_new * sum(width) floats; clones and children get zero Adam state) and, when out_source is not
 * NULL, an int32 [P_new] map: the source Gaussian of each surviving original, -1 for new rows (the
 * caller slices its statistics with it, as prune_points does). counts = {originals kept, clones
 * kept, Gaussians split, children kept per k}. */
int r3dg_densify_and_prune(const r3dg_param_layout* layout, const float* param, const float* exp_avg,
                           const float* exp_avg_sq, const float* xyz_accum, const float* normal_accum,
                           const float* denom, const float* max_radii2D, const r3dg_densify_args* args,
                           r3dg_alloc_fn alloc, void* alloc_ctx, r3dg_alloc_fn randn, void* randn_ctx,
                           float** out_param, float** out_exp_avg, float** out_exp_avg_sq, int** out_source,
                           int* P_new, int* counts, r3dg_stream_t stream);

/* reset_opacity (gaussian_model.py:688-691): opacity = inverse_sigmoid(min(sigmoid(opacity), 0.01))
 * and the opacity group's Adam state zeroed (replace_tensor_to_optimizer). */
int r3dg_reset_opacity(const r3dg_param_layout* layout, float* param, float* exp_avg, float* exp_avg_sq,
                       r3dg_stream_t stream);

/* ---- BVH visibility tracer (reference module bvh_tracing._C,
 *      bvh/src/bindings.cpp:9-11) ------------------------------------------------------------
 * Tree layout (the reference's, bvh/__init__.py:31-37): nodes int32 [2P-1, 5] rows
 * {parent, left, right, gaussian, leaf count}, internal nodes 0..P-2, leaf P-1+i holds the i-th
 * Gaussian in Morton order; aabbs f32 [2P-1, 6] rows {lower xyz, upper xyz}; morton u64 [P]
 * sorted keys (30-bit Morton code << 31 | Gaussian index). */

/* RayTracer.__init__ leaf boxes (bvh/__init__.py:29-59): per Gaussian the min / max of the 8
 * corners mean ± 3 s_k R[:, k] (R = build_rotation of the re-normalised quaternion, r x y z),
 * written as [P, 6] rows to leaf_aabbs (pass aabbs + 6 (P - 1) to fill the tree's leaf rows). */
int r3dg_bvh_leaf_aabbs(int P, const float* means3D, const float* scales, const float* rotations,
                        float* leaf_aabbs, r3dg_stream_t stream);

/* create_bvh (bvh/src/bvh.cu:8-26, construct.cu:148-265): Karras LBVH over the leaf boxes in
 * aabbs rows P-1..2P-2 (input, in Gaussian order). Writes every field of nodes, the internal and
 * (Morton-sorted) leaf rows of aabbs, and morton. P >= 1. Scratch from scratch_alloc. */
int r3dg_bvh_build(int P, int32_t* nodes, float* aabbs, uint64_t* morton, r3dg_alloc_fn scratch_alloc,
                   void* scratch_ctx, r3dg_stream_t stream);

/* trace_bvh_opacity (bvh/src/bvh.cu:87-117, trace.cu:199-286): per ray the transmittance through
 * the Gaussians it meets (cov3D_inv: [P, 6] upper-triangular inverse covariance, the
 * get_inverse_covariance of gaussian_model.py:410-413). Outputs: num_contributes int32 [R],
 * rendered_opacity f32 [R] (0 and 0 once the transmittance drops below 0.9). num_gaussians = P of
 * the tree (2P-1 nodes); it bounds the traversal, so a malformed tree cannot hang the GPU.
 * Scratch from scratch_alloc: 128 B per Gaussian (packed node and Gaussian records), plus 16 B per
 * ray and a radix-sort workspace when the rays are traced in Morton order (>= 256k rays). */
int r3dg_bvh_trace_opacity(int num_rays, int num_gaussians, const int32_t* nodes, const float* aabbs, const float* rays_o,
                           const float* rays_d, const float* means3D, const float* cov3D_inv,
                           const float* opacities, const float* normals, int32_t* num_contributes,
                           float* rendered_opacity, r3dg_alloc_fn scratch_alloc, void* scratch_ctx,
                           r3dg_stream_t stream);

/* trace_bvh (bvh/src/bvh.cu:28-85, trace.cu:8-196): per ray the Gaussians of every crossed
 * subtree of <= 4 leaves, sorted by (ray, t); num_contributes int32 [R] is their count per ray.
 * The three lists (int32 [L], f32 [L, 3], int32 [L]) come from alloc; *num_rendered = L (one
 * blocking device-to-host copy, as the reference). The reference's covs3D / opacities arguments
 * do not enter its arithmetic and are not taken here. */
int r3dg_bvh_trace(int num_rays, int num_gaussians, const int32_t* nodes, const float* aabbs, const float* rays_o,
                   const float* rays_d, const float* means3D, int32_t* num_contributes, r3dg_alloc_fn alloc,
                   void* alloc_ctx, int* num_rendered, int32_t** point_list, float** position_list,
                   int32_t** ray_id_list, r3dg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* R3DG_HIP_H */
