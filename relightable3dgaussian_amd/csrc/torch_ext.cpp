// torch_ext.cpp -- pybind module `_C`: the reference operator surface over the C ABI.
//
// Mirrors r3dg_rasterization._C (reference r3dg-rasterization/ext.cu:21-35): the same 14
// function names, argument order and return tuples, so gaussian_renderer/neilf.py and
// scene/gaussian_model.py call it unchanged. Documented extensions:
//   (1) None / 0 shader-manager, texture and post-pass handles mean "defaults";
//   (2) every launch goes on the current HIP stream of means3D's device, and all buffers
//       (including the three state buffers) live on that device;
//   (3) extra entry points used by the shipped wrapper and the parity tests
//       (rasterize_gaussians_backward_ex, render_equation_forward_with_rand, rasterizer_state,
//       feature_groups, create_shader_manager, shader_manager_info).
// Errors from the C ABI surface as RuntimeError with the library's message.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <map>
#include <optional>
#include <string>
#include <tuple>
#include <vector>

#include "r3dg_hip.h"

namespace {

void check(int rc, const char* what) {
    if (rc != R3DG_OK) throw std::runtime_error(std::string(what) + ": " + r3dg_last_error());
}

// empty tensor (numel 0) means "absent", as the reference's data_ptr of an empty tensor
const float* opt_ptr(const torch::Tensor& t) { return t.numel() == 0 ? nullptr : t.data_ptr<float>(); }

// every entry point's inputs go to its first tensor's device, which must be a GPU: a host tensor
// is refused here, before its pointer could reach a kernel (there is no CPU path)
torch::Tensor dev_contig(const torch::Tensor& t, const torch::Device& dev) {
    TORCH_CHECK(dev.is_cuda(), "the HIP rasterizer takes tensors on a GPU device, got ", dev);
    if (t.numel() == 0) return t;
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, "expected a float32 tensor");
    return t.to(dev).contiguous();
}

struct TensorAlloc {
    torch::TensorOptions opts;
    torch::Tensor t;
};
void* tensor_alloc(void* ctx, size_t n) {
    auto* a = static_cast<TensorAlloc*>(ctx);
    a->t = torch::empty({(int64_t)std::max<size_t>(n, 256)}, a->opts);
    return a->t.data_ptr();
}

r3dg_stream_t stream_of(const torch::Device& dev) {
    return (r3dg_stream_t)c10::hip::getCurrentHIPStream(dev.index()).stream();
}

using FwdResult = std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
                             torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
                             torch::Tensor, torch::Tensor, torch::Tensor>;

// RasterizeGaussiansCUDA (rasterize_points.cu:39-181)
FwdResult rasterize_gaussians(const torch::Tensor& background, double time, double dt, const torch::Tensor& means3D,
                              const torch::Tensor& features, const torch::Tensor& colors,
                              const torch::Tensor& opacity, const torch::Tensor& scales,
                              const torch::Tensor& rotations, double scale_modifier,
                              const torch::Tensor& cov3D_precomp, const torch::Tensor& viewmatrix,
                              const torch::Tensor& viewmatrix_inv, const torch::Tensor& projmatrix,
                              const torch::Tensor& projmatrix_inv, double tan_fovx, double tan_fovy, double cx,
                              double cy, int64_t image_height, int64_t image_width, const torch::Tensor& sh,
                              int64_t degree, const torch::Tensor& campos, bool prefiltered,
                              bool computer_pseudo_normal, std::optional<int64_t> d_textureManager_ptr,
                              std::optional<int64_t> h_shShaderManager_ptr,
                              std::optional<int64_t> h_splatShaderManager_ptr,
                              std::optional<std::vector<int64_t>> postProcessingPasses, bool debug) {
    if (means3D.ndimension() != 2 || means3D.size(1) != 3)
        throw std::runtime_error("means3D must have dimensions (num_points, 3)");
    TORCH_CHECK(means3D.is_cuda(), "means3D must be a GPU tensor (this build has no CPU path)");
    const torch::Device dev = means3D.device();
    const c10::OptionalDeviceGuard guard(dev);
    const int P = (int)means3D.size(0);
    const int S = features.numel() == 0 && features.dim() < 2 ? 0 : (int)features.size(1);
    const int H = (int)image_height, W = (int)image_width;
    auto fopt = means3D.options().dtype(torch::kFloat32);

    auto m3 = dev_contig(means3D, dev), ft = dev_contig(features, dev), co = dev_contig(colors, dev);
    auto op = dev_contig(opacity, dev), sc = dev_contig(scales, dev), ro = dev_contig(rotations, dev);
    auto c3 = dev_contig(cov3D_precomp, dev), shc = dev_contig(sh, dev), bg = dev_contig(background, dev);
    auto vm = dev_contig(viewmatrix, dev), vmi = dev_contig(viewmatrix_inv, dev);
    auto pm = dev_contig(projmatrix, dev), pmi = dev_contig(projmatrix_inv, dev), cp = dev_contig(campos, dev);

    torch::Tensor out_color = torch::empty({H, W, 3}, fopt);
    torch::Tensor out_opacity = torch::empty({H, W, 1}, fopt);
    torch::Tensor out_depth = torch::empty({H, W, 1}, fopt);
    torch::Tensor out_stencil = torch::empty({H, W, 1}, fopt);
    torch::Tensor out_feature = torch::empty({H, W, S}, fopt);
    torch::Tensor out_shader = torch::empty({H, W, 3}, fopt);
    torch::Tensor out_normal = torch::empty({H, W, 3}, fopt);
    torch::Tensor out_xyz = torch::empty({H, W, 3}, fopt);
    torch::Tensor radii = torch::empty({P}, means3D.options().dtype(torch::kInt32));

    auto bopt = torch::TensorOptions().dtype(torch::kUInt8).device(dev);
    TensorAlloc ga{bopt, torch::empty({0}, bopt)}, ba{bopt, torch::empty({0}, bopt)}, ia{bopt, torch::empty({0}, bopt)};

    std::vector<int64_t> passes = postProcessingPasses.value_or(std::vector<int64_t>{});
    r3dg_raster_settings s{};
    s.struct_size = sizeof(s);
    s.P = P; s.S = S; s.D = (int)degree; s.M = shc.numel() == 0 ? 0 : (int)shc.size(1);
    s.W = W; s.H = H;
    s.tan_fovx = (float)tan_fovx; s.tan_fovy = (float)tan_fovy; s.cx = (float)cx; s.cy = (float)cy;
    s.scale_modifier = (float)scale_modifier; s.time = (float)time; s.dt = (float)dt;
    s.prefiltered = prefiltered; s.compute_pseudo_normal = computer_pseudo_normal; s.debug = debug;
    s.bg = bg.data_ptr<float>();
    s.viewmatrix = vm.data_ptr<float>(); s.viewmatrix_inv = opt_ptr(vmi);
    s.projmatrix = pm.data_ptr<float>(); s.projmatrix_inv = opt_ptr(pmi);
    s.campos = cp.data_ptr<float>();
    s.sh_shader_manager = h_shShaderManager_ptr.value_or(0);
    s.splat_shader_manager = h_splatShaderManager_ptr.value_or(0);
    s.texture_manager = d_textureManager_ptr.value_or(0);
    s.post_passes = passes.data();
    s.n_post_passes = (int)passes.size();
    r3dg_gaussians g{};
    g.means3D = m3.data_ptr<float>(); g.features = opt_ptr(ft); g.colors_precomp = opt_ptr(co);
    g.opacity = opt_ptr(op); g.scales = opt_ptr(sc); g.rotations = opt_ptr(ro);
    g.cov3D_precomp = opt_ptr(c3); g.sh = opt_ptr(shc);
    r3dg_forward_outputs o{};
    o.color = out_color.data_ptr<float>(); o.opacity = out_opacity.data_ptr<float>();
    o.depth = out_depth.data_ptr<float>(); o.stencil = out_stencil.data_ptr<float>();
    o.feature = S > 0 ? out_feature.data_ptr<float>() : nullptr; o.shader_color = out_shader.data_ptr<float>();
    o.normal = out_normal.data_ptr<float>(); o.surface_xyz = out_xyz.data_ptr<float>();
    o.radii = P > 0 ? radii.data_ptr<int>() : nullptr;
    int rendered = 0;
    // the binning's tile counts: transient, returned to the caching allocator (stream-ordered) on exit
    TensorAlloc hist{bopt, torch::empty({0}, bopt)};
    check(r3dg_rasterize_gaussians_ex(&s, &g, &o, tensor_alloc, &ga, tensor_alloc, &ba, tensor_alloc, &ia, tensor_alloc,
                                      &hist, &rendered, stream_of(dev)),
          "rasterize_gaussians");
    // n_contrib is a view into the image state buffer (reference: from_blob, rasterize_points.cu:179)
    const int64_t off = (int64_t)r3dg_image_state_n_contrib_offset(H, W);
    torch::Tensor n_contrib = ia.t.narrow(0, off, (int64_t)H * W * 4).view(torch::kInt32).view({H, W, 1});
    return {rendered, n_contrib, out_color, out_opacity, out_depth, out_stencil, out_feature, out_shader,
            out_normal, out_xyz, radii, ga.t, ba.t, ia.t};
}

using BwdResult = std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
                             torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>;

BwdResult backward_impl(const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& features,
                        const torch::Tensor& radii, const torch::Tensor& colors, const torch::Tensor& scales,
                        const torch::Tensor& rotations, double scale_modifier, const torch::Tensor& cov3D_precomp,
                        const torch::Tensor& viewmatrix, const torch::Tensor& projmatrix, double tan_fovx,
                        double tan_fovy, const torch::Tensor& dL_dout_color, const torch::Tensor& dL_dout_opacity,
                        const torch::Tensor& dL_dout_depth, const torch::Tensor& dL_dout_feature,
                        const torch::Tensor& sh, int64_t degree, const torch::Tensor& campos,
                        const torch::Tensor& geomBuffer, int64_t R, const torch::Tensor& binningBuffer,
                        const torch::Tensor& imageBuffer, bool backward_geometry, bool debug, int H, int W,
                        bool color_hwc, bool feature_native, int n_chunks = 1,
                        const py::object& chunk_cb = py::none(), bool packed_dense = false) {
    const torch::Device dev = means3D.device();
    const c10::OptionalDeviceGuard guard(dev);
    const int P = (int)means3D.size(0);
    const int S = features.numel() == 0 && features.dim() < 2 ? 0 : (int)features.size(1);
    const int M = sh.numel() == 0 ? 0 : (int)sh.size(1);
    auto fopt = means3D.options().dtype(torch::kFloat32);
    // packed_dense: the five dense gradients are column views of one [P, 11 + S] array (means3D 3,
    // opacity 1, scales 3, rotations 4, features S), so a Gaussian range of them is one contiguous
    // span (r3dg_backward_outputs.dense_stride; one collective per chunk in view_parallel.py)
    const int DW = 11 + S;
    torch::Tensor dense = packed_dense ? torch::empty({P, DW}, fopt) : torch::Tensor();
    torch::Tensor dL_dmeans3D = packed_dense ? dense.narrow(1, 0, 3) : torch::empty({P, 3}, fopt);
    torch::Tensor dL_dmeans2D = torch::empty({P, 3}, fopt);
    torch::Tensor dL_dfeatures = packed_dense ? dense.narrow(1, 11, S) : torch::empty({P, S}, fopt);
    torch::Tensor dL_dcolors = torch::empty({P, 3}, fopt);
    torch::Tensor dL_dopacity = packed_dense ? dense.narrow(1, 3, 1) : torch::empty({P, 1}, fopt);
    torch::Tensor dL_dcov3D = torch::empty({P, 6}, fopt);
    torch::Tensor dL_dsh = torch::empty({P, M, 3}, fopt);
    torch::Tensor dL_dscales = packed_dense ? dense.narrow(1, 4, 3) : torch::empty({P, 3}, fopt);
    torch::Tensor dL_drotations = packed_dense ? dense.narrow(1, 7, 4) : torch::empty({P, 4}, fopt);
    if (P == 0) return {dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dfeatures, dL_dcov3D, dL_dsh,
                        dL_dscales, dL_drotations};

    auto m3 = dev_contig(means3D, dev), ft = dev_contig(features, dev), co = dev_contig(colors, dev);
    auto sc = dev_contig(scales, dev), ro = dev_contig(rotations, dev), c3 = dev_contig(cov3D_precomp, dev);
    auto shc = dev_contig(sh, dev), bg = dev_contig(background, dev), vm = dev_contig(viewmatrix, dev);
    auto pm = dev_contig(projmatrix, dev), cp = dev_contig(campos, dev);
    auto gc = dev_contig(dL_dout_color, dev), go = dev_contig(dL_dout_opacity, dev);
    auto gd = dev_contig(dL_dout_depth, dev), gf = dev_contig(dL_dout_feature, dev);
    torch::Tensor rad = radii.to(dev).to(torch::kInt32).contiguous();

    r3dg_raster_settings s{};
    s.struct_size = sizeof(s);
    s.P = P; s.S = S; s.D = (int)degree; s.M = M; s.W = W; s.H = H;
    s.tan_fovx = (float)tan_fovx; s.tan_fovy = (float)tan_fovy; s.scale_modifier = (float)scale_modifier;
    s.debug = debug;
    s.bg = bg.data_ptr<float>(); s.viewmatrix = vm.data_ptr<float>(); s.projmatrix = pm.data_ptr<float>();
    s.campos = cp.data_ptr<float>();
    r3dg_gaussians g{};
    g.means3D = m3.data_ptr<float>(); g.features = opt_ptr(ft); g.colors_precomp = opt_ptr(co);
    g.scales = opt_ptr(sc); g.rotations = opt_ptr(ro); g.cov3D_precomp = opt_ptr(c3); g.sh = opt_ptr(shc);
    r3dg_backward_grads gr{};
    gr.dL_dout_color = gc.data_ptr<float>(); gr.color_hwc = color_hwc;
    gr.dL_dout_opacity = go.data_ptr<float>(); gr.dL_dout_depth = gd.data_ptr<float>();
    gr.dL_dout_feature = S > 0 ? gf.data_ptr<float>() : nullptr; gr.feature_native = feature_native;
    r3dg_backward_outputs o{};
    o.struct_size = sizeof(o);
    o.dL_dmeans2D = dL_dmeans2D.data_ptr<float>(); o.dL_dcolors = dL_dcolors.data_ptr<float>();
    o.dL_dopacity = dL_dopacity.data_ptr<float>(); o.dL_dmeans3D = dL_dmeans3D.data_ptr<float>();
    o.dL_dfeatures = S > 0 ? dL_dfeatures.data_ptr<float>() : nullptr; o.dL_dcov3D = dL_dcov3D.data_ptr<float>();
    o.dL_dsh = M > 0 ? dL_dsh.data_ptr<float>() : nullptr; o.dL_dscales = dL_dscales.data_ptr<float>();
    o.dL_drotations = dL_drotations.data_ptr<float>();
    o.dense_stride = packed_dense ? DW : 0;
    // chunked delivery: the Python callable runs (GIL held: we are inside the pybind call) after
    // each Gaussian range's kernels are enqueued; an exception is re-raised after the C call
    struct ChunkCtx {
        const py::object* cb;
        py::tuple outs;  // the 9 output tensors, handed to the callback
        bool failed = false;
        std::string what;
    } cctx{&chunk_cb, packed_dense ? py::make_tuple(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dfeatures,
                                                    dL_dcov3D, dL_dsh, dL_dscales, dL_drotations, dense)
                                   : py::make_tuple(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dfeatures,
                                                    dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)};
    o.n_chunks = n_chunks;
    if (!chunk_cb.is_none()) {
        o.chunk_ctx = &cctx;
        o.chunk_done = [](void* ctx, int c, int g0, int g1) {
            auto* k = static_cast<ChunkCtx*>(ctx);
            if (k->failed) return;
            try {
                (*k->cb)(c, g0, g1, k->outs);
            } catch (const std::exception& e) {
                k->failed = true;
                k->what = e.what();
            }
        };
    }
    auto bopt = torch::TensorOptions().dtype(torch::kUInt8).device(dev);
    TensorAlloc scratch{bopt, torch::empty({0}, bopt)};
    check(r3dg_rasterize_gaussians_backward(&s, &g, rad.data_ptr<int>(), &gr, geomBuffer.data_ptr(),
                                            binningBuffer.data_ptr(), imageBuffer.data_ptr(), (int)R,
                                            backward_geometry, tensor_alloc, &scratch, &o, stream_of(dev)),
          "rasterize_gaussians_backward");
    TORCH_CHECK(!cctx.failed, "rasterize_gaussians_backward: chunk callback raised: ", cctx.what);
    return {dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dfeatures, dL_dcov3D, dL_dsh, dL_dscales,
            dL_drotations};
}

// RasterizeGaussiansBackwardCUDA (rasterize_points.cu:183-275): grads are CHW / planar.
BwdResult rasterize_gaussians_backward(const torch::Tensor& background, const torch::Tensor& means3D,
                                       const torch::Tensor& features, const torch::Tensor& radii,
                                       const torch::Tensor& colors, const torch::Tensor& scales,
                                       const torch::Tensor& rotations, double scale_modifier,
                                       const torch::Tensor& cov3D_precomp, const torch::Tensor& viewmatrix,
                                       const torch::Tensor& projmatrix, double tan_fovx, double tan_fovy,
                                       const torch::Tensor& dL_dout_color, const torch::Tensor& dL_dout_opacity,
                                       const torch::Tensor& dL_dout_depth, const torch::Tensor& dL_dout_feature,
                                       const torch::Tensor& sh, int64_t degree, const torch::Tensor& campos,
                                       const torch::Tensor& geomBuffer, int64_t R, const torch::Tensor& binningBuffer,
                                       const torch::Tensor& imageBuffer, bool backward_geometry, bool debug) {
    const int H = (int)dL_dout_color.size(1), W = (int)dL_dout_color.size(2);
    return backward_impl(background, means3D, features, radii, colors, scales, rotations, scale_modifier,
                         cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_opacity,
                         dL_dout_depth, dL_dout_feature, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                         backward_geometry, debug, H, W, false, false);
}

// Same, taking the forward's own output layouts (HWC colour, native feature layout): the
// shipped autograd wrapper uses this so no transposes are needed.
BwdResult rasterize_gaussians_backward_ex(const torch::Tensor& background, const torch::Tensor& means3D,
                                          const torch::Tensor& features, const torch::Tensor& radii,
                                          const torch::Tensor& colors, const torch::Tensor& scales,
                                          const torch::Tensor& rotations, double scale_modifier,
                                          const torch::Tensor& cov3D_precomp, const torch::Tensor& viewmatrix,
                                          const torch::Tensor& projmatrix, double tan_fovx, double tan_fovy,
                                          const torch::Tensor& dL_dout_color, const torch::Tensor& dL_dout_opacity,
                                          const torch::Tensor& dL_dout_depth, const torch::Tensor& dL_dout_feature,
                                          const torch::Tensor& sh, int64_t degree, const torch::Tensor& campos,
                                          const torch::Tensor& geomBuffer, int64_t R,
                                          const torch::Tensor& binningBuffer, const torch::Tensor& imageBuffer,
                                          bool backward_geometry, bool debug, int64_t H, int64_t W) {
    return backward_impl(background, means3D, features, radii, colors, scales, rotations, scale_modifier,
                         cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_opacity,
                         dL_dout_depth, dL_dout_feature, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                         backward_geometry, debug, (int)H, (int)W, true, true);
}

// rasterize_gaussians_backward_ex with chunked delivery (include/r3dg_hip.h r3dg_backward_outputs):
// chunk_cb(chunk, g_begin, g_end, outputs) is called once the gradients of Gaussians [g_begin,
// g_end) are enqueued (outputs = the 9 result tensors), e.g. to start their all-reduce on a
// communication stream (view_parallel.py).
BwdResult rasterize_gaussians_backward_chunked(
    const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& features,
    const torch::Tensor& radii, const torch::Tensor& colors, const torch::Tensor& scales,
    const torch::Tensor& rotations, double scale_modifier, const torch::Tensor& cov3D_precomp,
    const torch::Tensor& viewmatrix, const torch::Tensor& projmatrix, double tan_fovx, double tan_fovy,
    const torch::Tensor& dL_dout_color, const torch::Tensor& dL_dout_opacity, const torch::Tensor& dL_dout_depth,
    const torch::Tensor& dL_dout_feature, const torch::Tensor& sh, int64_t degree, const torch::Tensor& campos,
    const torch::Tensor& geomBuffer, int64_t R, const torch::Tensor& binningBuffer, const torch::Tensor& imageBuffer,
    bool backward_geometry, bool debug, int64_t H, int64_t W, bool color_hwc, bool feature_native, int64_t n_chunks,
    const py::object& chunk_cb) {
    return backward_impl(background, means3D, features, radii, colors, scales, rotations, scale_modifier,
                         cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_opacity,
                         dL_dout_depth, dL_dout_feature, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                         backward_geometry, debug, (int)H, (int)W, color_hwc, feature_native, (int)n_chunks, chunk_cb);
}

// rasterize_gaussians_backward_chunked with the dense gradients packed (packed_dense above): the
// callback's outputs carry a 10th tensor, the [P, 11 + S] array whose rows [g_begin, g_end) hold
// the chunk's means3D / opacity / scales / rotations / features gradients contiguously.
BwdResult rasterize_gaussians_backward_chunked_packed(
    const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& features,
    const torch::Tensor& radii, const torch::Tensor& colors, const torch::Tensor& scales,
    const torch::Tensor& rotations, double scale_modifier, const torch::Tensor& cov3D_precomp,
    const torch::Tensor& viewmatrix, const torch::Tensor& projmatrix, double tan_fovx, double tan_fovy,
    const torch::Tensor& dL_dout_color, const torch::Tensor& dL_dout_opacity, const torch::Tensor& dL_dout_depth,
    const torch::Tensor& dL_dout_feature, const torch::Tensor& sh, int64_t degree, const torch::Tensor& campos,
    const torch::Tensor& geomBuffer, int64_t R, const torch::Tensor& binningBuffer, const torch::Tensor& imageBuffer,
    bool backward_geometry, bool debug, int64_t H, int64_t W, bool color_hwc, bool feature_native, int64_t n_chunks,
    const py::object& chunk_cb) {
    return backward_impl(background, means3D, features, radii, colors, scales, rotations, scale_modifier,
                         cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_opacity,
                         dL_dout_depth, dL_dout_feature, sh, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                         backward_geometry, debug, (int)H, (int)W, color_hwc, feature_native, (int)n_chunks, chunk_cb,
                         true);
}

// View-parallel SH-gradient exchange (include/r3dg_hip.h): this view's clamp-masked colour
// gradients of Gaussians [g0, g1) (the rank's all-gather payload) ...
torch::Tensor sh_color_grads(const torch::Tensor& geomBuffer, int64_t P, const torch::Tensor& dL_dcolors, int64_t g0,
                             int64_t g1) {
    const torch::Device dev = dL_dcolors.device();
    const c10::OptionalDeviceGuard guard(dev);
    TORCH_CHECK(dev.is_cuda() && dL_dcolors.is_contiguous() && dL_dcolors.scalar_type() == torch::kFloat32 &&
                    dL_dcolors.numel() == 3 * P && 0 <= g0 && g0 <= g1 && g1 <= P,
                "sh_color_grads: dL_dcolors must be a contiguous float32 CUDA [P,3] tensor, 0 <= g0 <= g1 <= P");
    TORCH_CHECK(geomBuffer.device() == dev && geomBuffer.is_contiguous() &&
                    (size_t)geomBuffer.nbytes() >= r3dg_geom_state_bytes((int)P, -1),
                "sh_color_grads: geomBuffer must be the forward's geometry state for these P Gaussians, on the "
                "gradients' device");
    auto out = torch::empty({g1 - g0, 3}, dL_dcolors.options());
    check(r3dg_sh_color_grads((int)P, (int)g0, (int)(g1 - g0), geomBuffer.data_ptr(), dL_dcolors.data_ptr<float>(),
                              out.data_ptr<float>(), stream_of(dev)),
          "sh_color_grads");
    return out;
}

// ... and the sum over the N views of their SH gradients, rebuilt from the gathered [N, n, 3]
// colour gradients and the views' camera centres [N, 3], into rows [g0, g0 + n) of dL_dsh.
void sh_grad_from_views(const torch::Tensor& means3D, const torch::Tensor& campos, const torch::Tensor& drgb,
                        int64_t degree, int64_t g0, torch::Tensor& dL_dsh) {
    const torch::Device dev = means3D.device();
    const c10::OptionalDeviceGuard guard(dev);
    TORCH_CHECK(drgb.dim() == 3 && drgb.size(2) == 3 && campos.dim() == 2 && campos.size(1) == 3 &&
                    campos.size(0) == drgb.size(0) && dL_dsh.dim() == 3 && dL_dsh.size(2) == 3 &&
                    dL_dsh.is_contiguous() && g0 >= 0 && g0 + drgb.size(1) <= dL_dsh.size(0),
                "sh_grad_from_views: drgb [N,n,3], campos [N,3], dL_dsh [P,M,3] contiguous");
    TORCH_CHECK(means3D.dim() == 2 && means3D.size(1) == 3 && means3D.size(0) >= g0 + drgb.size(1),
                "sh_grad_from_views: means3D must be [P,3] with P >= g0 + n");
    TORCH_CHECK(dL_dsh.device() == dev && dL_dsh.scalar_type() == torch::kFloat32 && dL_dsh.size(1) <= 16 &&
                    degree >= 0 && degree <= 3 && (degree + 1) * (degree + 1) <= dL_dsh.size(1),
                "sh_grad_from_views: dL_dsh must be a float32 [P,M,3] tensor on means3D's device, degree 0..3 with "
                "(degree+1)^2 <= M <= 16");
    auto m3 = dev_contig(means3D, dev), cp = dev_contig(campos, dev), d = dev_contig(drgb, dev);
    check(r3dg_sh_grad_from_views((int)g0, (int)drgb.size(1), (int)degree, (int)dL_dsh.size(1), (int)drgb.size(0),
                                  m3.data_ptr<float>(), cp.data_ptr<float>(), d.data_ptr<float>(),
                                  dL_dsh.data_ptr<float>(), stream_of(dev)),
          "sh_grad_from_views");
}

torch::Tensor mark_visible(torch::Tensor& means3D, torch::Tensor& viewmatrix, torch::Tensor& projmatrix) {
    const torch::Device dev = means3D.device();
    const c10::OptionalDeviceGuard guard(dev);
    const int P = (int)means3D.size(0);
    torch::Tensor present = torch::zeros({P}, means3D.options().dtype(torch::kBool));
    if (P == 0) return present;
    auto m3 = dev_contig(means3D, dev), vm = dev_contig(viewmatrix, dev), pm = dev_contig(projmatrix, dev);
    check(r3dg_mark_visible(P, m3.data_ptr<float>(), vm.data_ptr<float>(), pm.data_ptr<float>(),
                            (uint8_t*)present.data_ptr<bool>(), stream_of(dev)),
          "mark_visible");
    return present;
}

r3dg_brdf_inputs brdf_inputs(const std::vector<torch::Tensor>& t, int sample_num) {
    r3dg_brdf_inputs in{};
    in.P = (int)t[0].size(0);
    in.S_incident = (int)t[5].size(1);
    in.S_direct = (int)t[6].size(1);
    in.S_visibility = (int)t[7].size(1);
    in.sample_num = sample_num;
    in.base_color = t[0].data_ptr<float>(); in.roughness = t[1].data_ptr<float>();
    in.metallic = t[2].data_ptr<float>(); in.normals = t[3].data_ptr<float>();
    in.viewdirs = t[4].data_ptr<float>(); in.incidents_shs = t[5].data_ptr<float>();
    in.direct_shs = t[6].data_ptr<float>(); in.visibility_shs = t[7].data_ptr<float>();
    return in;
}

std::vector<torch::Tensor> prep_brdf(std::initializer_list<torch::Tensor> ts, const torch::Device& dev) {
    std::vector<torch::Tensor> r;
    for (const auto& t : ts) {
        TORCH_CHECK(t.scalar_type() == torch::kFloat32, "render_equation: expected float32 inputs");
        r.push_back(t.to(dev).contiguous());
    }
    return r;
}

std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> render_equation_forward_impl(
    const std::vector<torch::Tensor>& t, int64_t sample_num, bool is_training, const torch::Tensor* rand_in) {
    const torch::Device dev = t[0].device();
    const int P = (int)t[0].size(0);
    auto fopt = t[0].options().dtype(torch::kFloat32);
    torch::Tensor pbr = torch::empty({P, 3}, fopt);
    torch::Tensor dirs = torch::empty({P, sample_num, 3}, fopt);
    torch::Tensor diffuse = torch::empty({P, 3}, fopt);
    // the reference always draws the per-(Gaussian, sample) rotation (render_equation.cu:708)
    torch::Tensor rnd = rand_in ? rand_in->to(dev).contiguous() : torch::rand({P, sample_num, 1}, fopt);
    r3dg_brdf_inputs in = brdf_inputs(t, (int)sample_num);
    check(r3dg_render_equation_forward(&in, is_training, rnd.numel() ? rnd.data_ptr<float>() : nullptr,
                                       pbr.data_ptr<float>(), dirs.data_ptr<float>(), diffuse.data_ptr<float>(),
                                       stream_of(dev)),
          "render_equation_forward");
    return {pbr, dirs, diffuse};
}

// RenderEquationForwardCUDA (render_equation.cu:688-726)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> render_equation_forward(
    const torch::Tensor& base_color, const torch::Tensor& roughness, const torch::Tensor& metallic,
    const torch::Tensor& normals, const torch::Tensor& viewdirs, const torch::Tensor& incidents_shs,
    const torch::Tensor& direct_shs, const torch::Tensor& visibility_shs, int64_t sample_num, bool is_training,
    bool debug) {
    (void)debug;
    const torch::Device dev = base_color.device();
    const c10::OptionalDeviceGuard guard(dev);
    auto t = prep_brdf({base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs},
                       dev);
    return render_equation_forward_impl(t, sample_num, is_training, nullptr);
}

// test entry: explicit rotation randoms [P, sample_num(, 1)]
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> render_equation_forward_with_rand(
    const torch::Tensor& base_color, const torch::Tensor& roughness, const torch::Tensor& metallic,
    const torch::Tensor& normals, const torch::Tensor& viewdirs, const torch::Tensor& incidents_shs,
    const torch::Tensor& direct_shs, const torch::Tensor& visibility_shs, int64_t sample_num, bool is_training,
    const torch::Tensor& rand_float) {
    const torch::Device dev = base_color.device();
    const c10::OptionalDeviceGuard guard(dev);
    auto t = prep_brdf({base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs},
                       dev);
    return render_equation_forward_impl(t, sample_num, is_training, &rand_float);
}

// RenderEquationForwardCUDA_complex (render_equation.cu:220-274)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
render_equation_forward_complex(const torch::Tensor& base_color, const torch::Tensor& roughness,
                                const torch::Tensor& metallic, const torch::Tensor& normals,
                                const torch::Tensor& viewdirs, const torch::Tensor& incidents_shs,
                                const torch::Tensor& direct_shs, const torch::Tensor& visibility_shs,
                                int64_t sample_num) {
    const torch::Device dev = base_color.device();
    const c10::OptionalDeviceGuard guard(dev);
    auto t = prep_brdf({base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs},
                       dev);
    const int P = (int)t[0].size(0);
    const int64_t Ns = sample_num;
    auto fopt = t[0].options().dtype(torch::kFloat32);
    torch::Tensor pbr = torch::empty({P, 3}, fopt), dirs = torch::empty({P, Ns, 3}, fopt);
    torch::Tensor lights = torch::empty({P, Ns, 3}, fopt), local = torch::empty({P, Ns, 3}, fopt);
    torch::Tensor global = torch::empty({P, Ns, 3}, fopt), vis = torch::empty({P, Ns, 1}, fopt);
    torch::Tensor diffuse = torch::empty({P, 3}, fopt), local_diffuse = torch::empty({P, 3}, fopt);
    torch::Tensor accum = torch::empty({P, 1}, fopt), rgb_d = torch::empty({P, 3}, fopt);
    torch::Tensor rgb_s = torch::empty({P, 3}, fopt);
    r3dg_brdf_inputs in = brdf_inputs(t, (int)sample_num);
    r3dg_brdf_complex_outputs o{pbr.data_ptr<float>(),     dirs.data_ptr<float>(),  lights.data_ptr<float>(),
                                local.data_ptr<float>(),   global.data_ptr<float>(), vis.data_ptr<float>(),
                                diffuse.data_ptr<float>(), local_diffuse.data_ptr<float>(),
                                accum.data_ptr<float>(),   rgb_d.data_ptr<float>(), rgb_s.data_ptr<float>()};
    check(r3dg_render_equation_forward_complex(&in, &o, stream_of(dev)), "render_equation_forward_complex");
    return {pbr, dirs, lights, local, global, vis, diffuse, local_diffuse, accum, rgb_d, rgb_s};
}

// RenderEquationBackwardCUDA (render_equation.cu:494-547)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor>
render_equation_backward(const torch::Tensor& base_color, const torch::Tensor& roughness,
                         const torch::Tensor& metallic, const torch::Tensor& normals, const torch::Tensor& viewdirs,
                         const torch::Tensor& incidents_shs, const torch::Tensor& direct_shs,
                         const torch::Tensor& visibility_shs, int64_t sample_num, const torch::Tensor& incident_dirs,
                         const torch::Tensor& dL_dpbr, const torch::Tensor& dL_ddiffuse_light, bool debug) {
    (void)debug;
    const torch::Device dev = base_color.device();
    const c10::OptionalDeviceGuard guard(dev);
    auto t = prep_brdf({base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs,
                        incident_dirs, dL_dpbr, dL_ddiffuse_light},
                       dev);
    r3dg_brdf_inputs in = brdf_inputs(t, (int)sample_num);
    const int P = in.P;
    auto fopt = t[0].options().dtype(torch::kFloat32);
    torch::Tensor d_base = torch::empty({P, 3}, fopt), d_rough = torch::empty({P, 1}, fopt);
    torch::Tensor d_metal = torch::empty({P, 1}, fopt), d_n = torch::empty({P, 3}, fopt);
    torch::Tensor d_v = torch::empty({P, 3}, fopt), d_inc = torch::empty({P, in.S_incident, 3}, fopt);
    torch::Tensor d_dir = torch::empty({1, in.S_direct, 3}, fopt), d_vis = torch::empty({P, in.S_visibility, 1}, fopt);
    r3dg_brdf_grads o{d_base.data_ptr<float>(), d_rough.data_ptr<float>(), d_metal.data_ptr<float>(),
                      d_n.data_ptr<float>(),    d_v.data_ptr<float>(),     d_inc.data_ptr<float>(),
                      d_dir.data_ptr<float>(),  d_vis.data_ptr<float>()};
    auto bopt = torch::TensorOptions().dtype(torch::kUInt8).device(dev);
    TensorAlloc scratch{bopt, torch::empty({0}, bopt)};
    check(r3dg_render_equation_backward(&in, t[8].data_ptr<float>(), t[9].data_ptr<float>(), t[10].data_ptr<float>(),
                                        tensor_alloc, &scratch, &o, stream_of(dev)),
          "render_equation_backward");
    return {d_base, d_rough, d_metal, d_n, d_v, d_inc, d_dir, d_vis};
}

std::map<std::string, int64_t> shader_map(int kind) {
    std::map<std::string, int64_t> m;
    for (int i = 0; i < r3dg_shader_count(kind); ++i) m[r3dg_shader_name(kind, i)] = r3dg_shader_handle(kind, i);
    return m;
}

std::tuple<int64_t, int64_t> preprocess_model(torch::Tensor& xyz) {
    const torch::Device dev = xyz.device();
    const c10::OptionalDeviceGuard guard(dev);
    auto x = dev_contig(xyz, dev);
    int64_t a = 0, b = 0;
    check(r3dg_preprocess_model((int)xyz.size(0), x.numel() ? x.data_ptr<float>() : nullptr, &a, &b, stream_of(dev)),
          "PreprocessModel");
    return {a, b};
}

int64_t create_shader_manager(int64_t kind, const torch::Tensor& handles) {
    auto h = handles.to(torch::kCPU).to(torch::kInt64).contiguous();
    int64_t m = 0;
    check(r3dg_create_shader_manager((int)kind, (int)h.numel(), h.data_ptr<int64_t>(), &m,
                                     stream_of(torch::Device(torch::kCUDA, c10::hip::current_device()))),
          "create_shader_manager");
    return m;
}

std::tuple<std::vector<int64_t>, std::vector<int64_t>> shader_manager_info(int64_t mgr) {
    int n = 0;
    check(r3dg_shader_manager_info(mgr, &n, nullptr, nullptr), "shader_manager_info");
    std::vector<int64_t> h(n);
    std::vector<int> c(n);
    check(r3dg_shader_manager_info(mgr, &n, h.data(), c.data()), "shader_manager_info");
    return {h, std::vector<int64_t>(c.begin(), c.end())};
}

// AllocateTexture (texture.cu:86-101): the dict textureImport.py builds -- pixelData [H, W, C]
// float, height, width, encoding_mode, wrap_modes [2], normalizedCoords (CPU int32 tensors)
int64_t allocate_texture(const std::map<std::string, torch::Tensor>& d) {
    auto scalar = [&](const char* k, int i = 0) {
        auto it = d.find(k);
        if (it == d.end()) throw std::runtime_error(std::string("AllocateTexture: missing '") + k + "'");
        return it->second.to(torch::kCPU).to(torch::kInt64).contiguous().data_ptr<int64_t>()[i];
    };
    auto it = d.find("pixelData");
    if (it == d.end()) throw std::runtime_error("AllocateTexture: missing 'pixelData'");
    torch::Tensor pix = it->second.to(torch::kFloat32).contiguous();
    if (!pix.is_cuda()) pix = pix.cuda();
    const int H = (int)scalar("height"), W = (int)scalar("width"), mode = (int)scalar("encoding_mode");
    const int C = pix.numel() / std::max<int64_t>((int64_t)H * W, 1);
    if ((int64_t)C * H * W != pix.numel()) throw std::runtime_error("AllocateTexture: pixelData is not [H, W, C]");
    c10::OptionalDeviceGuard guard(pix.device());
    int64_t h = 0;
    check(r3dg_texture_create(pix.data_ptr<float>(), W, H, mode, (int)scalar("wrap_modes", 0),
                              (int)scalar("wrap_modes", 1), (int)scalar("normalizedCoords"), &h,
                              c10::hip::getCurrentHIPStream(pix.device().index()).stream()),
          "AllocateTexture");
    return h;
}
// UploadTexturesToDevice (texture.cu:237-246)
int64_t upload_textures(const std::vector<std::string>& names, const std::vector<int64_t>& textures,
                        int64_t error_texture) {
    if (names.size() != textures.size()) throw std::runtime_error("UploadTexturesToDevice: names/textures mismatch");
    std::vector<const char*> cn;
    for (const auto& n : names) cn.push_back(n.c_str());
    int64_t h = 0;
    check(r3dg_texture_manager_create((int)names.size(), cn.data(), textures.data(), error_texture, &h),
          "UploadTexturesToDevice");
    return h;
}

// parity / debug accessor: views of the sorted keys, point list, tile ranges and per-Gaussian state
std::vector<torch::Tensor> rasterizer_state(const torch::Tensor& geomBuffer, const torch::Tensor& binningBuffer,
                                            const torch::Tensor& imageBuffer, int64_t P, int64_t H, int64_t W,
                                            int64_t L) {
    r3dg_binning_view v{};
    check(r3dg_state_view((int)P, (int)H, (int)W, (int)L, geomBuffer.data_ptr(), binningBuffer.data_ptr(),
                          imageBuffer.data_ptr(), &v),
          "rasterizer_state");
    auto slice = [](const torch::Tensor& buf, const void* p, int64_t nbytes) {
        const int64_t off = (const char*)p - (const char*)buf.data_ptr();
        return buf.narrow(0, off, nbytes);
    };
    const int64_t T = ((W + 15) / 16) * ((H + 15) / 16);
    // the reference's sort key, rebuilt: tile << 32 | float bits of the instance's depth
    auto plist = slice(binningBuffer, v.point_list, 4 * L).view(torch::kInt32);
    auto dbits = slice(geomBuffer, v.depths, 4 * P).view(torch::kInt32).to(torch::kInt64).bitwise_and(0xffffffffLL);
    auto rng = slice(imageBuffer, v.ranges, 8 * T).view(torch::kInt32).view({T, 2}).to(torch::kInt64);
    auto tiles = torch::repeat_interleave(torch::arange(T, rng.options()), rng.select(1, 1) - rng.select(1, 0), 0, L);
    auto keys = tiles.bitwise_left_shift(32).bitwise_or(dbits.index_select(0, plist.to(torch::kInt64)));
    return {keys,
            plist,
            slice(imageBuffer, v.ranges, 8 * T).view(torch::kInt32).view({T, 2}),
            slice(geomBuffer, v.point_offsets, 4 * P).view(torch::kInt32),
            slice(geomBuffer, v.depths, 4 * P).view(torch::kFloat32),
            slice(geomBuffer, v.means2D, 8 * P).view(torch::kFloat32).view({P, 2}),
            slice(geomBuffer, v.conic_opacity, 16 * P).view(torch::kFloat32).view({P, 4}),
            slice(geomBuffer, v.rgb, 12 * P).view(torch::kFloat32).view({P, 3}),
            slice(geomBuffer, v.cov3D, 24 * P).view(torch::kFloat32).view({P, 6}),
            slice(geomBuffer, v.clamped, P)};
}

std::vector<int64_t> feature_groups(int64_t S) {
    int g[64];
    const int n = r3dg_feature_groups((int)S, g);
    return std::vector<int64_t>(g, g + n);
}

// ---- training step (include/r3dg_hip.h "training step on the device") ----

r3dg_param_layout make_layout(int64_t P, const std::vector<int64_t>& widths, const std::vector<int64_t>& roles) {
    TORCH_CHECK(!widths.empty() && widths.size() <= R3DG_MAX_GROUPS, "param layout: 1..16 groups");
    TORCH_CHECK(roles.size() == 4, "param layout: roles = [xyz, scaling, rotation, opacity] group indices");
    r3dg_param_layout L{};
    L.P = (int)P;
    L.n_groups = (int)widths.size();
    for (size_t g = 0; g < widths.size(); ++g) L.width[g] = (int)widths[g];
    L.xyz = (int)roles[0]; L.scaling = (int)roles[1]; L.rotation = (int)roles[2]; L.opacity = (int)roles[3];
    return L;
}

float* f32_ptr(const torch::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), what,
                ": expected a contiguous float32 device tensor");
    return t.data_ptr<float>();
}

void adam_step(int64_t P, const std::vector<int64_t>& widths, const std::vector<int64_t>& roles, torch::Tensor param,
               const torch::Tensor& grad, torch::Tensor exp_avg, torch::Tensor exp_avg_sq, int64_t lo, int64_t hi,
               const std::vector<double>& lrs, double beta1, double beta2, double eps, int64_t step) {
    const r3dg_param_layout L = make_layout(P, widths, roles);
    TORCH_CHECK(lrs.size() == widths.size(), "adam_step: one learning rate per group");
    TORCH_CHECK(grad.numel() == hi - lo && exp_avg.numel() == hi - lo && exp_avg_sq.numel() == hi - lo,
                "adam_step: grad / exp_avg / exp_avg_sq must hold the shard's hi - lo floats");
    const c10::OptionalDeviceGuard guard(param.device());
    std::vector<float> lr(lrs.begin(), lrs.end());
    check(r3dg_adam_step(&L, f32_ptr(param, "param"), f32_ptr(grad, "grad"), f32_ptr(exp_avg, "exp_avg"),
                         f32_ptr(exp_avg_sq, "exp_avg_sq"), lo, hi, lr.data(), beta1, beta2, eps, (int)step,
                         stream_of(param.device())),
          "adam_step");
}

// adam_step with one step count per group; steps[g] <= 0: group g has no gradient (skipped)
void adam_step_groups(int64_t P, const std::vector<int64_t>& widths, const std::vector<int64_t>& roles,
                      torch::Tensor param, const torch::Tensor& grad, torch::Tensor exp_avg, torch::Tensor exp_avg_sq,
                      int64_t lo, int64_t hi, const std::vector<double>& lrs, double beta1, double beta2, double eps,
                      const std::vector<int64_t>& steps) {
    const r3dg_param_layout L = make_layout(P, widths, roles);
    TORCH_CHECK(lrs.size() == widths.size() && steps.size() == widths.size(),
                "adam_step_groups: one learning rate and one step count per group");
    TORCH_CHECK(grad.numel() == hi - lo && exp_avg.numel() == hi - lo && exp_avg_sq.numel() == hi - lo,
                "adam_step_groups: grad / exp_avg / exp_avg_sq must hold the shard's hi - lo floats");
    const c10::OptionalDeviceGuard guard(param.device());
    std::vector<float> lr(lrs.begin(), lrs.end());
    std::vector<int> st(steps.begin(), steps.end());
    check(r3dg_adam_step_groups(&L, f32_ptr(param, "param"), f32_ptr(grad, "grad"), f32_ptr(exp_avg, "exp_avg"),
                                f32_ptr(exp_avg_sq, "exp_avg_sq"), lo, hi, lr.data(), st.data(), beta1, beta2, eps,
                                stream_of(param.device())),
          "adam_step_groups");
}

void densification_stats(const torch::Tensor& dL_dmeans2D, const torch::Tensor& normal_grad, const torch::Tensor& radii,
                         torch::Tensor xyz_accum, torch::Tensor normal_accum, torch::Tensor denom,
                         torch::Tensor max_radii2D) {
    const int P = (int)radii.size(0);
    TORCH_CHECK(radii.scalar_type() == torch::kInt32, "densification_stats: radii must be int32");
    TORCH_CHECK(dL_dmeans2D.dim() == 2 && dL_dmeans2D.size(0) == P && dL_dmeans2D.size(1) >= 2,
                "densification_stats: dL_dmeans2D must be [P, >=2]");
    TORCH_CHECK(normal_grad.numel() == 0 || normal_grad.numel() == 3 * (int64_t)P,
                "densification_stats: normal_grad must be [P, 3] or empty");
    const c10::OptionalDeviceGuard guard(radii.device());
    check(r3dg_densification_stats(P, f32_ptr(dL_dmeans2D, "dL_dmeans2D"), (int)dL_dmeans2D.size(1),
                                   normal_grad.numel() ? f32_ptr(normal_grad, "normal_grad") : nullptr,
                                   radii.data_ptr<int>(), f32_ptr(xyz_accum, "xyz_accum"),
                                   f32_ptr(normal_accum, "normal_accum"), f32_ptr(denom, "denom"),
                                   f32_ptr(max_radii2D, "max_radii2D"), stream_of(radii.device())),
          "densification_stats");
}

struct MultiAlloc {
    torch::TensorOptions opts;
    std::vector<torch::Tensor> ts;
};
void* multi_alloc(void* ctx, size_t n) {
    auto* a = static_cast<MultiAlloc*>(ctx);
    a->ts.push_back(torch::empty({(int64_t)std::max<size_t>((n + 3) / 4, 64)}, a->opts));
    return a->ts.back().data_ptr();
}
// noise source of densify_and_split: torch.randn on the device (the reference's torch.normal)
void* randn_alloc(void* ctx, size_t n) {
    auto* a = static_cast<MultiAlloc*>(ctx);
    a->ts.push_back(torch::randn({(int64_t)n}, a->opts));
    return a->ts.back().data_ptr();
}

std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, int64_t, std::vector<int64_t>> densify_and_prune(
    int64_t P, const std::vector<int64_t>& widths, const std::vector<int64_t>& roles, const torch::Tensor& param,
    const torch::Tensor& exp_avg, const torch::Tensor& exp_avg_sq, const torch::Tensor& xyz_accum,
    const torch::Tensor& normal_accum, const torch::Tensor& denom, const torch::Tensor& max_radii2D,
    double grad_threshold, double grad_normal_threshold, double percent_dense, double extent, double min_opacity,
    double max_screen_size, int64_t N, bool prune_only, const torch::Tensor& noise) {
    const r3dg_param_layout L = make_layout(P, widths, roles);
    const c10::OptionalDeviceGuard guard(param.device());
    r3dg_densify_args d{};
    d.grad_threshold = (float)grad_threshold; d.grad_normal_threshold = (float)grad_normal_threshold;
    d.percent_dense = (float)percent_dense; d.extent = (float)extent; d.min_opacity = (float)min_opacity;
    d.max_screen_size = (float)max_screen_size; d.N = (int)N; d.prune_only = prune_only ? 1 : 0;
    MultiAlloc out{param.options(), {}}, rnd{param.options(), {}};
    // a given noise tensor (tests / replicated ranks) replaces the device generator
    auto given_noise = [](void* ctx, size_t n) -> void* {
        auto* t = static_cast<torch::Tensor*>(ctx);
        return (size_t)t->numel() >= n ? t->data_ptr() : nullptr;
    };
    torch::Tensor nz = noise;
    float *np = nullptr, *nm = nullptr, *nv = nullptr;
    int* src = nullptr;
    int Pn = 0, counts[4] = {0, 0, 0, 0};
    auto opt = [](const torch::Tensor& t, const char* w) { return t.numel() ? f32_ptr(t, w) : nullptr; };
    check(r3dg_densify_and_prune(&L, f32_ptr(param, "param"), f32_ptr(exp_avg, "exp_avg"),
                                 f32_ptr(exp_avg_sq, "exp_avg_sq"), opt(xyz_accum, "xyz_accum"),
                                 opt(normal_accum, "normal_accum"), opt(denom, "denom"),
                                 opt(max_radii2D, "max_radii2D"), &d, multi_alloc, &out,
                                 noise.numel() ? (r3dg_alloc_fn)given_noise : randn_alloc,
                                 noise.numel() ? (void*)&nz : (void*)&rnd, &np, &nm, &nv, &src, &Pn, counts,
                                 stream_of(param.device())),
          "densify_and_prune");
    auto find = [&](void* p) {
        for (auto& t : out.ts)
            if (t.data_ptr() == p) return t;
        TORCH_CHECK(false, "densify_and_prune: output not found");
        return torch::Tensor();
    };
    int64_t W = 0;
    for (auto w : widths) W += w;
    const int64_t n = (int64_t)Pn * W;
    torch::Tensor source = torch::from_blob(src, {(int64_t)Pn}, [](void*) {}, param.options().dtype(torch::kInt32));
    source = source.clone();  // own the map (the scratch allocation is released on return)
    return {find(np).narrow(0, 0, n), find(nm).narrow(0, 0, n), find(nv).narrow(0, 0, n), source, (int64_t)Pn,
            std::vector<int64_t>{counts[0], counts[1], counts[2], counts[3]}};
}

void reset_opacity(int64_t P, const std::vector<int64_t>& widths, const std::vector<int64_t>& roles,
                   torch::Tensor param, const torch::Tensor& exp_avg, const torch::Tensor& exp_avg_sq) {
    const r3dg_param_layout L = make_layout(P, widths, roles);
    const c10::OptionalDeviceGuard guard(param.device());
    check(r3dg_reset_opacity(&L, f32_ptr(param, "param"), exp_avg.numel() ? f32_ptr(exp_avg, "exp_avg") : nullptr,
                             exp_avg_sq.numel() ? f32_ptr(exp_avg_sq, "exp_avg_sq") : nullptr,
                             stream_of(param.device())),
          "reset_opacity");
}

// ---- BVH visibility tracer: the reference's bvh_tracing._C (bvh/src/bindings.cpp:9-11) ----------

torch::Tensor cuda_f32(const torch::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda(), what, ": expected a GPU tensor (this build has no CPU path)");
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, what, ": expected float32");
    return t.contiguous();
}

// RayTracer.__init__ leaf boxes (bvh/__init__.py:29-59) in one launch -> [P, 6]
torch::Tensor bvh_leaf_aabbs(const torch::Tensor& means3D, const torch::Tensor& scales,
                             const torch::Tensor& rotations) {
    const auto m = cuda_f32(means3D, "bvh_leaf_aabbs"), s = cuda_f32(scales, "bvh_leaf_aabbs"),
               r = cuda_f32(rotations, "bvh_leaf_aabbs");
    const int64_t P = m.size(0);
    TORCH_CHECK(m.numel() == 3 * P && s.numel() == 3 * P && r.numel() == 4 * P,
                "bvh_leaf_aabbs: means3D [P,3], scales [P,3], rotations [P,4] expected");
    const c10::OptionalDeviceGuard guard(m.device());
    auto out = torch::empty({P, 6}, m.options());
    check(r3dg_bvh_leaf_aabbs((int)P, m.data_ptr<float>(), s.data_ptr<float>(), r.data_ptr<float>(),
                              out.data_ptr<float>(), stream_of(m.device())),
          "bvh_leaf_aabbs");
    return out;
}

// create_bvh (bvh/src/bvh.cu:8-26): fills nodes / aabbs in place (their leaf boxes are the input)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> create_bvh(const torch::Tensor& means3D,
                                                                   const torch::Tensor& scales,
                                                                   const torch::Tensor& rotations,
                                                                   torch::Tensor nodes, torch::Tensor aabbs) {
    (void)scales;
    (void)rotations;  // the reference takes them and does not read them (construct.cu:148-155)
    const int64_t P = means3D.size(0);
    TORCH_CHECK(nodes.is_cuda() && aabbs.is_cuda(), "create_bvh: expected GPU tensors");
    TORCH_CHECK(nodes.scalar_type() == torch::kInt32 && aabbs.scalar_type() == torch::kFloat32,
                "create_bvh: nodes int32, aabbs float32 expected");
    TORCH_CHECK(nodes.is_contiguous() && aabbs.is_contiguous(), "create_bvh: nodes / aabbs must be contiguous");
    TORCH_CHECK(P >= 1 && nodes.numel() == 5 * (2 * P - 1) && aabbs.numel() == 6 * (2 * P - 1),
                "create_bvh: nodes [2P-1,5] and aabbs [2P-1,6] expected");
    const c10::OptionalDeviceGuard guard(aabbs.device());
    auto morton = torch::empty({P}, aabbs.options().dtype(torch::kInt64));
    TensorAlloc scratch{aabbs.options().dtype(torch::kUInt8), {}};
    check(r3dg_bvh_build((int)P, nodes.data_ptr<int32_t>(), aabbs.data_ptr<float>(),
                         reinterpret_cast<uint64_t*>(morton.data_ptr<int64_t>()), tensor_alloc, &scratch,
                         stream_of(aabbs.device())),
          "create_bvh");
    return {nodes, aabbs, morton};
}

// trace_bvh_opacity (bvh/src/bvh.cu:87-117): outputs shaped like rays_o without its last axis
std::tuple<torch::Tensor, torch::Tensor> trace_bvh_opacity(const torch::Tensor& nodes, const torch::Tensor& aabbs,
                                                           const torch::Tensor& rays_o, const torch::Tensor& rays_d,
                                                           const torch::Tensor& means3D, const torch::Tensor& covs3D,
                                                           const torch::Tensor& opacities,
                                                           const torch::Tensor& normals) {
    TORCH_CHECK(nodes.is_cuda() && nodes.scalar_type() == torch::kInt32, "trace_bvh_opacity: nodes int32 on GPU");
    const auto o = cuda_f32(rays_o, "rays_o"), d = cuda_f32(rays_d, "rays_d");
    TORCH_CHECK(o.dim() >= 1 && o.size(-1) == 3 && d.numel() == o.numel(), "trace_bvh_opacity: rays [..., 3]");
    const int64_t R = o.numel() / 3;
    const c10::OptionalDeviceGuard guard(o.device());
    auto shape = o.sizes().slice(0, o.dim() - 1);
    auto contrib = torch::zeros(shape, o.options().dtype(torch::kInt32));
    auto vis = torch::ones(shape, o.options());
    const auto nd = nodes.contiguous(), bx = cuda_f32(aabbs, "aabbs"), m = cuda_f32(means3D, "means3D"),
               c = cuda_f32(covs3D, "covs3D"), op = cuda_f32(opacities, "opacities"), n = cuda_f32(normals, "normals");
    const int64_t P = m.numel() / 3;
    TORCH_CHECK(P >= 1 && nd.numel() == 5 * (2 * P - 1) && bx.numel() == 6 * (2 * P - 1) && c.numel() == 6 * P &&
                    op.numel() == P && n.numel() == 3 * P,
                "trace_bvh_opacity: tree / Gaussian shapes disagree");
    TensorAlloc scratch{o.options().dtype(torch::kUInt8), {}};
    check(r3dg_bvh_trace_opacity((int)R, (int)P, nd.data_ptr<int32_t>(), bx.data_ptr<float>(), o.data_ptr<float>(),
                                 d.data_ptr<float>(), m.data_ptr<float>(), c.data_ptr<float>(), op.data_ptr<float>(),
                                 n.data_ptr<float>(), contrib.data_ptr<int32_t>(), vis.data_ptr<float>(),
                                 tensor_alloc, &scratch, stream_of(o.device())),
          "trace_bvh_opacity");
    return {contrib, vis};
}

struct MultiAllocBvh {
    torch::TensorOptions opts;
    std::vector<torch::Tensor> ts;
};
void* multi_alloc_bvh(void* ctx, size_t n) {
    auto* a = static_cast<MultiAllocBvh*>(ctx);
    a->ts.push_back(torch::empty({(int64_t)std::max<size_t>(n, 256)}, a->opts));
    return a->ts.back().data_ptr();
}

// trace_bvh (bvh/src/bvh.cu:28-85)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor> trace_bvh(
    const torch::Tensor& nodes, const torch::Tensor& aabbs, const torch::Tensor& rays_o, const torch::Tensor& rays_d,
    const torch::Tensor& means3D, const torch::Tensor& covs3D, const torch::Tensor& opacities) {
    (void)covs3D;
    (void)opacities;  // unused by the reference's arithmetic (trace.cu:123-124 commented out)
    TORCH_CHECK(nodes.is_cuda() && nodes.scalar_type() == torch::kInt32, "trace_bvh: nodes int32 on GPU");
    const auto o = cuda_f32(rays_o, "rays_o"), d = cuda_f32(rays_d, "rays_d");
    const int64_t R = o.size(0);
    TORCH_CHECK(o.numel() == 3 * R && d.numel() == 3 * R, "trace_bvh: rays [R, 3]");
    const c10::OptionalDeviceGuard guard(o.device());
    const auto iopt = o.options().dtype(torch::kInt32);
    auto contrib = torch::zeros({R, 1}, iopt);
    const auto nd = nodes.contiguous(), bx = cuda_f32(aabbs, "aabbs"), m = cuda_f32(means3D, "means3D");
    const int64_t P = m.numel() / 3;
    TORCH_CHECK(P >= 1 && nd.numel() == 5 * (2 * P - 1) && bx.numel() == 6 * (2 * P - 1),
                "trace_bvh: tree shapes disagree");
    MultiAllocBvh al{o.options().dtype(torch::kUInt8), {}};
    int L = 0;
    int32_t *pt = nullptr, *rid = nullptr;
    float* pos = nullptr;
    check(r3dg_bvh_trace((int)R, (int)P, nd.data_ptr<int32_t>(), bx.data_ptr<float>(), o.data_ptr<float>(), d.data_ptr<float>(),
                         m.data_ptr<float>(), contrib.data_ptr<int32_t>(), multi_alloc_bvh, &al, &L, &pt, &pos, &rid,
                         stream_of(o.device())),
          "trace_bvh");
    if (L == 0)  // the reference's empty shapes (bvh.cu:48-53), ray_id_list float [0, 3] included
        return {contrib, torch::zeros({0, 1}, iopt), torch::zeros({0, 3}, o.options()), torch::zeros({0, 3}, o.options())};
    auto view = [&](void* p, std::vector<int64_t> shape, torch::ScalarType t) {
        for (auto& b : al.ts)
            if (b.data_ptr() == p) return b.narrow(0, 0, L * (t == torch::kFloat32 ? 12 : 4)).view(t).view(shape);
        TORCH_CHECK(false, "trace_bvh: output not found");
        return torch::Tensor();
    };
    return {contrib, view(pt, {L, 1}, torch::kInt32), view(pos, {L, 3}, torch::kFloat32),
            view(rid, {L, 1}, torch::kInt32)};
}

}  // namespace


// r3dg_get_options / r3dg_set_options (include/r3dg_hip.h) as a dict of the option fields
#define R3DG_OPTION_FIELDS(X)                                                                         \
    X(bwd_reduce) X(prof_sort_markers) X(test_bwd_dpp) X(test_bwd_wterms) X(test_no_cull)              \
    X(test_bin_atomic) X(test_bin_blocks) X(test_tile_order_spatial) X(test_bwd_srs) X(test_bvh_lanes) \
    X(test_bvh_sort) X(test_bvh_split) X(test_bin_one_pass)
std::map<std::string, int64_t> get_options() {
    r3dg_options o{};
    o.struct_size = sizeof(o);
    check(r3dg_get_options(&o), "get_options");
    std::map<std::string, int64_t> d;
#define X(f) d[#f] = o.f;
    R3DG_OPTION_FIELDS(X)
#undef X
    return d;
}
// sets the given fields (the others keep their values); returns the previous options
std::map<std::string, int64_t> set_options(const std::map<std::string, int64_t>& kv) {
    r3dg_options o{};
    o.struct_size = sizeof(o);
    check(r3dg_get_options(&o), "set_options");
    const std::map<std::string, int64_t> prev = get_options();
    for (const auto& it : kv) {
        bool known = false;
#define X(f) if (it.first == #f) { o.f = (int)it.second; known = true; }
        R3DG_OPTION_FIELDS(X)
#undef X
        TORCH_CHECK(known, "set_options: unknown option ", it.first);
    }
    check(r3dg_set_options(&o), "set_options");
    return prev;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "MI355X-native relightable Gaussian-splat rasterizer (drop-in for r3dg_rasterization._C)";
    // the reference surface (ext.cu:21-35)
    m.def("rasterize_gaussians", &rasterize_gaussians);
    m.def("rasterize_gaussians_backward", &rasterize_gaussians_backward);
    m.def("render_equation_forward", &render_equation_forward);
    m.def("render_equation_forward_complex", &render_equation_forward_complex);
    m.def("render_equation_backward", &render_equation_backward);
    m.def("mark_visible", &mark_visible);
    m.def("GetSplatShaderAddressMap", []() { return shader_map(R3DG_SHADER_SPLAT); });
    m.def("GetShShaderAddressMap", []() { return shader_map(R3DG_SHADER_SH); });
    m.def("GetPostProcessShaderAddressMap", []() { return shader_map(R3DG_SHADER_POST); });
    m.def("PreprocessModel", &preprocess_model);
    m.def("EncodeTextureMode", [](const std::string& s) { return r3dg_encode_texture_mode(s.c_str()); });
    m.def("EncodeWrapMode", [](const std::string& s) { return r3dg_encode_wrap_mode(s.c_str()); });
    m.def("AllocateTexture", &allocate_texture);
    m.def("UploadTexturesToDevice", &upload_textures);
    // extensions
    m.def("rasterize_gaussians_backward_ex", &rasterize_gaussians_backward_ex);
    m.def("rasterize_gaussians_backward_chunked", &rasterize_gaussians_backward_chunked);
    m.def("rasterize_gaussians_backward_chunked_packed", &rasterize_gaussians_backward_chunked_packed);
    m.def("render_equation_forward_with_rand", &render_equation_forward_with_rand);
    m.def("rasterizer_state", &rasterizer_state);
    m.def("sh_color_grads", &sh_color_grads);
    m.def("sh_grad_from_views", &sh_grad_from_views);
    m.def("feature_groups", &feature_groups);
    m.def("create_shader_manager", &create_shader_manager);
    m.def("shader_manager_info", &shader_manager_info);
    m.def("abi_version", []() { return r3dg_abi_version(); });
    m.def("get_options", &get_options);
    m.def("set_options", &set_options);
    // training step on the device (§8f rank 3)
    m.def("adam_step", &adam_step);
    m.def("adam_step_groups", &adam_step_groups);
    m.def("densification_stats", &densification_stats);
    m.def("densify_and_prune", &densify_and_prune);
    m.def("reset_opacity", &reset_opacity);
    // BVH visibility tracer (§8f rank 4): the reference's bvh_tracing._C names + the leaf boxes
    m.def("create_bvh", &create_bvh);
    m.def("trace_bvh", &trace_bvh);
    m.def("trace_bvh_opacity", &trace_bvh_opacity);
    m.def("bvh_leaf_aabbs", &bvh_leaf_aabbs);
    m.def("profile_enable", [](int64_t n) { check(r3dg_profile_enable((int)n), "profile_enable"); });
    m.def("profile_read", [](int64_t kernel) {
        int c = 0;
        float ms = 0.f;
        check(r3dg_profile_read((int)kernel, &c, &ms), "profile_read");
        return std::make_tuple((int64_t)c, (double)ms);
    });
}
