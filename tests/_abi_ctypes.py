"""ctypes mirror of include/r3dg_hip.h's rasterizer structs -- the binding INTEGRATION.md §2 shows a
non-Python host (or a Python host without the torch extension) would write. Every struct that
carries `struct_size` is filled through `new()`, which sets it; the library refuses any other value,
so a layout drift between this file and the header fails the call instead of reading garbage."""
from __future__ import annotations

import ctypes as C

ALLOC = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)
CHUNK_DONE = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int)
FP = C.POINTER(C.c_float)
vp = C.c_void_p


class RasterSettings(C.Structure):  # r3dg_raster_settings (rasterize_points.cu:39-71 arguments)
    _fields_ = [("struct_size", C.c_size_t), ("P", C.c_int), ("S", C.c_int), ("D", C.c_int), ("M", C.c_int),
                ("W", C.c_int), ("H", C.c_int), ("tan_fovx", C.c_float), ("tan_fovy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("scale_modifier", C.c_float), ("time", C.c_float),
                ("dt", C.c_float), ("prefiltered", C.c_int), ("compute_pseudo_normal", C.c_int),
                ("debug", C.c_int), ("bg", vp), ("viewmatrix", vp), ("viewmatrix_inv", vp), ("projmatrix", vp),
                ("projmatrix_inv", vp), ("campos", vp), ("sh_shader_manager", C.c_int64),
                ("splat_shader_manager", C.c_int64), ("texture_manager", C.c_int64), ("post_passes", vp),
                ("n_post_passes", C.c_int)]


class Gaussians(C.Structure):  # r3dg_gaussians
    _fields_ = [(n, vp) for n in ("means3D", "features", "colors_precomp", "opacity", "scales", "rotations",
                                  "cov3D_precomp", "sh")]


class ForwardOutputs(C.Structure):  # r3dg_forward_outputs
    _fields_ = [(n, vp) for n in ("color", "opacity", "depth", "stencil", "feature", "shader_color", "normal",
                                  "surface_xyz", "radii")]


class BackwardGrads(C.Structure):  # r3dg_backward_grads
    _fields_ = [("dL_dout_color", vp), ("color_hwc", C.c_int), ("dL_dout_opacity", vp), ("dL_dout_depth", vp),
                ("dL_dout_feature", vp), ("feature_native", C.c_int)]


class BackwardOutputs(C.Structure):  # r3dg_backward_outputs
    _fields_ = [("struct_size", C.c_size_t)] + [
        (n, vp) for n in ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dfeatures", "dL_dcov3D",
                          "dL_dsh", "dL_dscales", "dL_drotations")] + [
        ("n_chunks", C.c_int), ("chunk_done", CHUNK_DONE), ("chunk_ctx", vp), ("dense_stride", C.c_int)]


OPTION_FIELDS = ("bwd_reduce", "prof_sort_markers", "test_bwd_dpp", "test_bwd_wterms", "test_no_cull",
                 "test_bin_atomic", "test_bin_blocks", "test_tile_order_spatial", "test_bwd_srs", "test_bvh_lanes",
                 "test_bvh_sort", "test_bvh_split", "test_bin_one_pass")


class Options(C.Structure):  # r3dg_options
    _fields_ = [("struct_size", C.c_size_t)] + [(n, C.c_int) for n in OPTION_FIELDS]


def new(cls, **kw):
    """An instance with every field zero and struct_size set (if the struct has one)."""
    o = cls()
    if any(f[0] == "struct_size" for f in cls._fields_):
        o.struct_size = C.sizeof(cls)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def bind(lib):
    """Argument / return types of the entry points the tests call."""
    lib.r3dg_last_error.restype = C.c_char_p
    P = C.POINTER
    lib.r3dg_get_options.argtypes = [P(Options)]
    lib.r3dg_set_options.argtypes = [P(Options)]
    lib.r3dg_rasterize_gaussians_ex.argtypes = [P(RasterSettings), P(Gaussians), P(ForwardOutputs), ALLOC, vp,
                                                ALLOC, vp, ALLOC, vp, ALLOC, vp, P(C.c_int), vp]
    lib.r3dg_rasterize_gaussians_backward.argtypes = [P(RasterSettings), P(Gaussians), vp, P(BackwardGrads), vp, vp,
                                                      vp, C.c_int, C.c_int, ALLOC, vp, P(BackwardOutputs), vp]
    lib.r3dg_image_state_n_contrib_offset.restype = C.c_size_t
    lib.r3dg_image_state_n_contrib_offset.argtypes = [C.c_int, C.c_int]
    return lib
