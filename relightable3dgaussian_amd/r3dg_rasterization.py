"""Autograd wrapper: drop-in for gaussian_renderer/r3dg_rasterization.py of the reference.

Same public names and signatures (GaussianRasterizationSettings, GaussianRasterizer,
rasterize_gaussians, RenderEquation, RenderEquation_complex) over the HIP `_C`. Fixes the
reference wrapper's defects that break training:
  * backward takes all 11 output gradients (reference: 10, r3dg_rasterization.py:133-134);
  * `None` texture / shader-manager handles and post-pass list mean "defaults"
    (reference: pybind cannot convert None, rasterize_points.cu:67-70);
  * the forward's HWC colour and native feature layout are handed to the backward as they are
    (rasterize_gaussians_backward_ex) instead of being read as CHW (rasterize_points.cu:214-215).
Gradients of the stencil, shader colour, pseudo normal and surface xyz outputs are ignored, as
in the reference.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C


def cpu_deep_copy_tuple(input_tuple):
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def rasterize_gaussians(means3D, means2D, features, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, features, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _none_if_empty(t):
    return None if (t is None or t.numel() == 0) else t


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, features, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        args = (s.bg, s.time, s.dt, means3D, features, colors_precomp, opacities, scales, rotations,
                s.scale_modifier, cov3Ds_precomp, s.viewmatrix, s.viewmatrix_inv, s.projmatrix, s.projmatrix_inv,
                s.tanfovx, s.tanfovy, s.cx, s.cy, s.image_height, s.image_width, sh, s.sh_degree, s.campos,
                s.prefiltered, s.computer_pseudo_normal, s.d_textureManager_ptr or 0, s.h_shShaderManager_ptr or 0,
                s.h_splatShaderManager_ptr or 0, list(s.postProcessingPasses or []), s.debug)
        if s.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args)
        (num_rendered, num_contrib, color, opacity, depth, stencil, feature, shader_color, normal, surface_xyz, radii,
         geomBuffer, binningBuffer, imgBuffer) = out
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, features, scales, rotations, cov3Ds_precomp, radii, sh,
                              geomBuffer, binningBuffer, imgBuffer)
        ctx.mark_non_differentiable(num_contrib, radii)
        return num_rendered, num_contrib, color, opacity, depth, stencil, feature, shader_color, normal, surface_xyz, \
            radii

    @staticmethod
    def backward(ctx, grad_num_rendered, grad_num_contrib, grad_out_color, grad_out_opacity, grad_out_depth,
                 grad_out_stencil, grad_out_feature, grad_out_shader, grad_out_normal, grad_out_surface_xyz,
                 grad_out_radii):
        s = ctx.raster_settings
        (colors_precomp, means3D, features, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        H, W = s.image_height, s.image_width
        S = features.shape[1] if features.dim() == 2 else 0
        z = lambda g, shape: g if g is not None else torch.zeros(shape, device=means3D.device)  # noqa: E731
        args = (s.bg, means3D, features, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp,
                s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, z(grad_out_color, (H, W, 3)),
                z(grad_out_opacity, (H, W, 1)), z(grad_out_depth, (H, W, 1)), z(grad_out_feature, (H, W, S)), sh,
                s.sh_degree, s.campos, geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, s.backward_geometry,
                s.debug, H, W)
        if s.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                grads = _C.rasterize_gaussians_backward_ex(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            grads = _C.rasterize_gaussians_backward_ex(*args)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_features, grad_cov3Ds_precomp, grad_sh,
         grad_scales, grad_rotations) = grads
        return (grad_means3D, grad_means2D, grad_features if features.numel() else None,
                grad_sh if _none_if_empty(sh) is not None else None,
                grad_colors_precomp if _none_if_empty(colors_precomp) is not None else None, grad_opacities,
                grad_scales if _none_if_empty(scales) is not None else None,
                grad_rotations if _none_if_empty(rotations) is not None else None,
                grad_cov3Ds_precomp if _none_if_empty(cov3Ds_precomp) is not None else None, None)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    cx: float
    cy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    viewmatrix_inv: torch.Tensor
    projmatrix: torch.Tensor
    projmatrix_inv: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    backward_geometry: bool
    computer_pseudo_normal: bool
    debug: bool
    h_shShaderManager_ptr: int
    h_splatShaderManager_ptr: int
    time: float
    dt: float
    d_textureManager_ptr: int
    postProcessingPasses: list


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            visible = _C.mark_visible(positions, s.viewmatrix, s.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, features=None):
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = lambda: torch.empty(0, device=means3D.device)  # noqa: E731
        shs = empty() if shs is None else shs
        colors_precomp = empty() if colors_precomp is None else colors_precomp
        scales = empty() if scales is None else scales
        rotations = empty() if rotations is None else rotations
        cov3D_precomp = empty() if cov3D_precomp is None else cov3D_precomp
        if features is None:
            features = torch.empty_like(means3D[..., :0])
        return rasterize_gaussians(means3D, means2D, features, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, s)


class _RenderEquation(torch.autograd.Function):
    @staticmethod
    def forward(ctx, base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs,
                sample_num, is_training, debug=False):
        pbr, incident_dirs, diffuse_light = _C.render_equation_forward(base_color, roughness, metallic, normals,
                                                                       viewdirs, incidents_shs, direct_shs,
                                                                       visibility_shs, sample_num, is_training, debug)
        ctx.sample_num = sample_num
        ctx.debug = debug
        ctx.save_for_backward(base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs,
                              visibility_shs, incident_dirs)
        return pbr, incident_dirs, diffuse_light

    @staticmethod
    def backward(ctx, grad_pbr, grad_incident_dirs, grad_diffuse_light):
        (base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs,
         incident_dirs) = ctx.saved_tensors
        if grad_pbr is None:
            grad_pbr = torch.zeros_like(base_color)
        if grad_diffuse_light is None:
            grad_diffuse_light = torch.zeros_like(base_color)
        grads = _C.render_equation_backward(base_color, roughness, metallic, normals, viewdirs, incidents_shs,
                                            direct_shs, visibility_shs, ctx.sample_num, incident_dirs, grad_pbr,
                                            grad_diffuse_light, ctx.debug)
        return (*grads, None, None, None)


def RenderEquation_complex(base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs,
                           visibility_shs, sample_num):
    return _C.render_equation_forward_complex(base_color, roughness, metallic, normals, viewdirs, incidents_shs,
                                              direct_shs, visibility_shs, sample_num)


def RenderEquation(base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs, visibility_shs,
                   sample_num, is_training, debug=False):
    return _RenderEquation.apply(base_color, roughness, metallic, normals, viewdirs, incidents_shs, direct_shs,
                                 visibility_shs, sample_num, is_training, debug)


def settings_from_camera(cam, bg, sh_degree=3, scale_modifier=1.0, device="cuda", debug=False,
                         computer_pseudo_normal=True, backward_geometry=True) -> GaussianRasterizationSettings:
    """Build settings from relightable3dgaussian_amd.synthetic.Camera (the neilf.py:36-61 recipe)."""
    t = lambda a: torch.as_tensor(a, dtype=torch.float32, device=device)  # noqa: E731
    return GaussianRasterizationSettings(
        image_height=cam.height, image_width=cam.width, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, cx=cam.cx,
        cy=cam.cy, bg=t(bg), scale_modifier=scale_modifier, viewmatrix=t(cam.view), viewmatrix_inv=t(cam.view_inv),
        projmatrix=t(cam.proj), projmatrix_inv=t(cam.proj_inv), sh_degree=sh_degree, campos=t(cam.campos),
        prefiltered=False, backward_geometry=backward_geometry, computer_pseudo_normal=computer_pseudo_normal,
        debug=debug, h_shShaderManager_ptr=0, h_splatShaderManager_ptr=0, time=0.0, dt=0.0, d_textureManager_ptr=0,
        postProcessingPasses=[])
