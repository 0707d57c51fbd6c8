"""Drop-in replacement for the reference's installed `r3dg_rasterization` package
(r3dg-rasterization/setup.py: packages=['r3dg_rasterization'], ext 'r3dg_rasterization._C').

Put `integration/` (this directory's parent) on PYTHONPATH ahead of any CUDA build and the
reference's imports resolve to the MI355X build unchanged:
    scene/gaussian_model.py:18            from r3dg_rasterization import _C
    asset_processing/PostProcess.py:1     from r3dg_rasterization import _C
    gaussian_renderer/r3dg_rasterization.py:8   from r3dg_rasterization import _C
"""
import sys

from relightable3dgaussian_amd import _C  # noqa: F401  (raises ImportError if the HIP build is missing)
from relightable3dgaussian_amd.r3dg_rasterization import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer, RenderEquation, RenderEquation_complex, _RasterizeGaussians,
    _RenderEquation, cpu_deep_copy_tuple, rasterize_gaussians)

sys.modules.setdefault("r3dg_rasterization._C", _C)
