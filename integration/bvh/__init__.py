"""Drop-in replacement for the reference's `bvh` package (bvh/__init__.py: `RayTracer`).

With `integration/` on PYTHONPATH these reference imports resolve to the MI355X build unchanged:
    scene/gaussian_model.py:16        from bvh import RayTracer
    gaussian_renderer/neilf.py:6      from bvh import RayTracer
    relighting.py:15                  from bvh import RayTracer
"""
from relightable3dgaussian_amd.bvh import RayTracer  # noqa: F401  (ImportError if the HIP build is missing)
