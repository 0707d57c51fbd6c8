"""Drop-in replacement for the reference's compiled `bvh_tracing` package (bvh/setup.py,
ext `bvh_tracing._C`: create_bvh / trace_bvh / trace_bvh_opacity, bvh/src/bindings.cpp:9-11)."""
import sys

from relightable3dgaussian_amd import _C  # noqa: F401  (raises ImportError if the HIP build is missing)

sys.modules.setdefault("bvh_tracing._C", _C)
