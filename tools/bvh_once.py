"""One BVH build + one opacity trace of 1M rays (for rocprofv3 --pmc passes, tools/pmc_bvh.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    from bench_bvh import surface_scene
    from relightable3dgaussian_amd.bvh import RayTracer
    from tests.test_bvh import rays_from, scene

    which = sys.argv[1] if len(sys.argv) > 1 else "volume"
    sc = scene(1_000_000, seed=8, spread=1.0) if which == "volume" else surface_scene(1_000_000, seed=8)
    dev = lambda a: torch.as_tensor(a, device="cuda")  # noqa: E731
    means = dev(sc["means"])
    rt = RayTracer(means, dev(sc["scales"]), dev(sc["rots"]))
    o, d = rays_from(sc, 1_000_000, seed=2)
    res = rt.trace_visibility(dev(o), dev(d), means, dev(sc["cov_inv"]), dev(sc["opacity"]), dev(sc["normals"]))
    torch.cuda.synchronize()
    print(which, float(res["visibility"].mean()))


if __name__ == "__main__":
    main()
