"""Generate golden vectors from the REFERENCE's own PyTorch code (run in the CPU container).

The reference (Krapylet/Relightable3DGaussian, mounted read-only at /root/reference) ships no
tests or golden images, and its CUDA extension cannot be built here (no nvcc / GPU). Its
pure-PyTorch pieces are importable on CPU, so this script runs them on seeded inputs and
stores inputs + outputs as small .npz fixtures (data only, no reference source is copied):

  brdf.npz     rendering_equation_python (gaussian_renderer/neilf.py:437-519) forward outputs
               and autograd gradients of sum(pbr) + sum(diffuse_light)
  brdf_pi5.npz the same with the reference Python's np.pi replaced by the CUDA kernels' literal
               3.14159f (render_equation.cu:89,145,149,...): the Python path and the CUDA path
               differ only in that constant, which the sharp SG lobe amplifies (~2e-4 abs on pbr)
  sh.npz       eval_sh (utils/sh_utils.py) + 0.5, clamped -> computeColorFromSH      (§8c (3))
  cov3d.npz    build_scaling_rotation + strip_symmetric (utils/general_utils.py,
               scene/gaussian_model.py:24-28)                                       (§8c (4))
  camera.npz   getWorld2View2 / getProjectionMatrix (utils/graphics_utils.py) as consumed by
               scene/cameras.py:63-79 (transposed, full_proj = view @ proj)          (§8c (5))
  fib.npz      fibonacci_sphere_sampling(random_rotate=False) directions             (§8c (6))

How the reference is imported: `bvh`, `arguments`, `scene.*` and
`gaussian_renderer.r3dg_rasterization` are replaced by empty stub modules (they only matter for
CUDA paths), and a TorchFunctionMode rewrites device='cuda' to 'cpu' for the reference's
hard-coded allocations (utils/graphics_utils.py:16,21, utils/sh_utils.py:56,67).

Usage:  python tests/golden/make_golden.py  [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

HERE = os.path.dirname(os.path.abspath(__file__))


class CpuMode(TorchFunctionMode):
    """Rewrite device='cuda' keyword arguments (and .cuda()) to CPU."""

    def __torch_function__(self, func, types_, args=(), kwargs=None):
        kwargs = dict(kwargs or {})
        dev = kwargs.get("device")
        if dev is not None and "cuda" in str(dev):
            kwargs["device"] = "cpu"
        if getattr(func, "__name__", "") == "cuda":
            return args[0]
        return func(*args, **kwargs)


def load_reference(ref: str):
    sys.path.insert(0, ref)
    for name in ["bvh", "arguments", "scene", "scene.gaussian_model", "scene.cameras"]:
        m = types.ModuleType(name)
        m.RayTracer = object
        m.OptimizationParams = object
        m.GaussianModel = object
        m.Camera = object
        sys.modules[name] = m
    pkg = types.ModuleType("gaussian_renderer")
    pkg.__path__ = [os.path.join(ref, "gaussian_renderer")]
    sys.modules["gaussian_renderer"] = pkg
    stub = types.ModuleType("gaussian_renderer.r3dg_rasterization")
    for n in ["GaussianRasterizationSettings", "GaussianRasterizer", "RenderEquation", "RenderEquation_complex"]:
        setattr(stub, n, None)
    sys.modules["gaussian_renderer.r3dg_rasterization"] = stub
    spec = importlib.util.spec_from_file_location("gaussian_renderer.neilf",
                                                  os.path.join(ref, "gaussian_renderer", "neilf.py"))
    neilf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(neilf)
    import utils.general_utils as gu  # noqa: E402
    import utils.graphics_utils as gr  # noqa: E402
    import utils.sh_utils as sh  # noqa: E402
    return neilf, sh, gr, gu


class EnvLight:
    def __init__(self, shs):
        self.get_env_shs = shs


def brdf_inputs(P: int, seed: int, positive_local: bool):
    rng = np.random.default_rng(seed)
    base = rng.uniform(0, 1, (P, 3))
    rough = rng.uniform(0.05, 1, (P, 1))
    metal = rng.uniform(0, 1, (P, 1))
    n = rng.normal(size=(P, 3)); n /= np.linalg.norm(n, axis=1, keepdims=True)
    v = rng.normal(size=(P, 3)); v /= np.linalg.norm(v, axis=1, keepdims=True)
    inc = rng.normal(0, 0.1, (P, 16, 3))
    vis = rng.normal(0, 0.1, (P, 16, 1))
    env = rng.normal(0, 0.1, (1, 16, 3))
    if positive_local:  # keep every clamp inactive so autograd == the CUDA kernel's formulas
        inc[:, 0, :] = 2.0 + rng.uniform(0, 1, (P, 3))
        inc[:, 1:, :] *= 0.3
        vis *= 0.3
        env *= 0.3
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    return dict(base=f(base), rough=f(rough), metal=f(metal), normals=f(n), viewdirs=f(v),
                incidents=f(inc), visibility=f(vis), env=f(env))


class NumpyPi5(types.ModuleType):
    """numpy with pi = 3.14159 (the literal of the reference's CUDA render equation)."""

    def __init__(self):
        super().__init__("numpy_pi5")
        self.pi = float(np.float32(3.14159))

    def __getattr__(self, name):
        return getattr(np, name)


def brdf_fixture(neilf, P: int, Ns: int) -> dict:
    inp = brdf_inputs(P, 0, positive_local=False)
    t = {k: torch.from_numpy(v) for k, v in inp.items()}
    pbr, extra = neilf.rendering_equation_python(t["base"], t["rough"], t["metal"], t["normals"], t["viewdirs"],
                                                 t["incidents"], False, EnvLight(t["env"]), t["visibility"],
                                                 sample_num=Ns)
    out = {k: v for k, v in inp.items()}
    out.update(pbr=pbr.numpy(), diffuse_light=extra["diffuse_light"].numpy(),
               incident_dirs=extra["incident_dirs"].numpy(),
               incident_lights=extra["incident_lights"].numpy(),
               local_incident_lights=extra["local_incident_lights"].numpy(),
               global_incident_lights=extra["global_incident_lights"].numpy(),
               incident_visibility=extra["incident_visibility"].numpy(), sample_num=np.int32(Ns))
    ginp = brdf_inputs(P, 1, positive_local=True)
    gt = {k: torch.from_numpy(v).clone().requires_grad_(True) for k, v in ginp.items()}
    gpbr, gextra = neilf.rendering_equation_python(gt["base"], gt["rough"], gt["metal"], gt["normals"],
                                                   gt["viewdirs"], gt["incidents"], False, EnvLight(gt["env"]),
                                                   gt["visibility"], sample_num=Ns)
    (gpbr.sum() + gextra["diffuse_light"].sum()).backward()
    for k, v in ginp.items():
        out["g_" + k] = v
    for k in ["base", "rough", "metal", "incidents", "visibility", "env"]:
        out["grad_" + k] = gt[k].grad.numpy()
    out["g_pbr"] = gpbr.detach().numpy()
    out["g_diffuse_light"] = gextra["diffuse_light"].detach().numpy()
    out["g_incident_dirs"] = gextra["incident_dirs"].detach().numpy()
    out["g_local_min"] = np.float32(gextra["local_incident_lights"].min().item())
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    torch.set_num_threads(4)
    with CpuMode():
        neilf, shu, gr, gu = load_reference(args.reference)

        # ---- (1)+(2) BRDF forward outputs and gradients (no clamp active in the gradient case) ----
        P, Ns = 256, 24
        np.savez_compressed(os.path.join(HERE, "brdf.npz"), **brdf_fixture(neilf, P, Ns))
        shim = NumpyPi5()
        neilf.np, gr.np = shim, shim
        np.savez_compressed(os.path.join(HERE, "brdf_pi5.npz"), **brdf_fixture(neilf, P, Ns))
        neilf.np, gr.np = np, np

        # ---- (3) SH colour (CUDA direction convention: pos - campos) ----
        rng = np.random.default_rng(3)
        Pn = 512
        means = rng.uniform(-2, 2, (Pn, 3)).astype(np.float32)
        campos = np.array([0.3, -0.2, -4.0], np.float32)
        shs = rng.normal(0, 0.4, (Pn, 16, 3)).astype(np.float32)
        shs[:, 0] = rng.uniform(-2, 2, (Pn, 3))
        res = {}
        for deg in range(4):
            d = torch.from_numpy(means - campos)
            d = d / d.norm(dim=1, keepdim=True)
            c = shu.eval_sh(deg, torch.from_numpy(shs).transpose(1, 2)[..., :(deg + 1) ** 2], d)
            res[f"rgb_deg{deg}"] = torch.clamp_min(c + 0.5, 0.0).numpy()
        np.savez_compressed(os.path.join(HERE, "sh.npz"), means=means, campos=campos, shs=shs, **res)

        # ---- (4) cov3D from scale / normalised rotation ----
        s = np.exp(rng.uniform(np.log(0.01), np.log(0.5), (Pn, 3))).astype(np.float32)
        q = rng.normal(size=(Pn, 4)).astype(np.float32)
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        mod = 1.3
        L = gu.build_scaling_rotation(mod * torch.from_numpy(s), torch.from_numpy(q))
        cov = gu.strip_symmetric(L @ L.transpose(1, 2))
        np.savez_compressed(os.path.join(HERE, "cov3d.npz"), scales=s, rotations=q, scale_modifier=np.float32(mod),
                            cov3D=cov.numpy())

        # ---- (5) cameras (scene/cameras.py:63-79) ----
        cams = {}
        for name, (R, T, fovx, fovy) in {
            "m1": (np.eye(3), np.zeros(3), 2 * np.arctan(np.tan(np.pi / 6) * 1920 / 1080), np.pi / 3),
            "orbit": (np.array([[0.8, 0.0, -0.6], [0.36, 0.8, 0.48], [0.48, -0.6, 0.64]]), np.array([0.1, -0.2, 4.0]),
                      0.6911112, 0.6911112),
        }.items():
            w2v = torch.tensor(gr.getWorld2View2(R, T)).transpose(0, 1)
            proj = gr.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
            full = w2v.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
            cams[name + "_R"] = R.astype(np.float32)
            cams[name + "_T"] = T.astype(np.float32)
            cams[name + "_fov"] = np.array([fovx, fovy], np.float64)
            cams[name + "_view"] = w2v.numpy()
            cams[name + "_proj"] = full.numpy()
            cams[name + "_campos"] = w2v.inverse()[3, :3].numpy()
        np.savez_compressed(os.path.join(HERE, "camera.npz"), **cams)

        # ---- (6) Fibonacci directions ----
        nrm = rng.normal(size=(64, 3)).astype(np.float32)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        dirs, areas = gr.fibonacci_sphere_sampling(torch.from_numpy(nrm), 24, random_rotate=False)
        np.savez_compressed(os.path.join(HERE, "fib.npz"), normals=nrm, dirs=dirs.numpy(), areas=areas.numpy())
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
