"""In-tree build of the HIP library and the torch binding.

Produces (git-ignored, but shipped to the GPU box with the tree):
  relightable3dgaussian_amd/lib/libr3dg_hip.so   -- HIP kernels + the C ABI of include/r3dg_hip.h
  relightable3dgaussian_amd/lib/_C.so             -- pybind module mirroring r3dg_rasterization._C

`python relightable3dgaussian_amd/build.py` rebuilds what is out of date. hipcc cross-compiles
for gfx950 without a GPU, so this runs in the CPU container too.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
# experiment builds put their objects / libraries elsewhere (tools/exp_build.sh)
LIB = os.environ.get("R3DG_LIB_DIR") or os.path.join(PKG, "lib")
INC = os.path.join(ROOT, "include")
OBJ = os.environ.get("R3DG_OBJ_DIR") or os.path.join(PKG, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

HIP_SOURCES = ["preprocess.hip", "render_fwd.hip", "render_bwd.hip", "brdf.hip", "shaders.hip", "rasterizer.hip",
               "optim.hip", "bvh.hip"]
HIP_FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result",
             "-munsafe-fp-atomics", f"-I{INC}", f"-I{CSRC}"]
# the key path (projection, radius, rect) must not contract a*b+c into fma: see preprocess.hip
# render_bwd: the SLP vectorizer pairs the two unrolled blend steps into packed f32 ops plus
# register shuffles (more instructions, 30 more VGPRs); plain scalar code measures faster; in
# render_fwd it packs the blend's channel sums into v_pk_fma_f32 (4 cycles each, as two v_fma_f32):
# scalar FMAs measured 1.5 % faster; brdf.hip: the BRDF forwards 1.5-2 % faster unpacked
# brdf.hip: the render equation restates the oracle's operation sequence (no a*b+c contraction), so
# the BRDF outputs are bit-identical to it
# render_bwd.hip: the max-memory-clause scheduling strategy (same registers): render_bwd -0.3 %,
# gather -1.5 % at M1 (round 5; max-ilp: +17 %, iterative-ilp: +1 %)
PER_FILE_FLAGS = {"preprocess.hip": ["-ffp-contract=off"], "bvh.hip": ["-ffp-contract=off"],
                  "brdf.hip": ["-ffp-contract=off", "-fno-slp-vectorize"],
                  "render_bwd.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
                  "render_fwd.hip": ["-fno-slp-vectorize"]}


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd[:3]) + " ...")


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs + [os.path.join(INC, "r3dg_hip.h")]


def build_hip(jobs: int = 8) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    hdrs = _headers()
    objs, cmds = [], []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace(".hip", ".o"))
        objs.append(o)
        if _newer(o, [s] + hdrs + [__file__]):
            extra = os.environ.get("R3DG_EXTRA_HIPFLAGS", "").split()  # experiment builds only
            cmds.append([HIPCC, "-c", s, "-o", o] + HIP_FLAGS + PER_FILE_FLAGS.get(src, []) + extra)
    with ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    so = os.path.join(LIB, "libr3dg_hip.so")
    if _newer(so, objs):
        _run([HIPCC, "-shared", "-o", so, *objs, "--offload-arch=gfx950", "-fPIC",
              "-Wl,-soname,libr3dg_hip.so"])
    return so


def build_torch_ext() -> str:
    """pybind module `_C` (csrc/torch_ext.cpp) linked against libr3dg_hip.so."""
    import torch
    from torch.utils import cpp_extension

    src = os.path.join(CSRC, "torch_ext.cpp")
    so = os.path.join(LIB, "_C.so")
    libso = os.path.join(LIB, "libr3dg_hip.so")
    if not _newer(so, [src, libso] + _headers() + [__file__]):
        return so
    inc = cpp_extension.include_paths() + [sysconfig.get_paths()["include"], INC, CSRC,
                                           os.path.join(ROCM, "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", so,
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-Wno-deprecated-declarations"]
    cmd += [f"-I{p}" for p in inc]
    cmd += [f"-L{LIB}", "-lr3dg_hip", f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10", "-lc10_hip", "-ltorch_hip", f"-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tlib}"]
    _run(cmd)
    return so


def build(jobs: int = 8, torch_ext: bool = True) -> None:
    build_hip(jobs)
    if torch_ext:
        build_torch_ext()


if __name__ == "__main__":
    build()
    print("built", os.listdir(LIB))
