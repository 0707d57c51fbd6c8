"""Gaussian PLY files: the reference's checkpoint point-cloud format.

Restates `GaussianModel.construct_list_of_attributes` / `save_ply` / `load_ply`
(scene/gaussian_model.py:630-656, 658-686, 693-793) without the `plyfile` dependency (absent from
this image): one `vertex` element of float32 properties, written as `plyfile` writes it
(binary little-endian, `property float <name>`), read from binary (either endianness) or ASCII
files with any numeric property types, properties matched by name as the reference does
(`f_rest_*`, `scale_*`, `rot*`, ... sorted by their numeric suffix).

Arrays use the reference's parameter shapes under the trainer's group names
(`relightable3dgaussian_amd/trainer.py` BASE_GROUPS / PBR_GROUPS): xyz [P,3], normal [P,3],
f_dc [P,1,3], f_rest [P,(D+1)^2-1,3], opacity [P,1], scaling [P,3], rotation [P,4]; with PBR
base_color [P,3], roughness [P,1], metallic [P,1], incidents_dc [P,1,3], incidents_rest
[P,(D+1)^2-1,3], visibility_dc [P,1,1], visibility_rest [P,15,1]. Values are the raw (pre-
activation) parameters, as the reference stores them.
"""
from __future__ import annotations

import os

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2", "ushort": "u2",
    "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4", "float": "f4", "float32": "f4",
    "double": "f8", "float64": "f8",
}


def attribute_names(sh_degree: int = 3, use_pbr: bool = True) -> list[str]:
    """construct_list_of_attributes (scene/gaussian_model.py:630-656)."""
    n_rest = 3 * ((sh_degree + 1) ** 2 - 1)
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)]
    names += [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"]
    names += [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]
    if use_pbr:
        names += [f"base_color_{i}" for i in range(3)] + ["roughness", "metallic"]
        names += [f"incidents_dc_{i}" for i in range(3)] + [f"incidents_rest_{i}" for i in range(n_rest)]
        names += ["visibility_dc_0"] + [f"visibility_rest_{i}" for i in range(15)]
    return names


def _channel_major(a: np.ndarray) -> np.ndarray:
    """[P, K, C] parameter -> [P, C*K] columns in the reference's transpose(1, 2).flatten order."""
    return np.ascontiguousarray(np.transpose(a, (0, 2, 1))).reshape(a.shape[0], -1)


def save_ply(path: str, params: dict, use_pbr: bool | None = None) -> None:
    """save_ply (scene/gaussian_model.py:658-686). params: name -> array/tensor (trainer names)."""
    def np_(x):
        return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)

    p = {k: np_(v).astype(np.float32, copy=False) for k, v in params.items()}
    if use_pbr is None:
        use_pbr = "base_color" in p
    P = p["xyz"].shape[0]
    sh_degree = int(round(np.sqrt(p["f_rest"].shape[1] + 1))) - 1
    cols = [p["xyz"], p["normal"], _channel_major(p["f_dc"]), _channel_major(p["f_rest"]), p["opacity"].reshape(P, 1),
            p["scaling"], p["rotation"]]
    if use_pbr:
        cols += [p["base_color"], p["roughness"].reshape(P, 1), p["metallic"].reshape(P, 1),
                 _channel_major(p["incidents_dc"]), _channel_major(p["incidents_rest"]),
                 _channel_major(p["visibility_dc"]), _channel_major(p["visibility_rest"])]
    names = attribute_names(sh_degree, use_pbr)
    data = np.ascontiguousarray(np.concatenate([c.reshape(P, -1) for c in cols], axis=1), dtype="<f4")
    assert data.shape[1] == len(names)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    header = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % P
    header += "".join("property float %s\n" % n for n in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(data.tobytes())


def read_vertices(path: str) -> np.ndarray:
    """The `vertex` element of a PLY file as a numpy structured array (plyfile's PlyData.read for
    the single-element files the reference writes; list properties are not supported)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements = None, []
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii", "replace").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                elements.append((tok[1], int(tok[2]), []))
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError(f"{path}: list properties are not supported")
                if tok[1] not in _PLY_TYPES:
                    raise ValueError(f"{path}: unknown property type {tok[1]}")
                elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        if fmt not in ("binary_little_endian", "binary_big_endian", "ascii"):
            raise ValueError(f"{path}: unsupported format {fmt}")
        end = "<" if fmt == "binary_little_endian" else ">"
        for name, count, props in elements:
            dtype = np.dtype([(n, end + t) for n, t in props])
            if fmt == "ascii":
                rows = [f.readline().split() for _ in range(count)]
                arr = np.zeros(count, dtype=dtype)
                if count:
                    vals = np.asarray(rows, dtype=np.float64)
                    for k, (n, _) in enumerate(props):
                        arr[n] = vals[:, k]
            else:
                buf = f.read(dtype.itemsize * count)
                if len(buf) != dtype.itemsize * count:
                    raise ValueError(f"{path}: truncated element {name}")
                arr = np.frombuffer(buf, dtype=dtype)
            if name == "vertex":
                return arr
    raise ValueError(f"{path}: no vertex element")


def _sorted(names, prefix):
    sel = [n for n in names if n.startswith(prefix)]
    return sorted(sel, key=lambda x: int(x.split("_")[-1]))


def load_ply(path: str, max_sh_degree: int = 3, use_pbr: bool = True) -> dict:
    """load_ply (scene/gaussian_model.py:693-793) -> name -> float32 numpy array (trainer names)."""
    v = read_vertices(path)
    names = v.dtype.names
    P = v.shape[0]
    col = lambda n: np.asarray(v[n], dtype=np.float32)  # noqa: E731
    stack = lambda ns: np.stack([col(n) for n in ns], axis=1) if ns else np.zeros((P, 0), np.float32)  # noqa: E731
    n_rest = 3 * (max_sh_degree + 1) ** 2 - 3
    out = {"xyz": stack(["x", "y", "z"]), "normal": stack(["nx", "ny", "nz"]),
           "opacity": col("opacity")[:, None]}
    out["f_dc"] = stack([f"f_dc_{i}" for i in range(3)]).reshape(P, 3, 1).transpose(0, 2, 1)
    rest = _sorted(names, "f_rest_")
    if len(rest) != n_rest:
        raise ValueError(f"{path}: {len(rest)} f_rest_* properties, expected {n_rest} for SH degree {max_sh_degree}")
    out["f_rest"] = stack(rest).reshape(P, 3, n_rest // 3).transpose(0, 2, 1)
    out["scaling"] = stack(_sorted(names, "scale_"))
    out["rotation"] = stack(_sorted(names, "rot"))
    if use_pbr:
        out["base_color"] = stack(_sorted(names, "base_color"))
        out["roughness"] = col("roughness")[:, None]
        out["metallic"] = col("metallic")[:, None]
        out["incidents_dc"] = stack([f"incidents_dc_{i}" for i in range(3)]).reshape(P, 3, 1).transpose(0, 2, 1)
        inc = _sorted(names, "incidents_rest_")
        if len(inc) != n_rest:
            raise ValueError(f"{path}: {len(inc)} incidents_rest_* properties, expected {n_rest}")
        out["incidents_rest"] = stack(inc).reshape(P, 3, n_rest // 3).transpose(0, 2, 1)
        out["visibility_dc"] = col("visibility_dc_0").reshape(P, 1, 1)
        vis = _sorted(names, "visibility_rest_")
        if len(vis) != 15:
            raise ValueError(f"{path}: {len(vis)} visibility_rest_* properties, expected 15")
        out["visibility_rest"] = stack(vis).reshape(P, 1, 15).transpose(0, 2, 1)
    return {k: np.ascontiguousarray(a, dtype=np.float32) for k, a in out.items()}


__all__ = ["attribute_names", "save_ply", "load_ply", "read_vertices"]
