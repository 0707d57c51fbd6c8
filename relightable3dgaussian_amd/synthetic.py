"""Cameras and synthetic scenes for benchmarks and parity tests (no datasets exist offline).

Camera matrices restate utils/graphics_utils.py getWorld2View2 / getProjectionMatrix and the
transposed convention of scene/cameras.py:63-79 (pinned by tests/golden/camera.npz). Scenes
follow SURVEY.md §8d: "M1" (the metric scene: 1M Gaussians, 1920x1080), the lego-like
ball scene "C2", and small variants for parity tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


def world2view(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """getWorld2View2(R, t) with translate 0 and scale 1 (graphics_utils.py:136-146)."""
    Rt = np.zeros((4, 4), np.float64)
    Rt[:3, :3] = np.asarray(R, np.float64).T
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def projection(znear: float, zfar: float, fovx: float, fovy: float) -> np.ndarray:
    """getProjectionMatrix (graphics_utils.py:149-168)."""
    tan_y, tan_x = math.tan(fovy / 2), math.tan(fovx / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = np.zeros((4, 4), np.float32)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    """The raster-settings view of scene/cameras.py Camera (matrices already transposed)."""

    width: int
    height: int
    fovx: float
    fovy: float
    view: np.ndarray      # world_view_transform
    view_inv: np.ndarray  # world_view_transform_inverse
    proj: np.ndarray      # full_proj_transform
    proj_inv: np.ndarray  # full_proj_transform_inverse
    campos: np.ndarray    # camera_center

    @property
    def tanfovx(self) -> float:
        return math.tan(self.fovx * 0.5)

    @property
    def tanfovy(self) -> float:
        return math.tan(self.fovy * 0.5)

    @property
    def cx(self) -> float:
        return self.width / 2.0  # Camera.get_intrinsics without fx (cameras.py:104-111)

    @property
    def cy(self) -> float:
        return self.height / 2.0

    @property
    def focal(self) -> tuple[float, float]:
        return self.width / (2.0 * self.tanfovx), self.height / (2.0 * self.tanfovy)


def make_camera(R, T, fovx: float, fovy: float, width: int, height: int, znear: float = 0.01,
                zfar: float = 100.0) -> Camera:
    import torch  # matrix products in float32 exactly as scene/cameras.py does them

    w2v = torch.tensor(world2view(R, T)).transpose(0, 1)
    proj = torch.tensor(projection(znear, zfar, fovx, fovy)).transpose(0, 1)
    full = w2v.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    return Camera(width, height, fovx, fovy, w2v.numpy().copy(), w2v.inverse().numpy().copy(), full.numpy().copy(),
                  full.inverse().numpy().copy(), w2v.inverse()[3, :3].numpy().copy())


def look_at(eye, target=(0.0, 0.0, 0.0), up=(0.0, -1.0, 0.0)):
    """(R, T) of a camera at `eye` looking at `target` (COLMAP convention, +z forward, y down)."""
    eye, target, up = (np.asarray(v, np.float64) for v in (eye, target, up))
    z = target - eye
    z /= np.linalg.norm(z)
    x = np.cross(up, z)
    if np.linalg.norm(x) < 1e-8:
        x = np.cross(np.array([0.0, 0.0, 1.0]), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R_c2w = np.stack([x, y, z], axis=1)  # columns: camera axes in world
    R_w2c = R_c2w.T
    T = -R_w2c @ eye
    return R_c2w, T  # the reference stores R as camera-to-world rotation (getWorld2View uses R.T)


def orbit_camera(azimuth_deg: float, elevation_deg: float, radius: float, fov: float, width: int,
                 height: int) -> Camera:
    az, el = math.radians(azimuth_deg), math.radians(elevation_deg)
    eye = radius * np.array([math.cos(el) * math.sin(az), -math.sin(el), -math.cos(el) * math.cos(az)])
    R, T = look_at(eye)
    fovy = fov
    fovx = 2 * math.atan(math.tan(fov / 2) * width / height)
    return make_camera(R, T, fovx, fovy, width, height)


@dataclass
class Scene:
    means3D: np.ndarray
    scales: np.ndarray
    rotations: np.ndarray
    opacity: np.ndarray
    sh: np.ndarray
    features: np.ndarray

    @property
    def P(self) -> int:
        return int(self.means3D.shape[0])


def m1_camera(width: int = 1920, height: int = 1080) -> Camera:
    fovy = math.pi / 3  # 60 degrees, fy = fx = 935.3 at 1080p
    fovx = 2 * math.atan(math.tan(fovy / 2) * width / height)
    return make_camera(np.eye(3), np.zeros(3), fovx, fovy, width, height)


def m1_scene(P: int = 1_000_000, S: int = 11, seed: int = 0, cam: Camera | None = None) -> Scene:
    """SURVEY.md §8d "M1": camera at the origin looking +z, Gaussians in the view frustum at z in
    [3, 8], log-uniform scales in [0.003, 0.03], random unit quaternions, opacity U(0.05, 0.95),
    degree-3 SH with DC ~ (U(0,1) - 0.5) / C0 and rest N(0, 0.05^2), features U(0, 1)."""
    cam = cam or m1_camera()
    rng = np.random.default_rng(seed)
    z = rng.uniform(3, 8, P)
    x = rng.uniform(-1, 1, P) * z * cam.tanfovx * 1.05
    y = rng.uniform(-1, 1, P) * z * cam.tanfovy * 1.05
    means = np.stack([x, y, z], 1).astype(np.float32)
    scales = np.exp(rng.uniform(np.log(0.003), np.log(0.03), (P, 3))).astype(np.float32)
    q = rng.normal(size=(P, 4))
    rot = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    opacity = rng.uniform(0.05, 0.95, (P, 1)).astype(np.float32)
    sh = np.empty((P, 16, 3), np.float32)
    sh[:, 0] = (rng.uniform(0, 1, (P, 3)) - 0.5) / 0.28209479
    sh[:, 1:] = rng.normal(0, 0.05, (P, 15, 3))
    feats = rng.uniform(0, 1, (P, S)).astype(np.float32)
    return Scene(means, scales, rot, opacity, sh, feats)


def ball_scene(P: int = 300_000, S: int = 21, seed: int = 0, radius: float = 1.3) -> Scene:
    """SURVEY.md §8d "C2" (lego stand-in): Gaussians uniformly in a ball of radius 1.3."""
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(P, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = radius * rng.uniform(0, 1, (P, 1)) ** (1 / 3)
    means = (d * r).astype(np.float32)
    scales = np.exp(rng.uniform(np.log(0.002), np.log(0.02), (P, 3))).astype(np.float32)
    q = rng.normal(size=(P, 4))
    rot = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    opacity = rng.uniform(0.05, 0.95, (P, 1)).astype(np.float32)
    sh = np.empty((P, 16, 3), np.float32)
    sh[:, 0] = (rng.uniform(0, 1, (P, 3)) - 0.5) / 0.28209479
    sh[:, 1:] = rng.normal(0, 0.05, (P, 15, 3))
    feats = rng.uniform(0, 1, (P, S)).astype(np.float32)
    return Scene(means, scales, rot, opacity, sh, feats)


def needle_scene(P: int = 300, S: int = 11, seed: int = 0, cam: Camera | None = None,
                 sigma_px=(100.0, 1000.0), opacity=(0.005, 0.05)) -> Scene:
    """Adversarial scene for the quadrant cull (r3dg_common.h quadrant_live): large, needle-shaped,
    faint splats on the screen diagonals, as trained scenes hold in their backgrounds. For the
    M1 camera (identity rotation, +z forward): the long axis has a screen-space sigma log-uniform
    in `sigma_px`, at 45 or 135 degrees (+-2); the two short axes are 1e-6 world units, so the 2D
    covariance's short axis is the 0.3 px^2 low-pass floor (forward.cu:110-111); opacity uniform
    in `opacity`; means projected anywhere in [-600, W+600] x [-600, H+600] px, mostly far from
    the tiles the splat covers. The conic form's terms reach ~1e6 along the needle and cancel to
    a few units: the regime where a fixed cull margin is smaller than the fp32 rounding."""
    cam = cam or m1_camera()
    rng = np.random.default_rng(seed)
    fx, fy = cam.focal
    z = rng.uniform(3, 8, P)
    u = rng.uniform(-600, cam.width + 600, P)
    v = rng.uniform(-600, cam.height + 600, P)
    means = np.stack([(u - cam.cx) / fx * z, (v - cam.cy) / fy * z, z], 1).astype(np.float32)
    sig = np.exp(rng.uniform(np.log(sigma_px[0]), np.log(sigma_px[1]), P))
    scales = np.full((P, 3), 1e-6, np.float64)
    scales[:, 0] = sig * z / fx
    theta = np.radians(np.where(rng.uniform(size=P) < 0.5, 45.0, 135.0) + rng.uniform(-2, 2, P))
    rot = np.zeros((P, 4))
    rot[:, 0], rot[:, 3] = np.cos(theta / 2), np.sin(theta / 2)  # (w, x, y, z): about the view axis
    op = rng.uniform(opacity[0], opacity[1], (P, 1)).astype(np.float32)
    sh = np.empty((P, 16, 3), np.float32)
    sh[:, 0] = (rng.uniform(0, 1, (P, 3)) - 0.5) / 0.28209479
    sh[:, 1:] = rng.normal(0, 0.05, (P, 15, 3))
    feats = rng.uniform(0, 1, (P, S)).astype(np.float32)
    return Scene(means, scales.astype(np.float32), rot.astype(np.float32), op, sh, feats)


def small_scene(P: int = 2000, S: int = 11, seed: int = 0, width: int = 64, height: int = 48,
                scale_range=(0.02, 0.2)) -> tuple[Scene, Camera]:
    """Small parity scene: an M1-style frustum fill at a size the CPU oracle finishes in seconds."""
    fovy = math.radians(50)
    fovx = 2 * math.atan(math.tan(fovy / 2) * width / height)
    R, T = look_at((0.15, -0.1, -0.2), (0.0, 0.0, 4.0))
    cam = make_camera(R, T, fovx, fovy, width, height)
    rng = np.random.default_rng(seed)
    z = rng.uniform(2.5, 6, P)
    x = rng.uniform(-1, 1, P) * z * math.tan(fovx / 2) * 1.2
    y = rng.uniform(-1, 1, P) * z * math.tan(fovy / 2) * 1.2
    means = np.stack([x, y, z], 1).astype(np.float32)
    scales = np.exp(rng.uniform(np.log(scale_range[0]), np.log(scale_range[1]), (P, 3))).astype(np.float32)
    q = rng.normal(size=(P, 4))
    rot = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    opacity = rng.uniform(0.05, 0.99, (P, 1)).astype(np.float32)
    sh = np.empty((P, 16, 3), np.float32)
    sh[:, 0] = (rng.uniform(0, 1, (P, 3)) - 0.5) / 0.28209479
    sh[:, 1:] = rng.normal(0, 0.1, (P, 15, 3))
    feats = rng.uniform(0, 1, (P, S)).astype(np.float32)
    return Scene(means, scales, rot, opacity, sh, feats), cam


def brdf_inputs(P: int, seed: int = 0, S: int = 16) -> dict:
    """SURVEY.md §8d "C1" BRDF inputs."""
    rng = np.random.default_rng(seed)
    n = rng.normal(size=(P, 3)); n /= np.linalg.norm(n, axis=1, keepdims=True)
    v = rng.normal(size=(P, 3)); v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    return dict(base=f(rng.uniform(0, 1, (P, 3))), rough=f(rng.uniform(0.05, 1, (P, 1))),
                metal=f(rng.uniform(0, 1, (P, 1))), normals=f(n), viewdirs=f(v),
                incidents=f(rng.normal(0, 0.1, (P, S, 3))), visibility=f(rng.normal(0, 0.1, (P, S, 1))),
                env=f(rng.normal(0, 0.1, (1, S, 3))))
