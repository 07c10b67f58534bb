"""Synthetic scenes and cameras for the rasterizer path.

Camera conventions restate the reference's
  utils/graphics_utils.py:44-92   getWorld2View2 / getProjectionMatrix
  scene/cameras.py:70-73          world_view_transform / full_proj_transform / camera_center
and the per-Gaussian activations restate the GaussianModel getters the
renderer feeds the rasterizer with:
  scene/gaussian_model.py:146-212 get_scaling_n_opacity_with_3D_filter,
                                  get_rotation, get_features, get_sg_*.

Every tensor is generated on the CPU from a seeded torch.Generator, so CPU,
GPU and every rank see identical values.  This module is product-side
plumbing (bench.py, smoke(), tests); it does not touch the oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


# --------------------------------------------------------------------------
# Cameras (graphics_utils.py:44-92, cameras.py:70-73)
# --------------------------------------------------------------------------
def world2view(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """getWorld2View2(R, t) with translate=0, scale=1: w2c = [R^T | t]."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def projection(znear: float, zfar: float, fovx: float, fovy: float) -> torch.Tensor:
    tan_y = math.tan(fovy / 2)
    tan_x = math.tan(fovx / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
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
    """The attributes of scene/cameras.py::Camera that render() reads."""

    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor  # [4,4], column-major W2C (transposed)
    full_proj_transform: torch.Tensor  # [4,4]
    camera_center: torch.Tensor  # [3]

    def to(self, device) -> "Camera":
        return Camera(self.image_width, self.image_height, self.FoVx, self.FoVy,
                      self.world_view_transform.to(device), self.full_proj_transform.to(device),
                      self.camera_center.to(device))


def make_camera(W: int, H: int, R: np.ndarray | None = None, T: np.ndarray | None = None,
                fovx_deg: float = 60.0, znear: float = 0.01, zfar: float = 100.0) -> Camera:
    R = np.eye(3) if R is None else R
    T = np.zeros(3) if T is None else T
    fovx = math.radians(fovx_deg)
    fovy = 2.0 * math.atan(math.tan(fovx / 2) * H / W)
    wvt = torch.tensor(world2view(R, T)).transpose(0, 1).contiguous()
    proj = projection(znear, zfar, fovx, fovy).transpose(0, 1)
    full = (wvt.unsqueeze(0).bmm(proj.unsqueeze(0))).squeeze(0).contiguous()
    center = wvt.inverse()[3, :3].contiguous()
    return Camera(W, H, fovx, fovy, wvt, full, center)


def orbit_cameras(n: int, W: int, H: int, center_z: float = 6.0, max_deg: float = 20.0) -> list[Camera]:
    """C4's views: n cameras rotated in [-max_deg, +max_deg] about y around
    (0, 0, center_z), each looking at that point."""
    cams = []
    angles = np.linspace(-max_deg, max_deg, n) if n > 1 else np.zeros(1)
    c = np.array([0.0, 0.0, center_z])
    for a in angles:
        th = math.radians(float(a))
        Rc = np.array([[math.cos(th), 0, math.sin(th)], [0, 1, 0], [-math.sin(th), 0, math.cos(th)]])
        pos = c - Rc @ np.array([0.0, 0.0, center_z])  # camera looks along its +z toward c
        t = -Rc.T @ pos
        cams.append(make_camera(W, H, Rc, t))
    return cams


# --------------------------------------------------------------------------
# Gaussians (gaussian_model.py:146-212)
# --------------------------------------------------------------------------
@dataclass
class RawGaussians:
    """Un-activated parameters, as GaussianModel stores them."""

    xyz: torch.Tensor  # [P,3]
    features_dc: torch.Tensor  # [P,1,3]
    features_rest: torch.Tensor  # [P,SHM-1,3]
    scaling: torch.Tensor  # [P,3] (log)
    rotation: torch.Tensor  # [P,4]
    opacity: torch.Tensor  # [P,1] (logit)
    sg_axis: torch.Tensor  # [P,SGM,3]
    sg_sharpness: torch.Tensor  # [P,SGM] (pre-softplus)
    sg_color: torch.Tensor  # [P,SGM,3]
    filter_3D: torch.Tensor  # [P,1]

    def to(self, device) -> "RawGaussians":
        return RawGaussians(*[getattr(self, f).to(device) for f in self.__dataclass_fields__])

    def requires_grad_(self) -> "RawGaussians":
        for f in self.__dataclass_fields__:
            if f != "filter_3D":
                getattr(self, f).requires_grad_(True)
        return self

    # ---- getters (gaussian_model.py:146-212) ----
    def get_scaling_n_opacity_with_3D_filter(self):
        opacity = torch.sigmoid(self.opacity)
        scales = torch.exp(self.scaling)
        scales_square = torch.square(scales)
        det1 = scales_square.prod(dim=1)
        scales_after_square = scales_square + torch.square(self.filter_3D)
        det2 = scales_after_square.prod(dim=1)
        coef = det1.sqrt() * det2.rsqrt()
        scales = scales_after_square.sqrt()
        return scales, opacity * coef[..., None]

    def get_rotation(self):
        return torch.nn.functional.normalize(self.rotation)

    def get_features(self):
        return torch.cat((self.features_dc, self.features_rest), dim=1)

    def get_sg_axis(self):
        return torch.nn.functional.normalize(self.sg_axis, dim=2)

    def get_sg_sharpness(self):
        return torch.nn.functional.softplus(self.sg_sharpness)

    def get_sg_color(self):
        return self.sg_color


@torch.no_grad()
def compute_filter_3D(xyz: torch.Tensor, cameras) -> torch.Tensor:
    """Mip-Splatting 3D filter, restating gaussian_model.py:225-262: per
    Gaussian the smallest depth over the training cameras that see it (in front
    of z = 0.2 and within 1.15x the half field of view), over the largest focal
    length, times sqrt(0.2).  `cameras` expose R [3,3] (stored transposed, as
    the reference keeps it), T [3], image_width, image_height, Fx, Fy."""
    distance = torch.full((xyz.shape[0],), float("inf"), device=xyz.device)
    valid_points = torch.zeros(xyz.shape[0], device=xyz.device, dtype=torch.bool)
    focal_length = 0.0
    for cam in cameras:
        xyz_cam = torch.addmm(cam.T[None, :].to(xyz), xyz, cam.R.to(xyz))
        z = xyz_cam[:, 2]
        valid_depth = z > 0.2
        uv_abs = torch.abs(xyz_cam[:, :2] / z.unsqueeze(-1))
        bx = cam.image_width / cam.Fx * 0.575
        by = cam.image_height / cam.Fy * 0.575
        valid = valid_depth & (uv_abs[:, 0] <= bx) & (uv_abs[:, 1] <= by)
        distance = torch.where(valid, torch.minimum(distance, z), distance)
        valid_points = valid_points | valid
        focal_length = max(focal_length, cam.Fx)
    distance[~valid_points] = distance[valid_points].max()
    return (distance / focal_length * (0.2 ** 0.5))[..., None]


def make_gaussians(P: int, sh_degree: int = 3, sg_degree: int = 0, seed: int = 0, fovx_deg: float = 60.0,
                   aspect: float = 1080 / 1920, z_range=(2.0, 10.0), log_scale_mean: float = math.log(0.02),
                   log_scale_std: float = 0.5, opacity_std: float = 1.5,
                   sh_max_degree: int | None = None) -> RawGaussians:
    """SURVEY §8(d) synthetic scene (seed 0 by default).  `sh_max_degree`
    sizes the SH rows as GaussianModel does ((max_sh_degree + 1)^2 rows,
    gaussian_model.py:264-266) while `sh_degree` is the active degree: the
    reference's SH warm-up (train.py:130) renders 16-row SH at degree 0..3."""
    g = torch.Generator().manual_seed(seed)
    tanx = math.tan(math.radians(fovx_deg) / 2)
    tany = tanx * aspect
    z = torch.empty(P).uniform_(z_range[0], z_range[1], generator=g)
    u = torch.empty(P).uniform_(-1, 1, generator=g)
    v = torch.empty(P).uniform_(-1, 1, generator=g)
    xyz = torch.stack([u * z * 1.1 * tanx, v * z * 1.1 * tany, z], 1)
    shm = ((sh_degree if sh_max_degree is None else sh_max_degree) + 1) ** 2
    dc = torch.randn(P, 1, 3, generator=g) * 0.5
    rest = torch.randn(P, shm - 1, 3, generator=g) * 0.05
    scaling = torch.randn(P, 3, generator=g) * log_scale_std + log_scale_mean
    rotation = torch.randn(P, 4, generator=g)
    opacity = torch.randn(P, 1, generator=g) * opacity_std
    sg_axis = torch.randn(P, sg_degree, 3, generator=g)
    sg_sharp = torch.randn(P, sg_degree, generator=g)
    sg_color = torch.randn(P, sg_degree, 3, generator=g) * 0.05
    filt = torch.zeros(P, 1)
    return RawGaussians(xyz, dc, rest, scaling, rotation, opacity, sg_axis, sg_sharp, sg_color, filt)


def activated_inputs(raw: RawGaussians) -> dict:
    """The tensors render() hands to GaussianRasterizer (gaussian_renderer/__init__.py:53-82)."""
    scales, opacity = raw.get_scaling_n_opacity_with_3D_filter()
    return dict(
        means3D=raw.xyz,
        shs=raw.get_features(),
        sg_axis=raw.get_sg_axis(),
        sg_sharpness=raw.get_sg_sharpness(),
        sg_color=raw.get_sg_color(),
        opacities=opacity,
        scales=scales,
        rotations=raw.get_rotation(),
    )


def upstream_grads(H: int, W: int, seed: int = 1, scale: float = 1e-3) -> dict:
    """Synthetic dL/d{color, median depth, alpha, normal}."""
    g = torch.Generator().manual_seed(seed)
    return dict(
        color=torch.randn(3, H, W, generator=g) * scale,
        mdepth=torch.randn(1, H, W, generator=g) * scale,
        alpha=torch.zeros(1, H, W),
        normal=torch.randn(3, H, W, generator=g) * scale,
    )


def tetra_points(inp):
    """GaussianModel.get_tetra_points (scene/gaussian_model.py:496-519): per
    Gaussian the 8 corners of its box at 1.5 scale and 6 axis points at 3
    scale, rotated, then every centre: 15 points per Gaussian, the point set
    mesh_extract_tetrahedra.py:75 integrates."""
    q = torch.nn.functional.normalize(inp["rotations"], dim=1)
    r, x, y, z = q.unbind(1)
    Rm = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
                      torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
                      torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
    near = [[sx * 1.5, sy * 1.5, sz * 1.5] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    far = [[3, 0, 0], [0, 3, 0], [0, 0, 3], [-3, 0, 0], [0, -3, 0], [0, 0, -3]]
    verts = torch.tensor(near + far, dtype=torch.float32, device=q.device)
    local = verts[None] * inp["scales"][:, None]
    corners = (local @ Rm.transpose(1, 2) + inp["means3D"][:, None]).reshape(-1, 3)
    return torch.cat([corners, inp["means3D"]], 0).contiguous()
