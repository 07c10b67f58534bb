"""render() — the caller of the rasterizer, mirroring the reference's
gaussian_renderer/__init__.py:18-98 (argument meaning, settings construction,
returned dict).  Differences: the screen-space dummy tensor is created on the
Gaussians' device instead of a hard-coded "cuda", and `pipe` may be any object
with a `debug` attribute.  integrate / evaluate_sdf (:101-222) and
sample_depth (:225-278) follow.
"""
from __future__ import annotations

import math

import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, kernel_size, scaling_modifier=1.0,
           require_depth: bool = True):
    """Render the scene.  `pc` exposes the GaussianModel getters
    (get_xyz, get_scaling_n_opacity_with_3D_filter, get_rotation, get_features,
    get_sg_axis, get_sg_sharpness, get_sg_color, active_sh_degree,
    active_sg_degree) as properties or zero-argument methods."""

    def _get(name):
        v = getattr(pc, name)
        return v() if callable(v) else v

    xyz = _get("get_xyz")
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:  # noqa: BLE001 - same tolerance as the reference
        pass
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, kernel_size=kernel_size, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, sg_degree=pc.active_sg_degree, campos=viewpoint_camera.camera_center,
        prefiltered=False, require_depth=require_depth, debug=getattr(pipe, "debug", False))
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    scales, opacity = _get("get_scaling_n_opacity_with_3D_filter")
    image, radii, median_depth, alpha, normal = rasterizer(
        means3D=xyz, means2D=screenspace_points, shs=_get("get_features"), sg_axis=_get("get_sg_axis"),
        sg_sharpness=_get("get_sg_sharpness"), sg_color=_get("get_sg_color"), colors_precomp=None,
        opacities=opacity, scales=scales, rotations=_get("get_rotation"), cov3D_precomp=None)
    return {"render": image, "mask": alpha, "median_depth": median_depth, "viewspace_points": screenspace_points,
            "visibility_filter": radii > 0, "radii": radii, "normal": normal}


def _query_rasterizer(viewpoint_camera, pc, pipe, kernel_size, scaling_modifier, bg):
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, kernel_size=kernel_size, bg=bg, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, sg_degree=pc.active_sg_degree, campos=viewpoint_camera.camera_center,
        prefiltered=False, debug=getattr(pipe, "debug", False), require_depth=True)
    return GaussianRasterizer(raster_settings=raster_settings)


def _query_gaussians(pc, pipe, scaling_modifier):
    """means3D, opacity, scales, rotations, cov3D_precomp as the reference's
    point queries take them (gaussian_renderer/__init__.py:131-143)."""

    def _get(name, *a):
        v = getattr(pc, name)
        return v(*a) if callable(v) else v

    scales = rotations = cov3D_precomp = None
    if getattr(pipe, "compute_cov3D_python", False):
        cov3D_precomp = _get("get_covariance", scaling_modifier)
    else:
        scales = _get("get_scaling_with_3D_filter")
        rotations = _get("get_rotation")
    return _get("get_xyz"), _get("get_opacity_with_3D_filter"), scales, rotations, cov3D_precomp


def integrate(points3D, viewpoint_camera, pc, pipe, kernel_size, scaling_modifier=1.0):
    """Opacity of the Gaussian field at world points [PN, 3] seen from
    `viewpoint_camera` (gaussian_renderer/__init__.py:101-160; called by the
    tetrahedral mesh extraction, mesh_extract_tetrahedra.py:75)."""
    rasterizer = _query_rasterizer(viewpoint_camera, pc, pipe, kernel_size, scaling_modifier, None)
    means3D, opacity, scales, rotations, cov3D_precomp = _query_gaussians(pc, pipe, scaling_modifier)
    alpha_integrated, inside = rasterizer.integrate(points3D=points3D, means3D=means3D, opacities=opacity,
                                                    scales=scales, rotations=rotations,
                                                    cov3D_precomp=cov3D_precomp, view2gaussian_precomp=None)
    return {"alpha_integrated": alpha_integrated, "inside": inside}


def evaluate_sdf(points3D, viewpoint_camera, pc, pipe, kernel_size, scaling_modifier=1.0):
    """Median depth along each point's ray and the point's signed distance to
    it (gaussian_renderer/__init__.py:162-222)."""
    rasterizer = _query_rasterizer(viewpoint_camera, pc, pipe, kernel_size, scaling_modifier, None)
    means3D, opacity, scales, rotations, cov3D_precomp = _query_gaussians(pc, pipe, scaling_modifier)
    depth, sdf, inside = rasterizer.evaluate_sdf(points3D=points3D, means3D=means3D, opacities=opacity,
                                                 scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp,
                                                 view2gaussian_precomp=None)
    return {"depth": depth, "sdf": sdf, "inside": inside}


def sample_depth(points3D, viewpoint_camera, pc, pipe, kernel_size, scaling_modifier=1.0):
    """Median depth of the Gaussians at world points seen from
    `viewpoint_camera` (gaussian_renderer/__init__.py:225-278; called by the
    multi-view loss, utils/loss_utils.py:160).  `pc` exposes get_xyz,
    get_opacity_with_3D_filter, get_scaling_with_3D_filter, get_rotation
    (and get_covariance when pipe.compute_cov3D_python)."""

    def _get(name, *a):
        v = getattr(pc, name)
        return v(*a) if callable(v) else v

    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, kernel_size=kernel_size, bg=0, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, sg_degree=pc.active_sg_degree, campos=viewpoint_camera.camera_center,
        prefiltered=False, debug=getattr(pipe, "debug", False), require_depth=True)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    scales = rotations = cov3D_precomp = None
    if getattr(pipe, "compute_cov3D_python", False):
        cov3D_precomp = _get("get_covariance", scaling_modifier)
    else:
        scales = _get("get_scaling_with_3D_filter")
        rotations = _get("get_rotation")
    depth, inside = rasterizer.sample_depth(points3D=points3D, means3D=_get("get_xyz"),
                                            opacities=_get("get_opacity_with_3D_filter"), scales=scales,
                                            rotations=rotations, cov3D_precomp=cov3D_precomp)
    return {"sampled_depth": depth, "inside": inside}
