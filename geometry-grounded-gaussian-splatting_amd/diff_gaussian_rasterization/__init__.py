"""MI355X drop-in for the reference's `diff_gaussian_rasterization` package.

Same public surface as DGR/diff_gaussian_rasterization/__init__.py:
  rasterize_gaussians(...)                 (:23-50)
  _RasterizeGaussians (autograd.Function)  (:53-251)
  GaussianRasterizationSettings (15 fields, same order)  (:254-269)
  GaussianRasterizer (nn.Module): forward, markVisible   (:272-336)
so `from diff_gaussian_rasterization import GaussianRasterizationSettings,
GaussianRasterizer` (gaussian_renderer/__init__.py:14) works unchanged once
this directory's parent is on sys.path.  The compute lives in libgsr.so
(hand-written HIP for gfx950) behind `_C`.

  GaussianRasterizer.integrate / evaluate_sdf (forward-only)  (:338-468)
  GaussianRasterizer.sample_depth + _SampleDepth (autograd.Function)  (:470-655)
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

# Rasterizer colour backwards (SH path) run in this process; gsr_dist.FactoredViewGrads
# checks that exactly one ran between two gradient exchanges (its contract).
_colour_backward_calls = 0


def colour_backward_count() -> int:
    """Number of _RasterizeGaussians backwards that produced SH gradients."""
    return _colour_backward_calls


# The view-parallel gradient exchange run inside every rasterizer backward
# (gsr_dist.OverlappedViewGrads.install); None: the reference's single-view backward.
_view_exchange = None


def set_view_exchange(exchange) -> None:
    global _view_exchange
    _view_exchange = exchange


def cpu_deep_copy_tuple(input_tuple):
    copied_tensors = [item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple]
    return tuple(copied_tensors)


def rasterize_gaussians(means3D, means2D, sh, sg_axis, sg_sharpness, sg_color, colors_precomp, opacities, scales,
                        rotations, cov3Ds_precomp, raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, sg_axis, sg_sharpness, sg_color, colors_precomp,
                                     opacities, scales, rotations, cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, sg_axis, sg_sharpness, sg_color, colors_precomp, opacities, scales,
                rotations, cov3Ds_precomp, raster_settings, sh_rest=None):
        # (sh_rest, not in the reference: the split SH layout, sh = DC rows [P, 1, 3], GaussianRasterizer)
        s = raster_settings
        kw_rest = {} if sh_rest is None else {"sh_rest": sh_rest}
        args = (s.bg, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh, sg_axis,
                sg_sharpness, sg_color, s.sh_degree, s.sg_degree, s.scale_modifier, s.viewmatrix, s.projmatrix,
                s.tanfovx, s.tanfovy, s.kernel_size, s.image_height, s.image_width, s.campos, s.prefiltered,
                s.require_depth, s.debug)
        if s.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians(*args, **kw_rest)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args, **kw_rest)
        num_rendered, color, alpha, normal, mdepth, radii, geomBuffer, binningBuffer, imgBuffer, tileBuffer = out
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        # unused outputs reach the backward as None (zero upstream gradient: the kernels skip them)
        # instead of as materialised zero images; radii has no gradient
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh, sg_axis,
                              sg_sharpness, sg_color, alpha, normal, mdepth, radii, geomBuffer, binningBuffer,
                              imgBuffer, tileBuffer, sh_rest)
        return color, radii, mdepth, alpha, normal

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_mdepth, grad_alpha, grad_normal):
        global _colour_backward_calls
        num_rendered = ctx.num_rendered
        s = ctx.raster_settings
        (means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh, sg_axis, sg_sharpness, sg_color,
         alpha, normal, mdepth, radii, geomBuffer, binningBuffer, imgBuffer, tileBuffer, sh_rest) = ctx.saved_tensors
        args = (s.bg, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh, sg_axis,
                sg_sharpness, sg_color, s.sh_degree, s.sg_degree, s.scale_modifier, s.viewmatrix, s.projmatrix,
                s.tanfovx, s.tanfovy, s.kernel_size, grad_color, grad_mdepth, grad_alpha, grad_normal, alpha, normal,
                mdepth, s.campos, radii, geomBuffer, num_rendered, binningBuffer, imgBuffer, tileBuffer,
                s.require_depth, s.debug)
        ex = _view_exchange
        kw = {} if sh_rest is None else {"sh_rest": sh_rest}
        if ex is not None:  # gsr_dist.OverlappedViewGrads: the exchange rides on the backward's Gaussian ranges
            ex.begin(s.campos, means3D.shape[0], scales.numel() > 0, sh.numel() > 0)
            kw["exchange"] = ex
        try:
            if s.debug:
                cpu_args = cpu_deep_copy_tuple(args)
                try:
                    g = _C.rasterize_gaussians_backward(*args, **kw)
                except Exception as ex_:
                    torch.save(cpu_args, "snapshot_bw.dump")
                    print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                    raise ex_
            else:
                g = _C.rasterize_gaussians_backward(*args, **kw)
        except BaseException:
            if ex is not None:  # the exchange's remaining collectives are posted, its works settled
                ex.abort()
            raise
        if ex is not None:
            ex.finish(g, means3D, sg_axis, sg_sharpness, sg_color, s.sh_degree, s.sg_degree)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh,
         grad_sg_axis, grad_sg_sharpness, grad_sg_color, grad_scales, grad_rotations) = g[:11]
        grad_sh_rest = g[11] if len(g) > 11 else None
        if sh.numel():
            _colour_backward_calls += 1
        return (grad_means3D, grad_means2D, grad_sh, grad_sg_axis, grad_sg_sharpness, grad_sg_color,
                grad_colors_precomp, grad_opacities, grad_scales, grad_rotations, grad_cov3Ds_precomp, None,
                grad_sh_rest)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    kernel_size: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    sg_degree: int
    campos: torch.Tensor
    prefiltered: bool
    require_depth: bool
    debug: bool


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            visible = _C.mark_visible(positions, s.viewmatrix, s.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, sg_axis=None, sg_sharpness=None, sg_color=None,
                colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None):
        raster_settings = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        # shs may also be the pair (features_dc [P, 1, 3], features_rest [P, M-1, 3]) as GaussianModel keeps
        # them: the kernels read and write the two as they are (no concatenation: gsr.h, the split SH layout)
        sh_rest = None
        if isinstance(shs, (tuple, list)):
            shs, sh_rest = shs
        if shs is None:
            shs = torch.Tensor([])
        if colors_precomp is None:
            colors_precomp = torch.Tensor([])
        if scales is None:
            scales = torch.Tensor([])
        if rotations is None:
            rotations = torch.Tensor([])
        if cov3D_precomp is None:
            cov3D_precomp = torch.Tensor([])
        if sh_rest is not None:
            return _RasterizeGaussians.apply(means3D, means2D, shs, sg_axis, sg_sharpness, sg_color, colors_precomp,
                                             opacities, scales, rotations, cov3D_precomp, raster_settings, sh_rest)
        return rasterize_gaussians(means3D, means2D, shs, sg_axis, sg_sharpness, sg_color, colors_precomp,
                                   opacities, scales, rotations, cov3D_precomp, raster_settings)

    def _query_args(self, points3D, means3D, opacities, scales, rotations, cov3D_precomp, view2gaussian_precomp):
        """Argument checks and the 18-argument tuple of DGR/__init__.py:349-388
        (kernel size 0.0 as the reference, whatever the settings hold)."""
        s = self.raster_settings
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        if scales is None:
            scales = torch.Tensor([])
        if rotations is None:
            rotations = torch.Tensor([])
        if cov3D_precomp is None:
            cov3D_precomp = torch.Tensor([])
        if view2gaussian_precomp is None:
            view2gaussian_precomp = torch.Tensor([])
        return (points3D, means3D, opacities, scales, rotations, s.scale_modifier, cov3D_precomp,
                view2gaussian_precomp, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 0.0, s.image_height,
                s.image_width, s.campos, s.prefiltered, s.debug)

    def _query(self, fn, args):
        if self.raster_settings.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                return fn(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        return fn(*args)

    def integrate(self, points3D, means3D, opacities, scales=None, rotations=None, cov3D_precomp=None,
                  view2gaussian_precomp=None):
        """Opacity of the Gaussian field at world points seen from this camera
        (DGR/__init__.py:338-402): returns (1 - transmittance [PN], inside [PN])."""
        args = self._query_args(points3D, means3D, opacities, scales, rotations, cov3D_precomp,
                                view2gaussian_precomp)
        num_rendered, transmittance, inside = self._query(_C.integrate_gaussians_to_points, args)
        return 1 - transmittance, inside

    def evaluate_sdf(self, points3D, means3D, opacities, scales=None, rotations=None, cov3D_precomp=None,
                     view2gaussian_precomp=None):
        """Median depth along each point's ray and its signed distance to the
        point (DGR/__init__.py:404-468): returns (depth, sdf, inside), [PN] each."""
        args = self._query_args(points3D, means3D, opacities, scales, rotations, cov3D_precomp,
                                view2gaussian_precomp)
        num_rendered, depth, sdf, inside = self._query(_C.evaluate_sdf_from_signle_view, args)
        return depth, sdf, inside

    def sample_depth(self, points3D, means3D, opacities, scales=None, rotations=None, cov3D_precomp=None):
        """Median depth of the Gaussians at world points seen from this camera
        (DGR/__init__.py:470-483): returns (camera-space point at the median
        depth along its ray [..., 3], inside [...] bool)."""
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        if scales is None:
            scales = torch.Tensor([])
        if rotations is None:
            rotations = torch.Tensor([])
        if cov3D_precomp is None:
            cov3D_precomp = torch.Tensor([])
        return _SampleDepth.apply(points3D, means3D, opacities, scales, rotations, cov3D_precomp, self.raster_settings)


class _SampleDepth(torch.autograd.Function):
    """DGR/__init__.py:486-655.  The forward passes kernel_size 0.0 and the
    backward the settings' kernel_size, as the reference does (:500-518, 598)."""

    @staticmethod
    def forward(ctx, points3D, means3D, opacities, scales, rotations, cov3D_precomp, raster_settings):
        s = raster_settings
        args = (points3D, means3D, opacities, scales, rotations, s.scale_modifier, cov3D_precomp, s.viewmatrix,
                s.projmatrix, s.tanfovx, s.tanfovy, 0.0, s.image_height, s.image_width, s.campos, s.prefiltered,
                s.debug)
        if s.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.sample_rasterized_depth(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.sample_rasterized_depth(*args)
        (num_rendered, num_points, num_duplicated_tiles, camera_points, inside, geomBuffer, binningBuffer,
         pointBuffer, pointBinningBuffer, tileBuffer, duplicatedTileBuffer) = out
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.num_points = num_points
        ctx.num_duplicated_tiles = num_duplicated_tiles
        ctx.save_for_backward(points3D, means3D, opacities, scales, rotations, cov3D_precomp, inside, geomBuffer,
                              binningBuffer, pointBuffer, pointBinningBuffer, tileBuffer, duplicatedTileBuffer)
        # (no zero-filled gradient for the bool `inside`, nor for unused points: None reaches backward)
        ctx.set_materialize_grads(False)
        return camera_points, inside

    @staticmethod
    def backward(ctx, grad_camera_points, grad_inside):
        if grad_camera_points is None:
            return None, None, None, None, None, None, None
        s = ctx.raster_settings
        (points3D, means3D, opacities, scales, rotations, cov3D_precomp, inside, geomBuffer, binningBuffer,
         pointBuffer, pointBinningBuffer, tileBuffer, duplicatedTileBuffer) = ctx.saved_tensors
        args = (points3D, means3D, opacities, scales, rotations, s.scale_modifier, cov3D_precomp, s.viewmatrix,
                s.projmatrix, inside, grad_camera_points, s.tanfovx, s.tanfovy, s.kernel_size, s.image_height,
                s.image_width, s.campos, geomBuffer, binningBuffer, pointBuffer, pointBinningBuffer, tileBuffer,
                duplicatedTileBuffer, ctx.num_rendered, ctx.num_points, ctx.num_duplicated_tiles, s.prefiltered,
                s.debug)
        if s.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                grads = _C.sample_rasterized_depth_backward(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            grads = _C.sample_rasterized_depth_backward(*args)
        grad_opacities, grad_means3D, grad_cov3D_precomp, grad_scales, grad_rotations, grad_points3D = grads
        return grad_points3D, grad_means3D, grad_opacities, grad_scales, grad_rotations, grad_cov3D_precomp, None
