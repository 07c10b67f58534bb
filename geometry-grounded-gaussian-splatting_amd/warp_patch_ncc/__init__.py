"""MI355X drop-in for the reference's `warp_patch_ncc` extension
(submodules/warp-patch-ncc/warp_patch_ncc/__init__.py): same WarpParams,
warp_patch_ncc() and _WarpPatchNCC (forward-mode gradients saved by the
forward, scaled by the upstream gradient in the backward).  The compute is
gsr_warp_patch_ncc in libgsr.so (csrc/ncc.hip); there is no CPU fallback.
"""
from __future__ import annotations

from typing import NamedTuple

import torch

from . import _C


class WarpParams(NamedTuple):
    R: torch.Tensor
    T: torch.Tensor
    fx_r: float
    fy_r: float
    cx_r: float
    cy_r: float
    fx_n: float
    fy_n: float
    cx_n: float
    cy_n: float
    debug: bool


def warp_patch_ncc(depths, normals, uvs, R, T, image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n,
                   debug):
    """NCC of the 7x7 half-step patch at each pixel `uvs` of the reference view
    against its homography warp (depth, normal, relative pose R, T) into the
    neighbouring view; returns (ncc [P], valid [P] bool)."""
    params = WarpParams(R.contiguous(), T.contiguous(), fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n, debug)
    return _WarpPatchNCC.apply(depths, normals, uvs, image_r, image_n, params)


class _WarpPatchNCC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, depths, normals, uvs, image_r, image_n, params):
        ncc, grad_depths, grad_normals, valid = _C.warp_patch_ncc(
            depths, normals, uvs, params.R, params.T, image_r, image_n, params.fx_r, params.fy_r, params.cx_r,
            params.cy_r, params.fx_n, params.fy_n, params.cx_n, params.cy_n, params.debug)
        ctx.save_for_backward(grad_depths, grad_normals)
        return ncc, valid

    @staticmethod
    def backward(ctx, grad_ncc, grad_valid):
        grad_depths, grad_normals = ctx.saved_tensors
        return grad_ncc * grad_depths, grad_ncc.unsqueeze(-1) * grad_normals, None, None, None, None
