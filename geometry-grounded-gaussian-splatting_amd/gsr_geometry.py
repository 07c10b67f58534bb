"""depth_to_normal on gfx950: drop-in for the reference's
utils/graphics_utils.py:103-119 (called at train.py:174) with the same
signature and outputs — (normal [3,H,W], valid [1,H,W] bool) — computed by
gsr_depth_to_normal_{forward,backward} (csrc/depth_normal.hip), differentiable
in depth.  `view` needs image_width, image_height, Fx, Fy, Cx, Cy."""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C as _G


def _lib():
    L = _G._load()
    if not getattr(L, "_dn_bound", False):
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.gsr_depth_to_normal_forward.restype = i
        L.gsr_depth_to_normal_forward.argtypes = [vp, i, i, f, f, f, f, vp, vp, vp]
        L.gsr_depth_to_normal_backward.restype = i
        L.gsr_depth_to_normal_backward.argtypes = [vp, i, i, f, f, f, f, vp, vp, vp]
        L._dn_bound = True
    return L


def _check(L, rc):
    if rc != 0:
        raise RuntimeError("gsr: " + L.gsr_last_error().decode())


class _DepthToNormal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, depth, H, W, Fx, Fy, Cx, Cy):
        if not depth.is_cuda or depth.dtype != torch.float32:
            raise RuntimeError("depth_to_normal: depth must be a float32 HIP tensor")
        d = depth.contiguous()
        L = _lib()
        normal = torch.empty(3, H, W, dtype=torch.float32, device=d.device)
        valid = torch.empty(1, H, W, dtype=torch.bool, device=d.device)
        with torch.cuda.device(d.device):
            _check(L, L.gsr_depth_to_normal_forward(d.data_ptr(), H, W, Fx, Fy, Cx, Cy, normal.data_ptr(),
                                                    valid.data_ptr(), _G._stream(d.device)))
        ctx.save_for_backward(d)
        ctx.cam = (H, W, Fx, Fy, Cx, Cy)
        ctx.mark_non_differentiable(valid)
        ctx.set_materialize_grads(False)  # (no zero-filled gradient for `valid`)
        return normal, valid

    @staticmethod
    def backward(ctx, g_normal, g_valid):
        if g_normal is None:
            return None, None, None, None, None, None, None
        (d,) = ctx.saved_tensors
        H, W, Fx, Fy, Cx, Cy = ctx.cam
        L = _lib()
        g = g_normal.contiguous()
        dd = torch.empty_like(d)
        with torch.cuda.device(d.device):
            _check(L, L.gsr_depth_to_normal_backward(d.data_ptr(), H, W, Fx, Fy, Cx, Cy, g.data_ptr(), dd.data_ptr(),
                                                     _G._stream(d.device)))
        return dd, None, None, None, None, None, None


def depth_to_normal(view, depth):
    """Normal map of `depth` [1,H,W] seen by `view` and the mask of pixels
    whose five taps have depth > 0 (utils/graphics_utils.py:103-119)."""
    W, H = int(view.image_width), int(view.image_height)
    if depth.shape[-2:] != (H, W):
        raise RuntimeError("depth_to_normal: depth must be [1, H, W] of the view")
    return _DepthToNormal.apply(depth, H, W, float(view.Fx), float(view.Fy), float(view.Cx), float(view.Cy))
