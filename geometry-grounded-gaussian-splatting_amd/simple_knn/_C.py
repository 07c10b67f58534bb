"""simple_knn._C.distCUDA2 over the C ABI (gsr_knn_mean_dist, include/gsr.h).

distCUDA2(points [P, 3] float32 HIP tensor) -> [P] float32: per point the
mean of the squared distances to its 3 nearest other points
(submodules/simple-knn/spatial.cu:15-25, simple_knn.cu:175-220).
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C as _G


def _lib():
    L = _G._load()
    if not getattr(L, "_knn_bound", False):
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.gsr_knn_mean_dist.restype = i
        L.gsr_knn_mean_dist.argtypes = [_G._ALLOC, vp, i, vp, vp, vp]
        L._knn_bound = True
    return L


def distCUDA2(points):
    if not isinstance(points, torch.Tensor) or not points.is_cuda:
        raise RuntimeError("distCUDA2: `points` must be a HIP device tensor")
    if points.dtype != torch.float32:
        raise RuntimeError("distCUDA2: `points` must be float32")
    if points.ndimension() != 2 or points.size(1) != 3:
        raise RuntimeError("distCUDA2: `points` must have shape (P, 3)")
    L = _lib()
    P = points.size(0)
    pts = points.contiguous()
    means = torch.zeros(P, dtype=torch.float32, device=points.device)  # torch::full({P}, 0.0), spatial.cu:21
    if P:
        scratch = _G._ByteBuffer(points.device)
        with torch.cuda.device(points.device):
            rc = L.gsr_knn_mean_dist(scratch.cb, None, P, ctypes.c_void_p(pts.data_ptr()),
                                     ctypes.c_void_p(means.data_ptr()), _G._stream(points.device))
        if rc != 0:
            raise RuntimeError("gsr: " + L.gsr_last_error().decode())
    return means
