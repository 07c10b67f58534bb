"""`warp_patch_ncc._C` — the reference extension's one entry point
(submodules/warp-patch-ncc/ext.cpp, warp_patch_ncc.cu:5-52), bound to
gsr_warp_patch_ncc in libgsr.so (the library of diff_gaussian_rasterization)."""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C as _G


def _lib():
    L = _G._load()
    if not getattr(L, "_ncc_bound", False):
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.gsr_warp_patch_ncc.restype = i
        L.gsr_warp_patch_ncc.argtypes = [i] + [vp] * 7 + [f] * 8 + [i] * 4 + [vp] * 4 + [vp]
        L._ncc_bound = True
    return L


def warp_patch_ncc(depths, normals, uvs, R, T, image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n,
                   debug):
    if normals.ndimension() != 2 or normals.size(1) != 3:
        raise RuntimeError("normals must have dimensions (num_points, 3)")
    L = _lib()
    P = depths.size(0)
    dev = depths.device
    fopt = dict(dtype=torch.float32, device=dev)
    ncc = torch.empty(P, **fopt)
    # contiguous, whatever the strides of `depths`: the kernel writes P floats in order
    grad_depths = torch.empty(depths.shape, **fopt)
    grad_normals = torch.empty(P, 3, **fopt)
    valid = torch.empty(P, dtype=torch.bool, device=dev)
    if P == 0:
        return ncc, grad_depths, grad_normals, valid
    args = {}
    for name, t in (("depths", depths), ("normals", normals), ("R", R), ("T", T), ("image_r", image_r),
                    ("image_n", image_n)):
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError(f"gsr warp_patch_ncc: `{name}` must be a float32 HIP tensor")
        args[name] = t.contiguous()
    if not uvs.is_cuda or uvs.dtype != torch.int32:
        raise RuntimeError("gsr warp_patch_ncc: `uvs` must be an int32 HIP tensor")
    if R.numel() != 9 or T.numel() != 3 or uvs.numel() != 2 * P or image_r.dim() != 2 or image_n.dim() != 2:
        raise RuntimeError("gsr warp_patch_ncc: R [3,3], T [3], uvs [P,2], images [H,W] expected")
    u = uvs.contiguous()
    Hr, Wr = image_r.shape
    Hn, Wn = image_n.shape
    with torch.cuda.device(dev):
        rc = L.gsr_warp_patch_ncc(
            P, args["depths"].data_ptr(), args["normals"].data_ptr(), u.data_ptr(), args["R"].data_ptr(),
            args["T"].data_ptr(), args["image_r"].data_ptr(), args["image_n"].data_ptr(), float(fx_r), float(fy_r),
            float(cx_r), float(cy_r), float(fx_n), float(fy_n), float(cx_n), float(cy_n), int(Hr), int(Wr), int(Hn),
            int(Wn), ncc.data_ptr(), grad_depths.data_ptr(), grad_normals.data_ptr(), valid.data_ptr(),
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    if rc != 0:
        raise RuntimeError("gsr: " + L.gsr_last_error().decode())
    if debug:
        torch.cuda.synchronize(dev)
    return ncc, grad_depths, grad_normals, valid
