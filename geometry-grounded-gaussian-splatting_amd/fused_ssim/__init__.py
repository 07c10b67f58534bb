"""MI355X drop-in for the external `fused_ssim` package the reference imports
(utils/loss_utils.py:18, `ssim()` at :48-49 calls fused_ssim(img1, img2,
padding="valid")): mean SSIM of img1 against img2 with the gradient w.r.t.
img1, computed by gsr_fused_ssim_{forward,backward} in libgsr.so
(csrc/ssim.hip).  The SSIM is that of the reference's own _ssim
(loss_utils.py:36-72).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C as _G

_ALLOC = _G._ALLOC


def _lib():
    L = _G._load()
    if not getattr(L, "_ssim_bound", False):
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.gsr_fused_ssim_forward.restype = i
        L.gsr_fused_ssim_forward.argtypes = [_ALLOC, vp, i, i, i, i, vp, vp, vp, vp, vp]
        L.gsr_fused_ssim_backward.restype = i
        L.gsr_fused_ssim_backward.argtypes = [i, i, i, i, vp, vp, vp, vp, vp, vp]
        L._ssim_bound = True
    return L


def _check(L, rc):
    if rc != 0:
        raise RuntimeError("gsr: " + L.gsr_last_error().decode())


def _planes(img, name):
    if not img.is_cuda or img.dtype != torch.float32:
        raise RuntimeError(f"fused_ssim: `{name}` must be a float32 HIP tensor")
    if img.dim() < 2:
        raise RuntimeError(f"fused_ssim: `{name}` must be [..., H, W]")
    H, W = img.shape[-2:]
    return img.contiguous(), img.numel() // (H * W), H, W


class _FusedSSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img1, img2, padding, train):
        L = _lib()
        a, NC, H, W = _planes(img1, "img1")
        b, NC2, H2, W2 = _planes(img2, "img2")
        if (NC, H, W) != (NC2, H2, W2):
            raise RuntimeError("fused_ssim: img1 and img2 must have the same shape")
        valid = {"same": 0, "valid": 1}[padding]
        out = torch.empty((), dtype=torch.float32, device=a.device)
        factors = torch.empty(3 * a.numel(), dtype=torch.float32, device=a.device) if train else None
        scratch = _G._ByteBuffer(a.device)
        with torch.cuda.device(a.device):
            _check(L, L.gsr_fused_ssim_forward(scratch.cb, None, NC, H, W, valid, a.data_ptr(), b.data_ptr(),
                                               out.data_ptr(), None if factors is None else factors.data_ptr(),
                                               _G._stream(a.device)))
        ctx.meta = (NC, H, W, valid, img1.shape)
        if train:
            ctx.save_for_backward(a, b, factors)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        L = _lib()
        NC, H, W, valid, shape = ctx.meta
        if not ctx.saved_tensors:
            raise RuntimeError("fused_ssim: called with train=False, no gradient available")
        a, b, factors = ctx.saved_tensors
        g = grad_out.contiguous().to(torch.float32).reshape(1)
        dimg1 = torch.empty_like(a)
        with torch.cuda.device(a.device):
            _check(L, L.gsr_fused_ssim_backward(NC, H, W, valid, a.data_ptr(), b.data_ptr(), factors.data_ptr(),
                                                g.data_ptr(), dimg1.data_ptr(), _G._stream(a.device)))
        return dimg1.reshape(shape), None, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    """Mean SSIM of img1 against img2 ([..., H, W] planes); differentiable in img1."""
    if padding not in ("same", "valid"):
        raise ValueError("padding must be 'same' or 'valid'")
    return _FusedSSIM.apply(img1, img2, padding, train)
