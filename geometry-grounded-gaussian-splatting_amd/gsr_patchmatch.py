"""PatchMatch.__call__ (utils/loss_utils.py:140-267) for the training step
with its torch body fused into the gsr_patchmatch_* kernels of libgsr.so
(csrc/ncc.hip): the lift of the view's median-depth points, sample_depth from
the nearest view (the package's GaussianRasterizer path, unchanged), and one
kernel for the reprojection, both masks, the weights, the NCC of the
normalised normals and the two masked means (plus a one-block finish).  The
reference's argwhere of the valid pixels — a host synchronisation in every
iteration — is gone: the NCC runs at the masked pixels of the full image.

Same values as gsr_train.patchmatch (the reference's torch formulation) up to
summation order; tests/test_gpu_train.py checks both losses and the gradients
they send into the median depth, the normals and the Gaussians.  There is no
CPU fallback.
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C as _G
from gaussian_renderer import sample_depth

PIXEL_NOISE_TH = 1.0  # arguments/__init__.py multi_view_pixel_noise_th


def _lib():
    L = _G._load()
    if not getattr(L, "_pm_bound", False):
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.gsr_patchmatch_lift.restype = i
        L.gsr_patchmatch_lift.argtypes = [i, i, f, f, f, f, vp, vp, vp, vp, vp]
        L.gsr_patchmatch_lift_backward.restype = i
        L.gsr_patchmatch_lift_backward.argtypes = [i, i, f, f, f, f, vp, vp, vp, vp]
        common = [i, i] + [vp] * 6 + [f] * 5 + [vp] * 4 + [f] * 8 + [i, i] + [vp] * 4
        L.gsr_patchmatch_terms_forward.restype = i
        L.gsr_patchmatch_terms_forward.argtypes = [_G._ALLOC, vp] + common + [vp, vp]
        L.gsr_patchmatch_terms_backward.restype = i
        L.gsr_patchmatch_terms_backward.argtypes = common + [vp] * 6
        L._pm_bound = True
    return L


def _check(L, rc):
    if rc != 0:
        raise RuntimeError("gsr: " + L.gsr_last_error().decode())


def _f32(t, name):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"gsr patchmatch: `{name}` must be a float32 HIP tensor")
    return t.contiguous()


class _Lift(torch.autograd.Function):
    """points [H, W, 3] = (median_depth * ray - T) @ M (loss_utils.py:147-153)."""

    @staticmethod
    def forward(ctx, md, T, M, intr):
        L = _lib()
        H, W = md.shape[-2:]
        md_c, T_c, M_c = _f32(md, "median_depth"), _f32(T, "T"), _f32(M, "M")
        pts = torch.empty(H, W, 3, dtype=torch.float32, device=md.device)
        with torch.cuda.device(md.device):
            _check(L, L.gsr_patchmatch_lift(H, W, *intr, T_c.data_ptr(), M_c.data_ptr(), md_c.data_ptr(),
                                            pts.data_ptr(), _G._stream(md.device)))
        ctx.save_for_backward(M_c)
        ctx.meta = (H, W, intr, md.shape)
        return pts

    @staticmethod
    def backward(ctx, g):
        L = _lib()
        (M_c,) = ctx.saved_tensors
        H, W, intr, shape = ctx.meta
        g = g.contiguous()
        dmd = torch.empty(shape, dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _check(L, L.gsr_patchmatch_lift_backward(H, W, *intr, M_c.data_ptr(), g.data_ptr(), dmd.data_ptr(),
                                                     _G._stream(g.device)))
        return dmd, None, None, None


class _Terms(torch.autograd.Function):
    """(geo_loss, ncc_loss) of PatchMatch from the sampled points."""

    @staticmethod
    def forward(ctx, md, normal, pin, inside, consts):
        L = _lib()
        H, W = md.shape[-2:]
        dev = md.device
        md_c, n_c, p_c = _f32(md, "median_depth"), _f32(normal, "normal"), _f32(pin, "points")
        ins = inside.contiguous()
        if (ins.dtype not in (torch.bool, torch.uint8) or ins.numel() != H * W or p_c.numel() != 3 * H * W
                or n_c.numel() != 3 * H * W):
            raise RuntimeError("gsr patchmatch: median_depth [.., H, W], normal [3, H, W], points [H, W, 3], "
                               "inside [H, W] bool expected")
        w = torch.empty(H * W, dtype=torch.float32, device=dev)
        flags = torch.empty(H * W, dtype=torch.uint8, device=dev)
        gd = torch.empty(H * W, dtype=torch.float32, device=dev)
        gn = torch.empty(H * W, 3, dtype=torch.float32, device=dev)
        out = torch.empty(4, dtype=torch.float32, device=dev)
        scratch = _G._ByteBuffer(dev)
        args = (H, W, md_c.data_ptr(), n_c.data_ptr(), p_c.data_ptr(), ins.data_ptr()) + consts.ptrs() + (
            w.data_ptr(), flags.data_ptr(), gd.data_ptr(), gn.data_ptr())
        with torch.cuda.device(dev):
            _check(L, L.gsr_patchmatch_terms_forward(scratch.cb, None, *args, out.data_ptr(), _G._stream(dev)))
        ctx.save_for_backward(md_c, n_c, p_c, ins, w, flags, gd, gn, out)
        ctx.consts = consts
        ctx.shapes = (md.shape, normal.shape, pin.shape)
        # (copies: `out` is saved for the backward, so the caller may change the returned losses in place)
        return out[0].clone(), out[1].clone()

    @staticmethod
    def backward(ctx, g_geo, g_ncc):
        L = _lib()
        md_c, n_c, p_c, ins, w, flags, gd, gn, out = ctx.saved_tensors
        H, W = md_c.shape[-2:]
        dev = md_c.device
        g = torch.stack([g_geo.reshape(()), g_ncc.reshape(())]).to(torch.float32).contiguous()
        dpin = torch.empty(ctx.shapes[2], dtype=torch.float32, device=dev)
        dmd = torch.empty(ctx.shapes[0], dtype=torch.float32, device=dev)
        dnormal = torch.empty(ctx.shapes[1], dtype=torch.float32, device=dev)
        args = (H, W, md_c.data_ptr(), n_c.data_ptr(), p_c.data_ptr(), ins.data_ptr()) + ctx.consts.ptrs() + (
            w.data_ptr(), flags.data_ptr(), gd.data_ptr(), gn.data_ptr())
        with torch.cuda.device(dev):
            _check(L, L.gsr_patchmatch_terms_backward(*args, out.data_ptr(), g.data_ptr(), dpin.data_ptr(),
                                                      dmd.data_ptr(), dnormal.data_ptr(), _G._stream(dev)))
        return dmd, dnormal, dpin, None, None


class _Consts:
    """The per-call constants of the terms kernels (device 3x3 / 3-vectors kept alive here)."""

    def __init__(self, view, nearest):
        with torch.no_grad():
            wv, wn = view.world_view_transform, nearest.world_view_transform
            self.tv = (-wv[:3, :3].T @ nearest.R @ nearest.T + wv[3, :3]).contiguous()  # loss_utils.py:155-158
            self.Mv = (nearest.R.transpose(1, 0) @ wv[:3, :3]).contiguous()
            r_rel = wn[:3, :3].transpose(-1, -2) @ wv[:3, :3]  # :232-235
            self.t_rel = (-r_rel @ wv[3, :3] + wn[3, :3]).contiguous()
            self.R_ncc = r_rel.T.contiguous()  # passed as warp_patch_ncc's R (:239)
        self.gray_r = _f32(view.gray_image.squeeze(), "view gray image")
        self.gray_n = _f32(nearest.gray_image.squeeze(), "nearest gray image")
        self.view, self.nearest = view, nearest

    def ptrs(self):
        v, n = self.view, self.nearest
        Hn, Wn = self.gray_n.shape
        return (self.Mv.data_ptr(), self.tv.data_ptr(), float(v.Fx), float(v.Fy), float(v.Cx), float(v.Cy),
                PIXEL_NOISE_TH, self.R_ncc.data_ptr(), self.t_rel.data_ptr(), self.gray_r.data_ptr(),
                self.gray_n.data_ptr(), float(v.Fx), float(v.Fy), float(v.Cx), float(v.Cy), float(n.Fx),
                float(n.Fy), float(n.Cx), float(n.Cy), int(Hn), int(Wn))


def patchmatch_fused(gaussians, render_pkg, view, nearest, kernel_size, pipe):
    """(ncc_loss, geo_loss) of PatchMatch.__call__ (utils/loss_utils.py:140-267)
    for `view` against `nearest`, as gsr_train.patchmatch, on the fused kernels.

    No nearest camera: the reference's two [1]-shaped zeros (loss_utils.py:141-142).
    An empty geometric or NCC mask gives 0-dim zeros where the reference returns
    [1]-shaped ones (loss_utils.py:223-224, 264-265): telling them apart would
    need the mask count on the host, i.e. a synchronisation per iteration; the
    value and its broadcast into the total loss are the same."""
    if nearest is None:
        z = lambda: torch.zeros(1, dtype=torch.float32, device=render_pkg["median_depth"].device)  # noqa: E731
        return z(), z()
    md = render_pkg["median_depth"]
    intr = (float(view.Fx), float(view.Fy), float(view.Cx), float(view.Cy))
    with torch.no_grad():
        M = view.R.T.contiguous()
    pts = _Lift.apply(md, view.T, M, intr)
    sampled = sample_depth(pts, nearest, gaussians, pipe, kernel_size)
    geo_loss, ncc_loss = _Terms.apply(md, render_pkg["normal"], sampled["sampled_depth"], sampled["inside"],
                                      _Consts(view, nearest))
    return ncc_loss, geo_loss
