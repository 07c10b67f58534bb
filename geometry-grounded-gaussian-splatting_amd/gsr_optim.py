"""Training update on gfx950.

FusedAdam — a drop-in for the `torch.optim.Adam(param_groups, lr=0.0,
eps=1e-15)` of GaussianModel.training_setup (scene/gaussian_model.py:342-351):
same constructor, `param_groups` (the reference's per-group "name"/"lr"
entries and its learning-rate schedule keep working) and per-parameter state
layout (`step`, `exp_avg`, `exp_avg_sq`, which densification edits in place,
gaussian_model.py cat/prune helpers), but `step()` is one HIP launch over all
parameters (libgsr.so gsr_adam_step, csrc/optim.hip) instead of a dozen
foreach kernels.

add_densification_stats — GaussianModel.add_densification_stats plus the
max_radii2D update (gaussian_model.py:818-821, train.py:236-237) as one
kernel (gsr_densify_stats).

scaling_n_opacity_with_3D_filter / normalize_rows — the activation getters
get_scaling_n_opacity_with_3D_filter and get_rotation
(gaussian_model.py:146-212) as autograd functions over one kernel each way
(gsr_scale_opacity_3d_filter*, gsr_normalize_rows*).
"""
from __future__ import annotations

import ctypes

import torch

from diff_gaussian_rasterization import _C


def _lib():
    L = _C._load()
    if not getattr(L, "_getters_bound", False):
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.gsr_scale_opacity_3d_filter.restype = i
        L.gsr_scale_opacity_3d_filter.argtypes = [i] + [vp] * 6
        L.gsr_scale_opacity_3d_filter_backward.restype = i
        L.gsr_scale_opacity_3d_filter_backward.argtypes = [i] + [vp] * 8
        L.gsr_normalize_rows.restype = i
        L.gsr_normalize_rows.argtypes = [i, i, vp, vp, vp]
        L.gsr_normalize_rows_backward.restype = i
        L.gsr_normalize_rows_backward.argtypes = [i, i, vp, vp, vp, vp]
        L._getters_bound = True
    return L


def _rc(L, rc):
    if rc != 0:
        raise RuntimeError("gsr: " + L.gsr_last_error().decode())


def _dev32(t, name):
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"gsr getters: `{name}` must be a float32 HIP tensor")
    return t.contiguous()


class _ScaleOpacity(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scaling, opacity, filter_3D):
        L = _lib()
        s, o, f = _dev32(scaling, "scaling"), _dev32(opacity, "opacity"), _dev32(filter_3D, "filter_3D")
        P = s.shape[0]
        if s.shape != (P, 3) or o.numel() != P or f.numel() != P:
            raise RuntimeError("gsr getters: scaling [P,3], opacity [P,1], filter_3D [P,1] expected")
        scales = torch.empty_like(s)
        op = torch.empty_like(o)
        with torch.cuda.device(s.device):
            _rc(L, L.gsr_scale_opacity_3d_filter(P, s.data_ptr(), o.data_ptr(), f.data_ptr(), scales.data_ptr(),
                                                 op.data_ptr(), _C._stream(s.device)))
        ctx.save_for_backward(s, o, f)
        ctx.set_materialize_grads(False)  # (a caller of one getter leaves the other output's gradient None)
        return scales, op

    @staticmethod
    def backward(ctx, g_scales, g_op):
        if g_scales is None and g_op is None:
            return None, None, None
        L = _lib()
        s, o, f = ctx.saved_tensors
        ds, do = torch.empty_like(s), torch.empty_like(o)
        gs = None if g_scales is None else g_scales.contiguous()
        go = None if g_op is None else g_op.contiguous()
        with torch.cuda.device(s.device):
            _rc(L, L.gsr_scale_opacity_3d_filter_backward(
                s.shape[0], s.data_ptr(), o.data_ptr(), f.data_ptr(), None if gs is None else gs.data_ptr(),
                None if go is None else go.data_ptr(), ds.data_ptr(), do.data_ptr(), _C._stream(s.device)))
        return ds, do, None


def scaling_n_opacity_with_3D_filter(scaling, opacity, filter_3D):
    """(sqrt(exp(s)^2 + f^2), sigmoid(o) sqrt(prod exp(s)^2 / prod(exp(s)^2 + f^2)))
    of gaussian_model.py's get_scaling_n_opacity_with_3D_filter, one kernel."""
    return _ScaleOpacity.apply(scaling, opacity, filter_3D)


class _NormalizeRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        L = _lib()
        xc = _dev32(x, "x")
        y = torch.empty_like(xc)
        n, D = xc.shape[0], xc[0].numel() if xc.shape[0] else 1
        with torch.cuda.device(xc.device):
            _rc(L, L.gsr_normalize_rows(n, D, xc.data_ptr(), y.data_ptr(), _C._stream(xc.device)))
        ctx.save_for_backward(xc)
        return y

    @staticmethod
    def backward(ctx, g):
        L = _lib()
        (xc,) = ctx.saved_tensors
        gc = g.contiguous()
        dx = torch.empty_like(xc)
        n, D = xc.shape[0], xc[0].numel() if xc.shape[0] else 1
        with torch.cuda.device(xc.device):
            _rc(L, L.gsr_normalize_rows_backward(n, D, xc.data_ptr(), gc.data_ptr(), dx.data_ptr(),
                                                 _C._stream(xc.device)))
        return dx


def normalize_rows(x):
    """F.normalize(x) over dim 1 for x [n, D] (get_rotation), one kernel."""
    return _NormalizeRows.apply(x)


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (no weight decay, no amsgrad) with a fused HIP step."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches = {}  # (betas, eps, step) -> [(tensors, lr)]
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                key = (beta1, beta2, group["eps"], float(st["step"]))
                batches.setdefault(key, []).append(((p, p.grad, st["exp_avg"], st["exp_avg_sq"]), group["lr"]))
        for (beta1, beta2, eps, step), items in batches.items():
            for k in range(0, len(items), _C.MAX_ADAM_GROUPS):
                chunk = items[k:k + _C.MAX_ADAM_GROUPS]
                _C.adam_step([t for t, _ in chunk], [lr for _, lr in chunk], step, beta1, beta2, eps)
        return loss


def add_densification_stats(gaussians, viewspace_point_tensor, radii):
    """The reference's two densification-statistics statements of a training
    iteration (train.py:236-237) for `gaussians` exposing max_radii2D [P],
    xyz_gradient_accum [P,1], xyz_gradient_accum_abs [P,1] and denom [P,1]."""
    _C.densify_stats(viewspace_point_tensor.grad, radii, gaussians.max_radii2D, gaussians.xyz_gradient_accum,
                     gaussians.xyz_gradient_accum_abs, gaussians.denom)
