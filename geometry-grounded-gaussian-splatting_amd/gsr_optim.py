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
"""
from __future__ import annotations

import torch

from diff_gaussian_rasterization import _C


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
