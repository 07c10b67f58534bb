"""GPU tests of depth_to_normal (csrc/depth_normal.hip)
against the float64 restatement of utils/graphics_utils.py:103-119
(oracle/ssim_ref.py), forward and autograd backward.

Tolerances: valid exact; normals (max abs) and dL/ddepth (relative L2): the
error against the float64 values is at most twice that of the reference's own
fp32 torch arithmetic (or 1e-5) — the central differences of back-projected
fp32 points cancel at 1080p.
"""
from __future__ import annotations

import pytest
import torch

from oracle import ssim_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class View:
    def __init__(self, W, H):
        self.image_width, self.image_height = W, H
        self.Fx, self.Fy, self.Cx, self.Cy = 0.9 * W, 0.9 * W, W / 2 - 0.5, H / 2 + 0.25


@pytest.mark.parametrize("W,H", [(40, 30), (1920, 1080)])
def test_depth_to_normal_matches_reference(W, H):
    import gsr_geometry as G

    g = torch.Generator().manual_seed(0)
    base = torch.rand(1, 1, H // 8 + 2, W // 8 + 2, generator=g) * 3 + 2
    depth = torch.nn.functional.interpolate(base, size=(H, W), mode="bicubic", align_corners=True)[0]
    depth[:, : H // 7, : W // 5] = 0.0  # holes (median depth 0 where undefined)
    depth = depth.float().contiguous()
    view = View(W, H)
    d = depth.to(DEV).requires_grad_(True)
    n, valid = G.depth_to_normal(view, d)
    # the depth-normal loss masks by `valid` (train.py:174-180); unmasked, the
    # degenerate cross products at hole edges take F.normalize's 1/eps branch
    gn = torch.randn(3, H, W, generator=g) * valid.cpu()
    (n * gn.to(DEV)).sum().backward()
    d64 = depth.double().requires_grad_(True)
    rn, rvalid = ssim_ref.depth_to_normal(d64, view.Fx, view.Fy, view.Cx, view.Cy)
    (rn * gn.double()).sum().backward()
    # the reference's own arithmetic is fp32 torch: the same formula in fp32
    d32 = depth.clone().requires_grad_(True)
    fn, _ = ssim_ref.depth_to_normal(d32, view.Fx, view.Fy, view.Cx, view.Cy)
    (fn * gn).sum().backward()
    assert torch.equal(valid.cpu(), rvalid)
    e_gpu = float((n.detach().cpu().double() - rn.detach()).abs().max())
    e_f32 = float((fn.detach().double() - rn.detach()).abs().max())
    assert e_gpu <= max(2 * e_f32, 1e-5), (e_gpu, e_f32)  # central differences of fp32 points cancel
    err = float((d.grad.cpu().double() - d64.grad).norm() / d64.grad.norm())
    err32 = float((d32.grad.double() - d64.grad).norm() / d64.grad.norm())
    assert err <= max(2 * err32, 1e-5), (err, err32)


@pytest.mark.parametrize("i", [0, 1])
def test_depth_to_normal_matches_reference_fixture(i):
    """Against utils/graphics_utils.py:103-119 run by the reference itself
    (fp32 torch, tests/golden/make_golden.py): valid exact, normals within
    1e-5, the gradient of <normal, upstream> within 1e-5 relative L2."""
    import os

    import numpy as np

    import gsr_geometry as G

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "losses.npz"))
    W, H, Fx, Fy, Cx, Cy = d[f"dn_view_{i}"]
    view = View(int(W), int(H))
    view.Fx, view.Fy, view.Cx, view.Cy = float(Fx), float(Fy), float(Cx), float(Cy)
    depth = torch.tensor(d[f"dn_depth_{i}"], device=DEV).requires_grad_(True)
    n, valid = G.depth_to_normal(view, depth)
    (n * torch.tensor(d[f"dn_upstream_{i}"], device=DEV)).sum().backward()
    assert np.array_equal(valid.cpu().numpy(), d[f"dn_valid_{i}"])
    assert np.abs(n.detach().cpu().numpy() - d[f"dn_normal_{i}"]).max() <= 1e-5
    g = d[f"dn_grad_{i}"].astype(np.float64)
    assert np.linalg.norm(depth.grad.cpu().double().numpy() - g) / np.linalg.norm(g) <= 1e-5
