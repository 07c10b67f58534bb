"""GPU tests of the fused SSIM (csrc/ssim.hip) against
the float64 restatement of the reference's SSIM (oracle/ssim_ref.py,
utils/loss_utils.py:36-72), in both paddings, with the gradient w.r.t. img1.

Tolerances: |mean_gpu - mean_ref| <= 1e-6; gradient ||a-b|| / ||b|| <= 1e-5
(fp32 separable window sums against float64 conv2d).
"""
from __future__ import annotations

import pytest
import torch

from oracle import ssim_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pair(shape, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.rand(shape, generator=g)
    b = (a + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)  # correlated, like a render and its target
    return a, b


@pytest.mark.parametrize("shape,padding", [((1, 3, 64, 80), "valid"), ((1, 3, 64, 80), "same"),
                                           ((1, 3, 37, 53), "valid"), ((2, 1, 17, 11), "valid"),
                                           ((1, 3, 1080, 1920), "valid")])
def test_fused_ssim_matches_reference(shape, padding):
    import fused_ssim as FS

    a, b = _pair(shape, 0)
    x = a.to(DEV).requires_grad_(True)
    v = FS.fused_ssim(x, b.to(DEV), padding=padding)
    v.backward()
    a64 = a.double().requires_grad_(True)
    r = ssim_ref.ssim(a64, b.double(), padding=padding)
    r.backward()
    assert abs(float(v) - float(r)) <= 1e-6, (float(v), float(r))
    gr = a64.grad
    err = float((x.grad.cpu().double() - gr).norm() / gr.norm())
    assert err <= 1e-5, err


@pytest.mark.parametrize("i", [0, 1, 2])
@pytest.mark.parametrize("padding", ["same", "valid"])
def test_fused_ssim_matches_reference_fixture(i, padding):
    """Against the reference's own _ssim (utils/loss_utils.py:36-72, run in
    fp32 torch by tests/golden/make_golden.py): mean within 1e-6, dSSIM/dimg1
    within 1e-5 relative L2."""
    import os

    import numpy as np

    import fused_ssim as FS

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "losses.npz"))
    x = torch.tensor(d[f"ssim_img1_{i}"], device=DEV).requires_grad_(True)
    v = FS.fused_ssim(x, torch.tensor(d[f"ssim_img2_{i}"], device=DEV), padding=padding)
    v.backward()
    want, g = float(d[f"ssim_{padding}_{i}"]), d[f"ssim_{padding}_grad_{i}"].astype(np.float64)
    assert abs(v.item() - want) <= 1e-6, (v.item(), want)
    assert np.linalg.norm(x.grad.cpu().double().numpy() - g) / np.linalg.norm(g) <= 1e-5


def test_fused_ssim_loss_term_and_no_grad():
    """1 - ssim(...) as train.py:189 uses it; train=False gives the value only."""
    import fused_ssim as FS

    a, b = _pair((1, 3, 48, 48), 1)
    x = a.to(DEV).requires_grad_(True)
    loss = 0.2 * (1.0 - FS.fused_ssim(x.unsqueeze(0)[0], b.to(DEV), padding="valid"))
    loss.backward()
    a64 = a.double().requires_grad_(True)
    (0.2 * (1.0 - ssim_ref.ssim(a64, b.double(), padding="valid"))).backward()
    assert float((x.grad.cpu().double() - a64.grad).norm() / a64.grad.norm()) <= 1e-5
    with torch.no_grad():
        v = FS.fused_ssim(a.to(DEV), b.to(DEV), padding="valid", train=False)
    assert abs(float(v) - float(ssim_ref.ssim(a.double(), b.double(), padding="valid"))) <= 1e-6
    same = FS.fused_ssim(b.to(DEV), b.to(DEV), padding="valid", train=False)
    assert abs(float(same) - 1.0) <= 1e-6
