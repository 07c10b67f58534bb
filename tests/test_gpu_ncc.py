"""GPU tests of warp_patch_ncc (csrc/ncc.hip) against
the C oracle's restatement of warp_patch_ncc_impl.cu (itself pinned to a
float64 autograd restatement in tests/test_oracle.py).

Tolerances, over the points both call valid (valid flags equal except warps
within float noise of the image margin, <= 0.2%): the GPU's relative L2
error against the exact (float64 autograd) values is at most twice the
oracle's, i.e. the HIP kernel is as accurate as the reference's own fp32
arithmetic; and GPU vs oracle: NCC <= 1e-4, gradients <= 2e-3 relative L2.
The forward-mode gradient is a small difference of 49-term sums, so one-ulp
differences (v_rcp_f32 for the homogeneous divide, as the reference's fast
math) move it by ~1e-4 relative.
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

import helpers as Hh
from oracle import gsr_oracle as O
import torch_ref as R_
from test_oracle import ncc_case

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("P,seed,size", [(1, 0, (48, 40, 52, 44)), (500, 1, (48, 40, 52, 44)),
                                         (20000, 2, (320, 240, 300, 250))])
def test_ncc_parity(P, seed, size):
    import warp_patch_ncc as W

    d, n, uv, R, T, ir, inn, K = ncc_case(P, seed, *size)
    o = O.warp_patch_ncc(d, n, uv, R, T, ir, inn, *K.values())
    ncc, gd, gn, valid = W._C.warp_patch_ncc(d.to(DEV), n.to(DEV), uv.to(DEV), R.reshape(3, 3).to(DEV), T.to(DEV),
                                             ir.to(DEV), inn.to(DEV), *K.values(), False)
    v = valid.cpu().numpy()
    assert (v != o["valid"]).mean() <= 2e-3  # warps landing within float noise of the image margin
    both = v & o["valid"]
    if P > 10:
        assert both.sum() > 0.3 * P
    # exact values: the float64 autograd restatement (tests/torch_ref.py)
    dd = d.double().clone().requires_grad_(True)
    nd = n.double().clone().requires_grad_(True)
    x_ncc, _ = R_.warp_patch_ncc(dd, nd, uv, R, T, ir, inn, *K.values())
    x_ncc.sum().backward()
    exact = {"ncc": x_ncc.detach().numpy(), "grad_depths": dd.grad.numpy(), "grad_normals": nd.grad.numpy()}

    def l2(a, b):
        a, b = np.asarray(a, np.float64)[both], np.asarray(b, np.float64)[both]
        return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)

    for name, mine in (("ncc", ncc), ("grad_depths", gd), ("grad_normals", gn)):
        m = mine.cpu().numpy()
        e_gpu, e_oracle = l2(m, exact[name]), l2(o[name], exact[name])
        # as accurate as the reference's own fp32 arithmetic (the oracle) ...
        assert e_gpu <= max(2.0 * e_oracle, 1e-5), (name, e_gpu, e_oracle)
        # ... and close to it
        assert l2(m, o[name]) <= (1e-4 if name == "ncc" else 2e-3), (name, l2(m, o[name]))
    assert float(ncc[~valid].abs().sum()) == 0 and float(gn[~valid].abs().sum()) == 0


def test_ncc_autograd_routing():
    """_WarpPatchNCC.backward scales the saved forward-mode gradients by the
    upstream gradient (warp_patch_ncc/__init__.py:71-74)."""
    import warp_patch_ncc as W

    d, n, uv, R, T, ir, inn, K = ncc_case(300, 3)
    dd = d.to(DEV).requires_grad_(True)
    nd = n.to(DEV).requires_grad_(True)
    ncc, valid = W.warp_patch_ncc(dd, nd, uv.to(DEV), R.reshape(3, 3).to(DEV), T.to(DEV), ir.to(DEV), inn.to(DEV),
                                  *K.values(), False)
    g = torch.rand(300, device=DEV)
    (ncc * g).sum().backward()
    _, gd, gn, _ = W._C.warp_patch_ncc(d.to(DEV), n.to(DEV), uv.to(DEV), R.reshape(3, 3).to(DEV), T.to(DEV),
                                       ir.to(DEV), inn.to(DEV), *K.values(), False)
    assert torch.equal(dd.grad, g * gd) and torch.equal(nd.grad, g[:, None] * gn)
