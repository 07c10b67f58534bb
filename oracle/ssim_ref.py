"""TEST INFRASTRUCTURE ONLY — float64 torch restatements of the reference's
SSIM (utils/loss_utils.py:36-72: gaussian(11, 1.5) window, _ssim with
C1 = 0.01^2, C2 = 0.03^2, conv2d with zero padding 5), the checker of the
fused SSIM kernel (csrc/ssim.hip).  "valid" padding (the mode loss_utils.ssim
requests from fused_ssim, :49) crops the map by 5 on each side before the
mean.  Gradients come from autograd."""
from __future__ import annotations

from math import exp

import torch
import torch.nn.functional as F


def window(window_size=11, sigma=1.5, dtype=torch.float64):
    g = torch.tensor([exp(-((x - window_size // 2) ** 2) / float(2 * sigma ** 2)) for x in range(window_size)],
                     dtype=torch.float32)
    g = (g / g.sum()).to(dtype)  # normalised in fp32 as loss_utils.py:38
    return g[:, None] @ g[None, :]


def ssim(img1, img2, padding="same", window_size=11):
    """Mean SSIM of [N, C, H, W] images (float64)."""
    C = img1.shape[1]
    w = window(window_size, dtype=img1.dtype).to(img1.device).expand(C, 1, window_size, window_size).contiguous()
    p = window_size // 2
    mu1 = F.conv2d(img1, w, padding=p, groups=C)
    mu2 = F.conv2d(img2, w, padding=p, groups=C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, w, padding=p, groups=C) - mu1_sq
    s2 = F.conv2d(img2 * img2, w, padding=p, groups=C) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=p, groups=C) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    if padding == "valid":
        m = m[:, :, p:-p, p:-p]
    return m.mean()


def depth_to_normal(depth, Fx, Fy, Cx, Cy):
    """float64 restatement of utils/graphics_utils.py:103-119 for a depth
    [1,H,W]: back-projected points, central differences, normalize(dy x dx)
    (eps 1e-12), zero border; valid = depth > 0 at the five taps."""
    _, H, W = depth.shape
    x = (torch.arange(W, dtype=torch.float32) - Cx) / Fx  # fp32 as the reference's arange
    y = (torch.arange(H, dtype=torch.float32) - Cy) / Fy
    x, y = x.to(depth.dtype), y.to(depth.dtype)
    pts = torch.cat([depth * x[None, None], depth * y[None, :, None], depth], dim=0)
    dy = pts[:, 2:, 1:-1] - pts[:, :-2, 1:-1]
    dx = pts[:, 1:-1, 2:] - pts[:, 1:-1, :-2]
    n = F.normalize(torch.cross(dy, dx, dim=0), dim=0)
    out = F.pad(n, (1, 1, 1, 1))
    v = depth > 0
    vi = v[:, 2:, 1:-1] & v[:, :-2, 1:-1] & v[:, 1:-1, 2:] & v[:, 1:-1, :-2] & v[:, 1:-1, 1:-1]
    valid = torch.zeros_like(depth, dtype=torch.bool)
    valid[:, 1:-1, 1:-1] = vi
    return out, valid
