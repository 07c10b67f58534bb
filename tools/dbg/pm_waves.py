"""Debug: how full the dense NCC's waves are (d_mask density per 64-pixel wave) at the e2e scene."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_train
from gaussian_renderer import render

step, view, nearest = gsr_train.synthetic_training_setup(1_000_000, 1920, 1080, device="cuda")
g = step.g
pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
t = gsr_train.patchmatch_terms(g, pkg, view, nearest, step.kernel_size, step.pipe)
m = t["d_mask"].reshape(-1)
n = m.numel() // 64 * 64
c = m[:n].view(-1, 64).sum(1)
tot = c.numel()
print("pixels", m.numel(), "d_mask", int(m.sum()), "ncc_mask", int(t["ncc_mask"].sum()))
print("waves", tot, "empty", int((c == 0).sum()), "full", int((c == 64).sum()), "partial", int(((c > 0) & (c < 64)).sum()))
print("lane efficiency of non-empty waves", float(c[c > 0].float().mean() / 64))
