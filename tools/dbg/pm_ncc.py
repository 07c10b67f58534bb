"""Debug: where the fused NCC gradient differs from the torch one (development)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_train
from gsr_patchmatch import patchmatch_fused
from gaussian_renderer import render

step, view, nearest = gsr_train.synthetic_training_setup(20_000, 320, 240, device="cuda", seed=3)
g = step.g
pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
md = pkg["median_depth"].detach().requires_grad_(True)
nrm = pkg["normal"].detach().requires_grad_(True)
pkg = dict(pkg, median_depth=md, normal=nrm)
ref = gsr_train.patchmatch(g, pkg, view, nearest, step.kernel_size, step.pipe)[0]
got = patchmatch_fused(g, pkg, view, nearest, step.kernel_size, step.pipe)[0]
print("ncc", float(ref), float(got))
ga, gn_a = torch.autograd.grad(got, [md, nrm])
gb, gn_b = torch.autograd.grad(ref, [md, nrm])
d = (ga - gb).abs().view(-1)
print("md rel", float((ga - gb).norm() / gb.norm()), "nonzero a/b", int((ga != 0).sum()), int((gb != 0).sum()),
      "both", int(((ga != 0) & (gb != 0)).sum()))
order = torch.argsort(d, descending=True)[:8]
for i in order.tolist():
    print(i, divmod(i, view.image_width), float(ga.view(-1)[i]), float(gb.view(-1)[i]))
s = torch.sort(d, descending=True).values
tot = float((d ** 2).sum())
print("share of squared diff in top 1/10/100 px:", [round(float((s[:k] ** 2).sum()) / tot, 3) for k in (1, 10, 100)])
print("normal rel", float((gn_a - gn_b).norm() / gn_b.norm()))
