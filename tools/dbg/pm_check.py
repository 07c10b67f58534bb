"""Debug: fused PatchMatch pieces against the torch formulation (development)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_train
import gsr_patchmatch as PM
from gaussian_renderer import render, sample_depth

step, view, nearest = gsr_train.synthetic_training_setup(20_000, 320, 240, device="cuda", seed=3)
g = step.g
pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
md = pkg["median_depth"].detach().requires_grad_(True)
rays, pixels, pixels_f = gsr_train._pixel_grids(view, md.device)
pts_t = gsr_train._mat3(md.squeeze().unsqueeze(-1) * rays - view.T, view.R.T)
intr = (float(view.Fx), float(view.Fy), float(view.Cx), float(view.Cy))
pts_f = PM._Lift.apply(md, view.T, view.R.T.contiguous(), intr)
print("lift max diff", float((pts_t - pts_f).abs().max()), float(pts_t.abs().max()))
gg = torch.randn_like(pts_t)
(a,) = torch.autograd.grad(pts_t, md, gg)
(b,) = torch.autograd.grad(pts_f, md, gg)
print("lift grad rel", float((a - b).norm() / a.norm()))
# terms with a fixed pin
s = sample_depth(pts_t.detach(), nearest, g, step.pipe, step.kernel_size)
pin = s["sampled_depth"].detach().requires_grad_(True)
inside = s["inside"]
with torch.no_grad():
    v2n_T = -view.world_view_transform[:3, :3].T @ nearest.R @ nearest.T + view.world_view_transform[3, :3]
    n2v_R = nearest.R.transpose(1, 0) @ view.world_view_transform[:3, :3]
piv = v2n_T + gsr_train._mat3(pin, n2v_R)
proj = piv[..., :2] / torch.clamp_min(piv[..., 2:], 1e-7)
proj = torch.addcmul(proj.new_tensor([view.Cx, view.Cy]), proj.new_tensor([view.Fx, view.Fy]), proj)
noise = torch.pairwise_distance(proj, pixels_f)
with torch.no_grad():
    dm = inside & (pin[..., -1] > 0.2) & (piv[..., -1] > 0.2) & (noise < 1.0) & (md.squeeze() > 0)
    w = torch.exp(-noise).masked_fill_(~dm, 0.0)
geo_t = gsr_train.masked_mean(w * noise, dm, empty=0.0)
geo_f, ncc_f = PM._Terms.apply(md, pkg["normal"].detach(), pin, inside, PM._Consts(view, nearest))
print("geo", float(geo_t), float(geo_f), "count", int(dm.sum()))
(a,) = torch.autograd.grad(geo_t, pin)
(b,) = torch.autograd.grad(geo_f, pin)
print("dpin rel", float((a - b).norm() / a.norm()), "nz", int((a != 0).any(-1).sum()), int((b != 0).any(-1).sum()))
d = (a - b).norm(dim=-1)
i = int(d.argmax())
print("worst", i, a.view(-1, 3)[i].tolist(), b.view(-1, 3)[i].tolist())
y, x = divmod(i, view.image_width)
pv = piv.view(-1, 3)[i].detach(); pr = proj.view(-1, 2)[i].detach(); nz = noise.view(-1)[i].detach()
print("pix", x, y, "pin", pin.view(-1, 3)[i].tolist(), "piv", pv.tolist(), "proj", pr.tolist(), "noise", float(nz),
      "w", float(w.view(-1)[i]), "dm", bool(dm.view(-1)[i]))
cnt = float(dm.sum())
gn_ = float(w.view(-1)[i]) / cnt
dvec = pr - pixels_f.view(-1, 2)[i] + 1e-6
gproj = gn_ * dvec / nz
z = pv[2]
gv = torch.stack([gproj[0] * view.Fx / z, gproj[1] * view.Fy / z, -(gproj[0] * view.Fx * pv[0] + gproj[1] * view.Fy * pv[1]) / z ** 2])
print("hand dpin", (n2v_R @ gv).tolist())
