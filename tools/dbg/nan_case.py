"""Debug: locate NaNs in the GPU backward of a small parity case."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import gsr_scene as S, helpers as Hh
from diff_gaussian_rasterization import _C
c = Hh.small_case(P=40, W=40, H=24, seed=0)
a = list(Hh.oracle_args(c))
dev = torch.device("cuda")
g = lambda t: torch.Tensor([]).to(dev) if t is None else (t.to(dev) if isinstance(t, torch.Tensor) else t)
ga = [g(x) for x in a] + [False]
out = _C.rasterize_gaussians(*ga)
K, color, alpha, normal, mdepth, radii = out[:6]
print("K", K, "alpha range", float(alpha.min()), float(alpha.max()), "nan imgs", [bool(torch.isnan(t).any()) for t in (color, alpha, normal, mdepth)])
gr = S.upstream_grads(c["H"], c["W"])
gr["alpha"] = torch.randn(1, c["H"], c["W"], generator=torch.Generator().manual_seed(5)) * 1e-3
for geom in (True,):
    gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gr["normal"]), alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7], out[8], out[9], geom, False)
    names = ["dmeans2D","dcolors","dopacity","dmeans3D","dcov3D","dsh","dsg_axis","dsg_sharpness","dsg_color","dscales","drotations"]
    for n, t in zip(names, gb):
        if t.numel():
            bad = torch.nonzero(~torch.isfinite(t.reshape(t.shape[0], -1)).all(1)).flatten().tolist()
            print(n, tuple(t.shape), "nonfinite rows:", bad[:10])
    nc = _C.debug_binning(out[7], out[9], K, c["H"], c["W"])
    print("radii", radii.tolist())
_C.KEEP_BWD_SCRATCH = True
gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gr["normal"]), alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7], out[8], out[9], True, False)
buf = _C.last_bwd_scratch
base = (-buf.data_ptr()) % 256
P = 40
acc = buf[base:base + P * 64].view(torch.float32).reshape(P, 16).cpu().numpy()
np.set_printoptions(linewidth=200, precision=3)
for gidx in (0, 1, 2):
    print(gidx, acc[gidx])
def run_bwd(gn):
    gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gn), alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7], out[8], out[9], True, False)
    buf = _C.last_bwd_scratch
    base = (-buf.data_ptr()) % 256
    acc = buf[base:base + P * 64].view(torch.float32).reshape(P, 16).cpu().numpy()
    return acc
acc0 = run_bwd(torch.zeros_like(gr["normal"]))
print("zero dL_dnormal: nan fields", np.argwhere(~np.isfinite(acc0))[:10].tolist())
gn = torch.zeros_like(gr["normal"]); gn[:, 0:8, :] = gr["normal"][:, 0:8, :]
acc1 = run_bwd(gn)
print("rows 0-7 only: nan fields", np.argwhere(~np.isfinite(acc1))[:10].tolist())
gn = torch.zeros_like(gr["normal"]); gn[:, 16:24, :] = gr["normal"][:, 16:24, :]
acc2 = run_bwd(gn)
print("rows 16-23 only: nan fields", np.argwhere(~np.isfinite(acc2))[:10].tolist())
nc = None
print("alpha==0 pixels:", int((alpha == 0).sum()))
