"""Full-C3 gradient parity detail (development tool): the GPU backward with
the forward's cached dT/dt_m (default) and with the recomputing pre-pass
(OPT_BWD_NO_CACHE) against the oracle backward on the GPU forward's state."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools", "dbg")]
import numpy as np, torch
import gsr_scene as S, helpers as Hh
from diff_gaussian_rasterization import _C
from oracle import gsr_oracle as O
from grad_report import full, g, compare, NAMES

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
c = full(1_000_000, 0) if cfg == "c3" else full(5_000_000, 7)
O.set_threads(16)
args = Hh.oracle_args(c)
ga = [g(a) for a in args] + [False]
out = _C.rasterize_gaussians(*ga)
K, color, alpha, normal, mdepth, radii = out[:6]
H, W = c["H"], c["W"]
gr = S.upstream_grads(H, W)
gr["alpha"] = torch.randn(1, H, W, generator=torch.Generator().manual_seed(5)) * 1e-3
o = O.forward(*args)
o["state"].set_n_contrib(Hh.gpu_n_contrib_for_oracle(out, o, H, W))
b = O.backward(o["state"], *args[:19], gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], alpha.cpu(), normal.cpu(),
               mdepth.cpu(), c["cam"].camera_center, o["radii"])
op = c["inp"]["opacities"].numpy().reshape(-1)
for nm, opt in (("cached", 0), ("no_cache", 1)):
    _C.set_option(_C.OPT_BWD_NO_CACHE, opt)
    gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gr["normal"]),
                                         alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7],
                                         out[8], out[9], True, False)
    compare([t.cpu() for t in gb], b, op, o["radii"], f"GPU {nm} vs oracle (fast-math exp, GPU state)")
_C.set_option(_C.OPT_BWD_NO_CACHE, 0)
# the same with the upstream median-depth gradient zeroed: what is left comes from colour / normal / alpha
gr0 = dict(gr, mdepth=torch.zeros_like(gr["mdepth"]))
b0 = O.backward(o["state"], *args[:19], gr0["color"], gr0["mdepth"], gr0["alpha"], gr0["normal"], alpha.cpu(),
                normal.cpu(), mdepth.cpu(), c["cam"].camera_center, o["radii"])
gb0 = _C.rasterize_gaussians_backward(*ga[:19], g(gr0["color"]), g(gr0["mdepth"]), g(gr0["alpha"]), g(gr0["normal"]),
                                      alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7],
                                      out[8], out[9], True, False)
compare([t.cpu() for t in gb0], b0, op, o["radii"], "no median-depth upstream gradient")
