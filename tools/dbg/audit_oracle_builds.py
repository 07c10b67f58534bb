"""Calibration of tests/flip_audit.py: the oracle against itself with libm expf
instead of the fast-math form (two fp32 builds of one algorithm) on the full
C3 scene, every differing pixel classified as the GPU audit does.
python tools/dbg/audit_oracle_builds.py   (~1 min on 8 threads; CPU only)"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import flip_audit as FA, gsr_scene as S, helpers as Hh
from oracle import gsr_oracle as O

O.set_threads(os.cpu_count() or 8)
W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H)
inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
c = dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
         require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))
a = Hh.oracle_args(c)
O.set_exp_mode(1); o1 = O.forward(*a)
O.set_exp_mode(0); o0 = O.forward(*a)
O.set_exp_mode(1)
n1, n0 = o1["state"].n_contrib().astype(np.int64), o0["state"].n_contrib().astype(np.int64)
ch = FA.PixelChains(o1, W, H, c["tanx"], c["tany"])
bad = n1 != n0
for name in ("color", "alpha", "normal", "mdepth"):
    bad |= (np.abs(o1[name] - o0[name]).astype(np.float64) > 1e-4 * np.abs(o1[name]).max()).reshape(-1, H, W).any(0)
for y, x in np.argwhere(bad):
    upto = int(max(n1[y, x], n0[y, x])) + 1
    print(f"pixel ({x}, {y}): last {n1[y, x]} / {n0[y, x]}, composite margin {FA.chain_margin(ch, int(x), int(y), upto):.2e}")
print(f"{int(bad.sum())} differing pixels of {W * H}")
