"""Debug (round 6): the worst per-pixel median-depth difference outside proven ties of a parity case,
with the GPU's reference passes (OPT_NO_REFINE) beside the refined result and the float64 vacancy T
at each depth.  python tools/dbg/md_worst.py [case: w16400 | c1clamp | c3]"""
import math
import os
import sys

sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo/tests"]
os.chdir("/root/repo")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import flip_audit as FA  # noqa: E402
import gsr_scene as S  # noqa: E402
import helpers as Hh  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from oracle import gsr_oracle as O  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "w16400"
if which == "w16400":
    c = Hh.small_case(P=600, W=16400, H=40, seed=9, log_scale=math.log(0.01))
elif which == "c1clamp":
    c = Hh.small_case(P=10000, W=256, H=256, seed=44, log_scale=math.log(0.03), opacity_max_logit=6.0, opacity_std=3.0)
else:
    W, H, P = 1920, 1080, 1_000_000
    cam = S.make_camera(W, H)
    raw = S.make_gaussians(P, aspect=H / W)
    inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    c = dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
             require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))
a = T._fwd_args(c)
O.set_threads(16)
o = O.forward(*a)
ga = [T._gpu(x) for x in a] + [False]
out = _C.rasterize_gaussians(*ga)
_C.set_option(_C.OPT_NO_REFINE, 1)
outp = _C.rasterize_gaussians(*ga)
_C.set_option(_C.OPT_NO_REFINE, 0)
md = out[4].cpu().numpy()[0].astype(np.float64)
mdp = outp[4].cpu().numpy()[0].astype(np.float64)
ref = o["mdepth"][0].astype(np.float64)
both = (md != 0) & (ref != 0)
rel = np.where(both, np.abs(md - ref) / np.where(both, np.abs(ref), 1), 0)
ch = FA.PixelChains(o, c["W"], c["H"], c["tanx"], c["tany"])
order = np.argsort(-rel.ravel())[:12]
for i in order:
    y, x = divmod(int(i), md.shape[1])
    tg, to, tp = (ch.depth_of(x, y, v[y, x]) for v in (md, ref, mdp))
    last, Tf, m0, _ = ch.composite(x, y)
    Tv = ch.vacancy(x, y, last, [tg, to, tp])
    mm = FA.mdepth_flip_margin(ch, x, y, tg, to)
    print(f"px ({x},{y}) rel {rel[y, x]:.2e}  t gpu {tg:.7f} oracle {to:.7f} gpu-passes {tp:.7f}  "
          f"T(gpu) {Tv[0]:.7f} T(oracle) {Tv[1]:.7f} T(passes) {Tv[2]:.7f}  tie margin {mm:.2e}  last {last} m0 {m0:.5f}")
