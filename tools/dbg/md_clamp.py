"""Median-depth mismatch diagnosis on the C1 clamp scene (development tool)."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import helpers as Hh
from diff_gaussian_rasterization import _C
from oracle import gsr_oracle as O

DEV = torch.device("cuda", 0)
c = Hh.small_case(P=10000, W=256, H=256, seed=44, log_scale=math.log(0.03), opacity_max_logit=6.0, opacity_std=3.0)
a = Hh.oracle_args(c)
ga = [torch.Tensor([]) if x is None else (x.to(DEV) if isinstance(x, torch.Tensor) else x) for x in a] + [False]
outs = {}
for nm, opt in (("refine", 0), ("bisect", 1)):
    _C.set_option(_C.OPT_NO_REFINE, opt)
    outs[nm] = _C.rasterize_gaussians(*ga)[4].cpu().numpy()[0]
_C.set_option(_C.OPT_NO_REFINE, 0)
for mode in (0, 1):
    O.set_exp_mode(mode)
    o = O.forward(*a)
    md = o["mdepth"][0]
    for nm, m in outs.items():
        d = np.abs(m - md)
        i = np.unravel_index(d.argmax(), d.shape)
        print(f"exp_mode {mode} {nm}: max|d|/max = {d.max() / np.abs(md).max():.2e} at {i}: gpu {m[i]:.7f} oracle {md[i]:.7f}"
              f"  pixels > 1e-4: {(d > 1e-4 * np.abs(md).max()).sum()}")
    print(f"exp_mode {mode} refine vs bisect (GPU): {np.abs(outs['refine'] - outs['bisect']).max() / np.abs(md).max():.2e}")
O.set_exp_mode(0)
