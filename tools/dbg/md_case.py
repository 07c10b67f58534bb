"""Debug: median depth of a small case vs the oracle, with and without the refinement."""
import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo/tests"]
os.chdir("/root/repo")
import numpy as np, torch
import test_gpu_parity as T
from diff_gaussian_rasterization import _C
from oracle import gsr_oracle as O
import helpers as Hh
c = Hh.small_case(P=40, W=40, H=24, seed=0)
a = T._fwd_args(c)
o = O.forward(*a)
ga = [T._gpu(x) for x in a] + [False]
for opt in (1, 0):
    _C.set_option(_C.OPT_NO_REFINE, opt)
    out = _C.rasterize_gaussians(*ga)
    md = out[4].cpu().numpy()[0]
    ref = o["mdepth"][0]
    d = np.abs(md - ref)
    idx = np.argsort(d.ravel())[::-1][:8]
    print("norefine", opt, "max|d|", d.max(), "n bad", int((d > 1e-4 * np.abs(ref).max()).sum()), "of", d.size)
    for i in idx:
        y, x = divmod(int(i), md.shape[1])
        print("  px", x, y, "gpu", md[y, x], "oracle", ref[y, x], "alpha", float(out[3][0, y, x]))
_C.set_option(_C.OPT_NO_REFINE, 0)
