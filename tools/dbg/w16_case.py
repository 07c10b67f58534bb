"""Debug: the median depth of one pixel of the W16400 small case (GPU vs oracle), with and without
the refinement.  python tools/dbg/w16_case.py [x y]  (GSR_LIB selects a build variant)"""
import sys, os, math
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo/tests"]
os.chdir("/root/repo")
import numpy as np, torch
import test_gpu_parity as T
import helpers as Hh
from diff_gaussian_rasterization import _C
from oracle import gsr_oracle as O
x, y = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (13802, 11)
c = Hh.small_case(P=600, W=16400, H=40, seed=9, log_scale=math.log(0.01))
a = T._fwd_args(c)
o = O.forward(*a)
ga = [T._gpu(x_) for x_ in a] + [False]
ref = o["mdepth"][0]
for opt in (0, 1):
    _C.set_option(_C.OPT_NO_REFINE, opt)
    out = _C.rasterize_gaussians(*ga)
    torch.cuda.synchronize()
    md = out[4].cpu().numpy()[0]
    d = np.abs(md - ref)
    print("norefine", opt, "pixel", md[y - 1:y + 2, x - 1:x + 2].tolist(), "oracle", ref[y - 1:y + 2, x - 1:x + 2].tolist())
    print("   n(|d| > 1e-3)", int((d > 1e-3).sum()), "worst", np.unravel_index(int(np.argmax(d)), d.shape), float(d.max()),
          flush=True)
_C.set_option(_C.OPT_NO_REFINE, 0)
