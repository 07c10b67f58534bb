"""Debug: forward + backward of one small case with the library GSR_LIB points at, saved for a
comparison between builds.  python tools/dbg/lib_compare.py OUT.npz [case kwargs as k=v ...]"""
import sys, os, math
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo/tests"]
os.chdir("/root/repo")
import numpy as np, torch
import test_gpu_parity as T
import helpers as Hh
import gsr_scene as S
from diff_gaussian_rasterization import _C
kw = {}
for a in sys.argv[2:]:
    k, v = a.split("=")
    kw[k] = float(v) if "." in v else int(v)
c = Hh.small_case(**kw)
ga = [T._gpu(x) for x in T._fwd_args(c)] + [False]
out = _C.rasterize_gaussians(*ga)
g = {k: T._gpu(v) for k, v in S.upstream_grads(c["H"], c["W"], seed=61).items()}
b = _C.rasterize_gaussians_backward(*ga[:19], g["color"], g["mdepth"], g["alpha"], g["normal"], out[2], out[3], out[4],
                                    T._gpu(c["cam"].camera_center), out[5], out[6], out[0], out[7], out[8], out[9],
                                    c["require_depth"], False)
np.savez(sys.argv[1], mdepth=out[4].cpu().numpy(), alpha=out[2].cpu().numpy(),
         dmeans2D=b[0].cpu().numpy(), dmeans3D=b[3].cpu().numpy(), dopac=b[2].cpu().numpy())
print("saved", sys.argv[1])
