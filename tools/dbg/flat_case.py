import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo/tests"]
os.chdir("/root/repo")
import numpy as np, torch
import test_gpu_parity as T
from diff_gaussian_rasterization import _C
import helpers as Hh
for opt in (0, 1):
    _C.set_option(_C.OPT_NO_REFINE, opt)
    for fl, seed in ((1000.0, 11), (20.0, 12)):
        try:
            T._run(Hh.small_case(P=2000, W=96, H=64, seed=seed, flat=fl))
            print("norefine", opt, "flat", fl, "OK")
        except AssertionError as e:
            print("norefine", opt, "flat", fl, "FAIL", e)
