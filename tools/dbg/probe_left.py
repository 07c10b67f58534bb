"""Development probe (round 6): how many sample_depth points the Halley walks leave to the passes, per pass wave, on small scenes of the parity tests' kind (STATS instance).  python tools/dbg/probe_left.py"""
import math, sys, os
sys.path[:0] = ["/root/repo/tests", "/root/repo/geometry-grounded-gaussian-splatting_amd", "/root/repo"]
import torch
import helpers as Hh
from test_oracle import sample_args, sample_points
from diff_gaussian_rasterization import _C
for ls in (0.12, 0.3, 0.6, 1.0):
    for ol in (2.0, 0.0, -1.0):
        c = Hh.small_case(P=400, W=96, H=64, seed=5, log_scale=math.log(ls), opacity_max_logit=ol, z_range=(2.0, 5.0))
        pts = sample_points(c, 6000, 105)
        ga = [x.cuda() if isinstance(x, torch.Tensor) else (torch.Tensor([]) if x is None else x) for x in sample_args(c, pts)] + [False]
        _C.set_option(_C.OPT_RENDER_STATS, 1)
        _C.debug_render_stats(reset=True)
        out = _C.sample_rasterized_depth(*ga)
        torch.cuda.synchronize()
        st = _C.debug_render_stats(reset=True)
        _C.set_option(_C.OPT_RENDER_STATS, 0)
        print(f"scale {ls} logit {ol}: inside {int(out[4].sum())} left {st[7]} pass waves {st[5]} per wave {st[7]/max(st[5],1):.2f}", flush=True)
