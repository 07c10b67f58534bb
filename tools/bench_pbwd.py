"""Backward-stage timing at C3 / C5 (development tool): render_bwd and
preprocess_bwd per call from HIP events, with the per-Gaussian backward's
gradient rows written per lane (GSR_OPT_PBWD_STAGE 2), through LDS as
whole-wave stores (1), and not at all (the DC-row mode of the overlapped view
exchange: gsr_rasterize_backward_ex dc_rows), interleaved.

  python tools/bench_pbwd.py [C3|C5] [steps] [OPT=VALUE ...]
"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch  # noqa: E402

import gsr_scene as S  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for kv in sys.argv[3:]:
    _C.set_option(*map(int, kv.split("=")))
P, sg = {"C3": (1_000_000, 0), "C5": (5_000_000, 7)}[cfg]
dev = torch.device("cuda")
W, H = 1920, 1080
cam = S.make_camera(W, H).to(dev)
raw = S.make_gaussians(P, sg_degree=sg, aspect=H / W)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(raw).items()}
tanx, tany = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
E = torch.Tensor([])
args = [torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
        inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, sg, 1.0, cam.world_view_transform,
        cam.full_proj_transform, tanx, tany, 0.0]
out = _C.rasterize_gaussians(*args, H, W, cam.camera_center, False, True, False)
K, color, alpha, normal, mdepth, radii = out[:6]
g = {k: v.to(dev) for k, v in S.upstream_grads(H, W).items()}


class DCOnly:
    """The exchange protocol without collectives: DC-row mode, one range."""
    chunks = 1

    def __init__(self):
        self.buf = None

    def dc_rows(self, P_, d):
        if self.buf is None:
            self.buf = torch.empty(3 * P_, device=d)
        return self.buf

    def on_chunk(self, b, e, grads):
        pass


def bwd(ex=None):
    kw = {} if ex is None else {"exchange": ex}
    return _C.rasterize_gaussians_backward(*args, g["color"], g["mdepth"], None, g["normal"], alpha, normal, mdepth,
                                           cam.camera_center, radii, out[6], K, out[7], out[8], out[9], True, False,
                                           **kw)


dc = DCOnly()
for _ in range(3):
    bwd()
    bwd(dc)
torch.cuda.synchronize()
res = {}
for name, ex, opt in (("per_lane", None, 2), ("staged", None, 1), ("dc_rows", dc, 0)) * 2:
    _C.set_option(_C.OPT_PBWD_STAGE, opt)
    _C.timing_collect()
    _C.timing_stages(["render_bwd", "preprocess_bwd"])
    _C.timing_enable(True)
    for _ in range(steps):
        bwd(ex)
    torch.cuda.synchronize()
    _C.timing_enable(False)
    st = _C.timing_collect()
    res.setdefault(name, []).append({k: round(v[0] / max(1, v[1]), 4) for k, v in st.items() if v[1]})
_C.timing_stages(None)
_C.set_option(_C.OPT_PBWD_STAGE, 0)
print(json.dumps({"config": cfg, "P": P, "ms_per_call": res}))
