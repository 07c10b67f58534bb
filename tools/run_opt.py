"""Run C3 forward + backward steps with one gsr_set_option value (for rocprofv3 passes; development tool).
python tools/run_opt.py OPT VALUE [steps]"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_scene as S
from diff_gaussian_rasterization import _C

opt, val = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda")
W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H).to(dev)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
E = torch.Tensor([])
fargs = (torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
         inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, 0, 1.0, cam.world_view_transform,
         cam.full_proj_transform, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 0.0)
_C.set_option(opt, val)
for _ in range(steps):
    _C.rasterize_gaussians(*fargs, H, W, cam.camera_center, False, True, False)
torch.cuda.synchronize()
print("done", opt, val, steps)
