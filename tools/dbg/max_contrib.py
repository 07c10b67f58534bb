import math, sys
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd"]
import numpy as np, torch
import gsr_scene as S
from diff_gaussian_rasterization import _C
dev = torch.device("cuda")
P, W, H = 1_000_000, 1920, 1080
cam = S.make_camera(W, H).to(dev)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
E = torch.Tensor([])
args = (torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
        inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, 0, 1.0, cam.world_view_transform,
        cam.full_proj_transform, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 0.0, H, W, cam.camera_center,
        False, True, False)
out = _C.rasterize_gaussians(*args)
ib = out[8]
off = (-ib.data_ptr()) % 256
nc = ib[off:off + 4 * W * H].view(torch.int32).cpu().numpy().reshape(H, W)
gy, gx = (H + 15) // 16, (W + 15) // 16
pad = np.zeros((gy * 16, gx * 16), np.int64); pad[:H, :W] = nc
mc = pad.reshape(gy, 16, gx, 16).max(axis=(1, 3)).ravel()
print("max_contrib quantiles 50/90/99/max", np.quantile(mc, [.5, .9, .99]), mc.max())
for t in (192, 224, 256, 288, 320, 352):
    print(t, "tiles above", int((mc > t).sum()), "of", len(mc))
print("per-pixel last quantiles", np.quantile(nc, [.5, .9, .99]))
