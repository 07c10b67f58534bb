"""Per-tile live list lengths at C3 / C5 (development tool)."""
import math, os, sys
sys.path[:0] = ["/root/repo", "/root/repo/geometry-grounded-gaussian-splatting_amd"]
import numpy as np, torch
import gsr_scene as S
from diff_gaussian_rasterization import _C
dev = torch.device("cuda")
for P, sgd in ((1_000_000, 0), (5_000_000, 7)):
    W, H = 1920, 1080
    cam = S.make_camera(W, H).to(dev)
    inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, sg_degree=sgd, aspect=H / W)).items()}
    E = torch.Tensor([])
    args = (torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
            inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, sgd, 1.0, cam.world_view_transform,
            cam.full_proj_transform, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 0.0, H, W, cam.camera_center,
            False, True, False)
    out = _C.rasterize_gaussians(*args)
    _, ranges = _C.debug_binning(out[7], out[9], out[0], H, W)
    L = (ranges[:, 1].astype(np.int64) - ranges[:, 0])
    print(P, "K", out[0], "K_live", L.sum(), "tiles", len(L), "mean", L.mean(), "q50/90/99/max", np.quantile(L, [.5, .9, .99]), L.max(),
          "tiles>2048", (L > 2048).sum(), ">4096", (L > 4096).sum(), ">8192", (L > 8192).sum())
    del inp, out
