"""integrate / evaluate_sdf timing at full size (development / DESIGN numbers).

1M Gaussians (the C3 scene), one 1080p view, the 15M tetra points of
GaussianModel.get_tetra_points (scene/gaussian_model.py:496-519) — the call
of mesh_extract_tetrahedra.py:75 (one view of the per-view loop).  Prints one
JSON line per query with ms per call, points per second and per-stage
HIP-event times.
"""
import json, math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_scene as S
from diff_gaussian_rasterization import _C

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H).to(dev)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
tanx, tany = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
pts = S.tetra_points(inp)
args = (pts, inp["means3D"], inp["opacities"], inp["scales"], inp["rotations"], 1.0, torch.Tensor([]),
        torch.Tensor([]), cam.world_view_transform, cam.full_proj_transform, tanx, tany, 0.0, H, W,
        cam.camera_center, False, False)

for name, fn in (("integrate", _C.integrate_gaussians_to_points), ("evaluate_sdf", _C.evaluate_sdf_from_signle_view)):
    for _ in range(2):
        out = fn(*args)
    torch.cuda.synchronize()
    _C.timing_collect()
    _C.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn(*args)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    _C.timing_enable(False)
    st = _C.timing_collect()
    inside = out[-1]
    print(json.dumps({"what": f"{name}, 1M Gaussians, 1920x1080, {pts.shape[0]} tetra points",
                      "ms_per_call": round(dt * 1e3, 4), "Gpoints_per_s": round(pts.shape[0] / dt / 1e9, 3),
                      "num_rendered": out[0], "points_in_view": int(inside.sum()) if name == "integrate" else None,
                      "inside": int(inside.sum()),
                      "stage_ms": {k: round(v / n, 4) for k, (v, n) in st.items() if n}}), flush=True)
