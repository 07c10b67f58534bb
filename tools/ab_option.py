"""A/B timing of a gsr_set_option switch at C3 (development tool).

python tools/ab_option.py OPT [VALUE_B] [steps]: times the C3 forward +
backward (1M Gaussians, 1080p, GEOM) with the option at 0 and at VALUE_B,
interleaved, and prints per-stage HIP-event medians plus the largest
output differences between the two settings (one JSON line per setting)."""
import json, math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_scene as S
from diff_gaussian_rasterization import _C

opt = int(sys.argv[1])
val_b = int(sys.argv[2]) if len(sys.argv) > 2 else 1
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda")
W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H).to(dev)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
gr = {k: v.to(dev) for k, v in S.upstream_grads(H, W).items()}
tanx, tany = math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2)
E = torch.Tensor([])
fargs = (torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
         inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, 0, 1.0, cam.world_view_transform,
         cam.full_proj_transform, tanx, tany, 0.0)


def step():
    out = _C.rasterize_gaussians(*fargs, H, W, cam.camera_center, False, True, False)
    K, color, alpha, normal, mdepth, radii = out[:6]
    g = _C.rasterize_gaussians_backward(*fargs, gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], alpha, normal,
                                        mdepth, cam.camera_center, radii, out[6], K, out[7], out[8], out[9], True,
                                        False)
    return color, mdepth, normal, g


res = {}
times = {0: [], val_b: []}
for it in range(steps + 2):
    for v in (0, val_b):
        _C.set_option(opt, v)
        _C.timing_collect()
        _C.timing_enable(True)
        o = step()
        torch.cuda.synchronize()
        _C.timing_enable(False)
        st = _C.timing_collect()
        if it >= 2:
            times[v].append({k: ms for k, (ms, n) in st.items() if n})
        res[v] = o
_C.set_option(opt, 0)
for v in (0, val_b):
    keys = times[v][0].keys()
    med = {k: round(sorted(t[k] for t in times[v])[len(times[v]) // 2], 4) for k in keys}
    print(json.dumps({"option": opt, "value": v, "stage_ms_median": med,
                      "total_ms": round(sum(med.values()), 4)}), flush=True)
a, b = res[0], res[val_b]
diff = {n: float((x - y).abs().max() / y.abs().max().clamp_min(1e-30))
        for n, x, y in (("color", a[0], b[0]), ("mdepth", a[1], b[1]), ("normal", a[2], b[2]))}
diff.update({f"grad{i}": float((x - y).abs().max() / y.abs().max().clamp_min(1e-30))
             for i, (x, y) in enumerate(zip(a[3], b[3])) if x.numel()})
print(json.dumps({"max_rel_diff": diff}))
