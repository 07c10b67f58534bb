"""sample_depth timing at full size (development / DESIGN numbers).

1M Gaussians (the C3 scene), 1080p: the points are the C3 view's median-depth
points (one per pixel, [H, W, 3]) re-observed by an orbit camera — the
multi-view loss's call (utils/loss_utils.py:147-166).  Times
GaussianRasterizer.sample_depth forward + autograd backward and prints the
per-stage HIP-event times as one JSON line.
"""
import json, math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_scene as S
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for kv in sys.argv[2:]:  # OPT=VALUE pairs (gsr_set_option), for A/B runs
    _C.set_option(*map(int, kv.split("=")))
dev = torch.device("cuda")
W, H, P = 1920, 1080, 1_000_000
cam0 = S.make_camera(W, H).to(dev)
raw = S.make_gaussians(P, aspect=H / W)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(raw).items()}
tanx, tany = math.tan(cam0.FoVx / 2), math.tan(cam0.FoVy / 2)


def settings(cam):
    return GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=tanx, tanfovy=tany, kernel_size=0.0, bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=3,
        sg_degree=0, campos=cam.camera_center, prefiltered=False, require_depth=True, debug=False)


with torch.no_grad():
    color, radii, md, alpha, normal = GaussianRasterizer(settings(cam0))(
        means3D=inp["means3D"], means2D=torch.zeros(P, 3, device=dev), opacities=inp["opacities"], shs=inp["shs"],
        sg_axis=inp["sg_axis"], sg_sharpness=inp["sg_sharpness"], sg_color=inp["sg_color"], scales=inp["scales"],
        rotations=inp["rotations"])
fx, fy = W / (2 * tanx), H / (2 * tany)
ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                        torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
d = md[0]
pts = torch.stack([(xs - (W - 1) / 2) / fx * d, (ys - (H - 1) / 2) / fy * d, d], -1).contiguous()
cam1 = S.orbit_cameras(8, W, H)[1].to(dev)
rz = GaussianRasterizer(settings(cam1))
params = {k: inp[k].clone().requires_grad_(True) for k in ("means3D", "opacities", "scales", "rotations")}
pts.requires_grad_(True)
g = torch.randn_like(pts) * 1e-2


def step():
    for t in list(params.values()) + [pts]:
        t.grad = None
    depth, inside = rz.sample_depth(points3D=pts, means3D=params["means3D"], opacities=params["opacities"],
                                    scales=params["scales"], rotations=params["rotations"])
    torch.autograd.backward([depth], [g])
    return inside


for _ in range(3):
    inside = step()
torch.cuda.synchronize()
_C.timing_collect()
_C.timing_enable(True)
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
_C.timing_enable(False)
st = _C.timing_collect()
_C.CAPTURE_SAMPLE = True
out = _C.sample_rasterized_depth(pts.detach(), params["means3D"].detach(), params["opacities"].detach(),
                                 params["scales"].detach(), params["rotations"].detach(), 1.0, torch.Tensor([]),
                                 cam1.world_view_transform, cam1.full_proj_transform, tanx, tany, 0.0, H, W,
                                 cam1.camera_center, False, False)
_C.CAPTURE_SAMPLE = False
stage_ms = {k: round(v / n, 4) for k, (v, n) in st.items() if n}
# roofline lines for the two sample kernels, per launch, against the HBM peak (both are
# VALU-bound: their PMC pipe-busy figures are in profiles/pmc_e2e.json).  Algorithmic bytes, with bench.py's
# convention for the forward (bench.sample_fwd_bytes: per tile its list read once up to the largest last
# contributor of its points, 4-B id + 48-B record, and per point in view 12 B in + 26 B out); the backward
# reads the same list entries and adds per entry the accumulator record's 10 fields read and written (80 B)
# and per point 46 B in (xy, last, median depth, inside, upstream gradient, dT/dt_m and its flag, the 3-D
# point) + 12 B out (the point's gradient).
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402

fwd_bytes, entries, n_in = B.sample_fwd_bytes(_C.last_sample)
bwd_bytes = entries * (4 + 48 + 80) + n_in * (46 + 12)
roof = {}
for name, nbytes in (("sample_fwd", fwd_bytes), ("sample_bwd", bwd_bytes)):
    ms = stage_ms.get(name)
    if ms:
        gbs = nbytes / (ms * 1e-3) / 1e9
        roof[name] = {"bound": "valu", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                      "frac": round(gbs / 8000.0, 5), "algorithmic_bytes_per_launch": int(nbytes),
                      "avg_launch_ms": ms, "list_entries": entries, "points_in_view": n_in}
print(json.dumps({"what": "sample_depth fwd+bwd (autograd), 1M Gaussians, 1920x1080 points from a second view",
                  "ms_per_call": round(dt * 1e3, 4), "calls_per_s": round(1 / dt, 2), "num_rendered": out[0],
                  "num_points": out[1], "inside": int(out[4].sum()), "stage_ms": stage_ms, "roofline": roof}))
if os.environ.get("SAMPLE_STATS"):  # the SAMPLE raster's counters (and, in a -DGSR_PHASE_CLOCK=1 build, clocks)
    _C.set_option(_C.OPT_RENDER_STATS, 1)
    _C.debug_render_stats(reset=True)
    _C.sample_rasterized_depth(pts.detach(), params["means3D"].detach(), params["opacities"].detach(),
                               params["scales"].detach(), params["rotations"].detach(), 1.0, torch.Tensor([]),
                               cam1.world_view_transform, cam1.full_proj_transform, tanx, tany, 0.0, H, W,
                               cam1.camera_center, False, False)
    torch.cuda.synchronize()
    s = _C.debug_render_stats(reset=True)
    _C.set_option(_C.OPT_RENDER_STATS, 0)
    print("walk wave-steps", s[0], "active lanes/step", round(s[1] / max(s[0], 1), 2), "composite wave-steps", s[2],
          "blending lanes/step", round(s[3] / max(s[2], 1), 2), "refine waves", s[4], "pass waves", s[5],
          "root updates", s[6], "lanes left", s[7], "dT walked exactly (loose continuation)", s[19])
    clock = bool(os.environ.get("GSR_PHASE_CLOCK"))  # (a -DGSR_PHASE_CLOCK=1 build: slots 8.. are clocks)
    if not clock:  # walk wave-steps and active lanes per walk index, and the grouped dT walk
        print("per walk: " + ", ".join(f"{name} {s[8 + 2 * k]} steps x {s[9 + 2 * k] / max(s[8 + 2 * k], 1):.1f} lanes"
                                       for k, name in enumerate(("walk1", "walk2", "walk3", "walk4+ and passes", "dT group")))
              + f"; passes etc. {s[0] - sum(s[8 + 2 * k] for k in range(5))} steps")
    if clock:
        for k, name in enumerate(("composite", "masks/staging", "probe walk", "Halley walks", "passes", "-", "-")):
            print(f"clock {name}: {s[8 + k]:.4g} ({s[8 + k] / s[15]:.3f})")
        print(f"clock prologue (in composite): {s[16]:.4g}; batches {s[17]} (per wave {s[17] / max(s[4], 1):.2f}), "
              f"with the wave's lanes all done {s[18]}")
