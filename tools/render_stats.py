"""Print the render_fwd diagnostic counters (GSR_OPT_RENDER_STATS) (development tool).

python tools/render_stats.py [P W H]   (default C3: 1000000 1920 1080; C2: 100000 800 800)"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import gsr_scene as S
from diff_gaussian_rasterization import _C

dev = torch.device("cuda")
P, W, H = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (1_000_000, 1920, 1080)
cam = S.make_camera(W, H).to(dev)
inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
E = torch.Tensor([])
args = (torch.zeros(3, device=dev), inp["means3D"], E, inp["opacities"], inp["scales"], inp["rotations"], E,
        inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, 0, 1.0, cam.world_view_transform,
        cam.full_proj_transform, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 0.0, H, W, cam.camera_center,
        False, True, False)
_C.set_option(_C.OPT_RENDER_STATS, 1)
_C.debug_render_stats(reset=True)
_C.rasterize_gaussians(*args)
torch.cuda.synchronize()
st = _C.debug_render_stats(reset=True)
_C.set_option(_C.OPT_RENDER_STATS, 0)
print("walk wave-steps", st[0], "active lanes/step", round(st[1] / max(st[0], 1), 2))
print("composite wave-steps", st[2], "blending lanes/step", round(st[3] / max(st[2], 1), 2))
print(f"P={P} {W}x{H}")
print("refine waves", st[4], "fallback waves", st[5], "refine lane-walks", st[6], "lanes left", st[7])
if os.environ.get("GSR_PHASE_CLOCK"):  # a -DGSR_PHASE_CLOCK=1 build: per-wave clock sums by phase
    names = ("composite", "outputs, staging, publish", "phase 1 probe walk", "phase 1 Halley walks", "phase 2",
             "phase 2b", "phase 3")
    tot = max(st[15], 1)
    for k, name in enumerate(names):
        print(f"clock {name}: {st[8 + k]:.4g} wave-cycles ({st[8 + k] / tot:.3f})")
    print(f"clock total to phase-3 end: {st[15]:.4g}")
    sys.exit(0)
if os.environ.get("GSR_LEFT_STATS"):  # a -DGSR_LEFT_STATS=1 build: why pixels are left to the passes
    print("left to the passes: no guess", st[12], "still live after its walks", st[13], "converged (Newton), conditioning", st[14],
          "| ill roots", st[15], "| the rest (bracket closed, conditioning):", st[7] - st[12] - st[13] - st[14])
    sys.exit(0)
for f, name in enumerate(("1 grid", "2 first walk", "2b grouped", "3 passes/dT")):
    print(f"phase {name}: walk wave-steps {st[8 + 2 * f]} active lanes/step {st[9 + 2 * f] / max(st[8 + 2 * f], 1):.2f}")
print("ill-conditioned roots kept", st[16], "phase-3 lanes", st[17], "passes skipped by brackets", st[18],
      "pixels skipping", st[19])
