"""depth_to_normal fwd+bwd at 1080p against the reference's torch formulation
on the same GPU.  One JSON line."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import torch
import gsr_geometry as G
from oracle import ssim_ref
from test_gpu_depth_normal import View

dev = torch.device("cuda")
W, H = 1920, 1080
view = View(W, H)
depth = (torch.rand(1, H, W, device=dev) + 2).contiguous()
gn = torch.randn(3, H, W, device=dev)


def run(fn, n=20):
    d = depth.clone().requires_grad_(True)
    for _ in range(3):
        (fn(d)[0] * gn).sum().backward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        (fn(d)[0] * gn).sum().backward()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


t_fused = run(lambda d: G.depth_to_normal(view, d))


def ref(d):
    x = (torch.arange(W, dtype=torch.float32, device=dev) - view.Cx) / view.Fx
    y = (torch.arange(H, dtype=torch.float32, device=dev) - view.Cy) / view.Fy
    pts = torch.cat([d * x[None, None], d * y[None, :, None], d], dim=0)
    dy = pts[:, 2:, 1:-1] - pts[:, :-2, 1:-1]
    dx = pts[:, 1:-1, 2:] - pts[:, 1:-1, :-2]
    n = torch.nn.functional.normalize(torch.cross(dy, dx, dim=0), dim=0)
    return torch.nn.functional.pad(n, (1, 1, 1, 1)), None


t_torch = run(ref)
print(json.dumps({"what": "depth_to_normal fwd+bwd (sum(n * g) backward), 1920x1080", "fused_ms": round(t_fused, 4),
                  "torch_ms": round(t_torch, 4), "speedup": round(t_torch / t_fused, 2)}))
