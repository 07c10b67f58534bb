"""Fused SSIM timing at 1080p (1x3x1080x1920, padding "valid", forward +
backward), against the reference's own torch formulation (_ssim with conv2d,
utils/loss_utils.py:52-72, valid crop) on the same GPU.  One JSON line."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch
import fused_ssim as FS
from oracle import ssim_ref

dev = torch.device("cuda")
a = torch.rand(1, 3, 1080, 1920, device=dev)
b = (a + 0.1 * torch.randn_like(a)).clamp(0, 1)


def run(fn, n=20):
    x = a.clone().requires_grad_(True)
    for _ in range(3):
        fn(x).backward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn(x).backward()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


t_fused = run(lambda x: 1.0 - FS.fused_ssim(x, b, padding="valid"))
t_torch = run(lambda x: 1.0 - ssim_ref.ssim(x, b, padding="valid"))
print(json.dumps({"what": "SSIM fwd+bwd, 1x3x1080x1920, valid", "fused_ms": round(t_fused, 4),
                  "torch_conv2d_ms": round(t_torch, 4), "speedup": round(t_torch / t_fused, 2)}))
