"""Training-update timing at the C3 scale (1M Gaussians, SH 3 + SG 7 lobes
of parameters, i.e. the full GaussianModel parameter set): FusedAdam.step()
(one HIP launch) against torch.optim.Adam (foreach, the reference's
optimizer on the GPU), plus the densification statistics.  Prints one JSON
line with the achieved HBM GB/s (28 B per parameter element per step)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import torch
import gsr_optim
from diff_gaussian_rasterization import _C
from test_gpu_optim import _groups

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda")


def timed(opt, groups, n=20):
    for grp in groups:
        grp["params"][0].grad = torch.randn_like(grp["params"][0]) * 1e-3
    for _ in range(3):
        opt.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        opt.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


gm = _groups(P, 0, dev)
elems = sum(g["params"][0].numel() for g in gm)
t_fused = timed(gsr_optim.FusedAdam(gm, lr=0.0, eps=1e-15), gm)
gt = _groups(P, 0, dev)
t_torch = timed(torch.optim.Adam(gt, lr=0.0, eps=1e-15), gt)
# kernel-only time of the fused step (HIP events around one launch)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
opt = gsr_optim.FusedAdam(gm, lr=0.0, eps=1e-15)
opt.step()
e0.record()
for _ in range(20):
    opt.step()
e1.record()
torch.cuda.synchronize()
k_ms = e0.elapsed_time(e1) / 20
vgrad = torch.randn(P, 3, device=dev)
radii = torch.randint(0, 4, (P,), device=dev, dtype=torch.int32)
stats = [torch.zeros(P, device=dev)] + [torch.zeros(P, 1, device=dev) for _ in range(3)]
_C.densify_stats(vgrad, radii, *stats)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    _C.densify_stats(vgrad, radii, *stats)
e1.record()
torch.cuda.synchronize()
d_ms = e0.elapsed_time(e1) / 20
print(json.dumps({"what": f"Adam step over the full GaussianModel parameter set, P={P}", "elements": elems,
                  "fused_ms": round(t_fused * 1e3, 4), "fused_event_ms": round(k_ms, 4),
                  "torch_foreach_ms": round(t_torch * 1e3, 4), "speedup": round(t_torch / t_fused, 2),
                  "fused_GBps": round(28 * elems / (k_ms * 1e-3) / 1e9, 1),
                  "densify_stats_ms": round(d_ms, 4), "densify_stats_GBps": round(P * 40 / (d_ms * 1e-3) / 1e9, 1)}))
