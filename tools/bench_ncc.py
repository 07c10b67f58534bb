"""warp_patch_ncc timing at the training scale: every pixel of a 1920x1080
view (the upper bound of the PatchMatch loss's valid set) against a 1080p
neighbour image.  One JSON line."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import torch
import warp_patch_ncc as W
from test_oracle import ncc_case

dev = torch.device("cuda")
Wd, Hd = 1920, 1080
d, n, uv, R, T, ir, inn, K = ncc_case(1, 0, Wd, Hd, Wd, Hd)
ys, xs = torch.meshgrid(torch.arange(Hd, dtype=torch.int32), torch.arange(Wd, dtype=torch.int32), indexing="ij")
uv = torch.stack([xs.reshape(-1), ys.reshape(-1)], 1).contiguous()
P = uv.shape[0]
g = torch.Generator().manual_seed(0)
d = (torch.rand(P, generator=g) * 2 + 2)
nrm = torch.randn(P, 3, generator=g) * 0.3
nrm[:, 2] = -1
n = nrm / nrm.norm(dim=1, keepdim=True)
args = [d.to(dev), n.to(dev), uv.to(dev), R.reshape(3, 3).to(dev), T.to(dev), ir.to(dev), inn.to(dev), *K.values(), False]
for _ in range(3):
    W._C.warp_patch_ncc(*args)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    out = W._C.warp_patch_ncc(*args)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(json.dumps({"what": "warp_patch_ncc, every pixel of a 1920x1080 view", "points": P, "ms": round(ms, 4),
                  "valid": int(out[3].sum()), "Mpoints_per_s": round(P / ms / 1e3, 1)}))
