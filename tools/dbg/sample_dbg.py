"""Development aid: per-point view of a sample_depth parity failure."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import helpers as Hh
from oracle import gsr_oracle as O
from test_oracle import sample_args, sample_points
from diff_gaussian_rasterization import _C
DEV = torch.device("cuda")
g_ = lambda x: x.to(DEV) if isinstance(x, torch.Tensor) else (torch.Tensor([]) if x is None else x)

def al(n): return (n + 255) // 256 * 256

c = Hh.small_case(P=2000, W=160, H=96, seed=2, log_scale=math.log(0.05))
pts = sample_points(c, 20000, 102)
a = list(sample_args(c, pts))
o = O.sample_forward(*a)
ga = [g_(x) for x in a] + [False]
out = _C.sample_rasterized_depth(*ga)
K, RN, TN, output, inside = out[:5]
PN = 20000
pbuf = out[7]
base = (256 - pbuf.data_ptr() % 256) % 256
raw = pbuf.cpu().numpy()[base:]
off_last = al(PN * 8); off_md = off_last + al(PN * 4); off_dT = off_md + al(PN * 4); off_c = off_dT + al(PN * 4)
last = raw[off_last:off_last + PN * 4].view(np.uint32)
md = raw[off_md:off_md + PN * 4].view(np.float32)
dT = raw[off_dT:off_dT + PN * 4].view(np.float32)
cached = raw[off_c:off_c + PN]
op = o["state"].points()
print("last mismatch", (last != op["n_contrib"]).sum(), "md relmax", Hh.rel_err(md, op["median_depth"]), "cached frac", cached.mean())
g = torch.randn(pts.shape, generator=torch.Generator().manual_seed(3)) * 1e-2
b = O.sample_backward(o["state"], *a[:9], o["inside"], g, c["tanx"], c["tany"], 0.0)
gb = _C.sample_rasterized_depth_backward(*ga[:9], inside, g_(g), c["tanx"], c["tany"], 0.0, c["H"], c["W"], g_(c["cam"].camera_center), *out[5:11], K, RN, TN, False, False)
for name, t in zip(["dopacity", "dmeans3D", "dcov3D", "dscales", "drotations", "dpoints3D"], gb):
    m, r = t.cpu().numpy().astype(np.float64), b[name]
    if np.any(r):
        print(name, "l2", np.linalg.norm(m - r) / np.linalg.norm(r), "relmax", Hh.rel_err(m, r))
m, r = gb[5].cpu().numpy(), b["dpoints3D"]
err = np.abs(m - r).max(1)
top = np.argsort(err)[-12:]
for i in top:
    print(i, "err %.3e ref %.3e" % (err[i], np.abs(r[i]).max()), "last", last[i], "md %.6f/%.6f" % (md[i], op["median_depth"][i]), "dT %.4e cached %d" % (dT[i], cached[i]), "inside", bool(o["inside"][i]))
