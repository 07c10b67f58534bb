"""Simulation (round 6): render_bwd work split.  For sampled C3 tiles (oracle
forward state): per list entry up to the tile's max contributor, which of the
tile's pixels the backward finds valid for it (contributor < the pixel's last,
power <= 0, alpha >= 1/255: exactly the forward's blended set).  Reports the
entries any pixel needs (the one-wave walk S), and the entries each 16x8 half
(two waves) or each 16x4 quarter needs (the sums a per-half / per-quarter walk
would do), plus the valid (pixel, entry) fraction.
python tools/sim/bwd_split_sim.py [tiles]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch  # noqa: E402
import gsr_scene as S  # noqa: E402
import helpers as Hh  # noqa: E402
from oracle import gsr_oracle as O  # noqa: E402

NT = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H)
raw = S.make_gaussians(P, aspect=H / W)
inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
c = dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
         require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))
O.set_threads(8)
o = O.forward(*Hh.oracle_args(c))
st = o["state"]
geo = st.geometry()
plist = st.binning()["point_list"].astype(np.int64)
ranges = st.tile_state()["ranges"].astype(np.int64)
nc = st.n_contrib().astype(np.int64)
gx, gy = (W + 15) // 16, (H + 15) // 16
rng = np.random.default_rng(1)
tot = dict(S=0, halves=0, quarters=0, valid=0, pix_steps=0)
for _ in range(NT):
    t = int(rng.integers(gx * gy))
    tx, ty = t % gx, t // gx
    a, b = ranges[t]
    ys, xs = np.mgrid[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16]
    inside = (xs < W) & (ys < H)
    last = np.where(inside, nc[np.minimum(ys, H - 1), np.minimum(xs, W - 1)], 0)
    mc = int(last.max())
    if mc == 0:
        continue
    g = plist[a:a + mc]
    m = geo["means2D"][g].astype(np.float32)
    co = geo["conic_opacity"][g].astype(np.float32)
    dx = m[:, 0, None, None] - xs[None].astype(np.float32)
    dy = m[:, 1, None, None] - ys[None].astype(np.float32)
    power = -0.5 * (co[:, 0, None, None] * dx * dx + co[:, 2, None, None] * dy * dy) - co[:, 1, None, None] * dx * dy
    alpha = np.minimum(0.99, co[:, 3, None, None] * np.exp(np.minimum(power, 0)))
    idx = np.arange(mc)[:, None, None]
    valid = (idx < last[None]) & (power <= 0) & (alpha >= 1 / 255) & inside[None]
    anyv = valid.reshape(mc, -1).any(1)
    tot["S"] += int(anyv.sum())
    tot["halves"] += int(valid[:, :8].reshape(mc, -1).any(1).sum() + valid[:, 8:].reshape(mc, -1).any(1).sum())
    tot["quarters"] += int(sum(valid[:, 4 * q:4 * q + 4].reshape(mc, -1).any(1).sum() for q in range(4)))
    tot["valid"] += int(valid.sum())
    tot["pix_steps"] += int(anyv.sum()) * 256
print({k: v for k, v in tot.items()})
print(f"halves / S = {tot['halves'] / tot['S']:.3f}, quarters / S = {tot['quarters'] / tot['S']:.3f}, "
      f"valid fraction of walked pixel-steps = {tot['valid'] / tot['pix_steps']:.3f}")
# pixels sorted by last contributor: the lower half's pair is idle for every walked entry at or past
# its largest last (a wave-uniform skip), how much of the walk that is
rng = np.random.default_rng(2)
skip = walked = 0
for _ in range(NT):
    t = int(rng.integers(gx * gy))
    tx, ty = t % gx, t // gx
    a, b = ranges[t]
    ys, xs = np.mgrid[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16]
    inside = (xs < W) & (ys < H)
    last = np.where(inside, nc[np.minimum(ys, H - 1), np.minimum(xs, W - 1)], 0).reshape(-1)
    mc = int(last.max())
    if mc == 0:
        continue
    g = plist[a:a + mc]
    m = geo["means2D"][g].astype(np.float32)
    co = geo["conic_opacity"][g].astype(np.float32)
    xs_, ys_ = xs.reshape(-1).astype(np.float32), ys.reshape(-1).astype(np.float32)
    dx = m[:, 0, None] - xs_[None]
    dy = m[:, 1, None] - ys_[None]
    power = -0.5 * (co[:, 0, None] * dx * dx + co[:, 2, None] * dy * dy) - co[:, 1, None] * dx * dy
    alpha = np.minimum(0.99, co[:, 3, None] * np.exp(np.minimum(power, 0)))
    valid = (np.arange(mc)[:, None] < last[None]) & (power <= 0) & (alpha >= 1 / 255)
    anyv = valid.any(1)
    lo_half_max = np.sort(last)[:128].max()
    e = np.nonzero(anyv)[0]
    walked += len(e)
    skip += int((e >= lo_half_max).sum())
print(f"last-sorted halves: the lower half idle for {skip / max(walked, 1):.3f} of the walked entries")
