"""Simulation (round 6): how much of a pixel's blended set can a median-depth
walk skip?  For sampled C3 pixels (oracle forward, float64 composite chains):
the blended contributors, m0, and per contributor whether its factor in the
vacancy transmittance can differ from a constant over the reference's first
window [m0 - 0.4, m0 + 0.4] (|u| = |t - t_peak| sc <= sqrt(26) somewhere in
it, sc = rsigma sqrt(0.5 log2 e); beyond that g = exp2(-u^2) < 2^-26 and
1 - a g rounds to exactly 1 in fp32).  Reports the mean blended count, the
mean count of "near" contributors, the mean index span up to the last near one
(a walk truncated there), and the far-behind prefix before the first near one.
python tools/sim/near_band_sim.py [P W H samples]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import torch  # noqa: E402
import gsr_scene as S  # noqa: E402
import helpers as Hh  # noqa: E402
import flip_audit as FA  # noqa: E402
from oracle import gsr_oracle as O  # noqa: E402

P, W, H, N = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (1_000_000, 1920, 1080, 3000)))
cam = S.make_camera(W, H)
raw = S.make_gaussians(P, aspect=H / W)
inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
c = dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
         require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))
O.set_threads(8)
o = O.forward(*Hh.oracle_args(c))
ch = FA.PixelChains(o, W, H, c["tanx"], c["tany"])
rng = np.random.default_rng(0)
SC = math.sqrt(0.5 * math.log2(math.e))
REACH = math.sqrt(26.0)
stats = []
for _ in range(N):
    x, y = int(rng.integers(W)), int(rng.integers(H))
    power, alpha, t_peak, rsig = ch.contributors(x, y)
    last, T, m0, _ = ch.composite(x, y)
    if last == 0 or T > 0.45:
        continue  # no median depth (not in range)
    lo, hi = max(m0 - 0.4, 0.0), max(m0 + 0.4, 0.0)
    bl = [k for k in range(last) if not (power[k] > 0 or alpha[k] < 1 / 255)]
    near = []
    for k in bl:
        sc = rsig[k] * SC
        if sc <= 0:
            nr = lo <= t_peak[k] <= hi  # a step inside the window
        else:
            nr = (t_peak[k] > lo - REACH / sc) and (t_peak[k] < hi + REACH / sc)
        near.append(nr)
    near = np.array(near, bool)
    if not near.any():
        continue
    idx = np.nonzero(near)[0]
    stats.append((len(bl), int(near.sum()), int(idx[-1]) + 1, int(idx[0]), last))
s = np.array(stats, np.float64)
print(f"{len(s)} pixels with a median depth: blended {s[:, 0].mean():.1f}, near {s[:, 1].mean():.1f}, "
      f"walk truncated at the last near one {s[:, 2].mean():.1f} blended entries, far-behind prefix "
      f"{s[:, 3].mean():.1f}, last contributor {s[:, 4].mean():.1f}")
print("quantiles of truncated/blended:", np.quantile(s[:, 2] / s[:, 0], [0.1, 0.5, 0.9, 0.99]))
# distribution of the blended contributors' depths around m0 and their reach
d, r = [], []
for _ in range(300):
    x, y = int(rng.integers(W)), int(rng.integers(H))
    power, alpha, t_peak, rsig = ch.contributors(x, y)
    last, T, m0, _ = ch.composite(x, y)
    if last == 0 or T > 0.45:
        continue
    for k in range(last):
        if not (power[k] > 0 or alpha[k] < 1 / 255):
            d.append(t_peak[k] - m0)
            r.append(REACH / max(rsig[k] * SC, 1e-30))
d, r = np.array(d), np.array(r)
print("t_peak - m0 quantiles:", np.quantile(d, [0.01, 0.1, 0.5, 0.9, 0.99]))
print("reach sqrt(26)/sc quantiles:", np.quantile(r, [0.01, 0.1, 0.5, 0.9, 0.99]))
# far fraction at the root itself (what a second walk near the first one's depth could skip)
fr = []
for _ in range(400):
    x, y = int(rng.integers(W)), int(rng.integers(H))
    power, alpha, t_peak, rsig = ch.contributors(x, y)
    last, T, m0, _ = ch.composite(x, y)
    if last == 0 or T > 0.45:
        continue
    ts = np.linspace(max(m0 - 0.4, 0), max(m0 + 0.4, 0), 4001)
    Tv = ch.vacancy(x, y, last, ts)
    k0 = int(np.argmax(Tv < 0.5))
    tm = ts[k0]
    bl = [k for k in range(last) if not (power[k] > 0 or alpha[k] < 1 / 255)]
    u = np.array([abs(tm - t_peak[k]) * rsig[k] * SC for k in bl])
    sc = np.array([rsig[k] * SC for k in bl])
    far = u - sc * 1e-3 * max(tm, 1.0) > math.sqrt(26.0)
    fr.append(far.mean())
print("far fraction at the root (margin 1e-3 max(t,1)): mean", np.mean(fr), "quantiles", np.quantile(fr, [0.1, 0.5, 0.9]))
