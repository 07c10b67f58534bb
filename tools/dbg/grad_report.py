"""Per-gradient GPU-vs-oracle report (development tool): relative L2, max
relative error and the Gaussian where the max error sits, for the small
parity cases and, with `full`, for full C3 and C5.

  python tools/dbg/grad_report.py [small] [c3] [c5]
"""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gsr_scene as S  # noqa: E402
import helpers as Hh  # noqa: E402
from diff_gaussian_rasterization import _C  # noqa: E402
from oracle import gsr_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
NAMES = ["dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dsg_axis", "dsg_sharpness", "dsg_color",
         "dscales", "drotations"]


def g(x):
    return torch.Tensor([]) if x is None else (x.to(DEV) if isinstance(x, torch.Tensor) else x)


def compare(gb, b, op, radii, tag):
    print(f"  -- {tag}", flush=True)
    for n, t in zip(NAMES, gb):
        a = t.cpu().numpy().astype(np.float64) if isinstance(t, torch.Tensor) else np.asarray(t, np.float64)
        r = b[n].astype(np.float64)
        if r.size == 0 or not np.any(r):
            continue
        l2 = np.linalg.norm(a - r) / np.linalg.norm(r)
        d = np.abs(a - r).reshape(a.shape[0], -1).max(1)
        i = int(d.argmax())
        mx = d[i] / np.abs(r).max()
        print(f"   {n:14s} L2 {l2:.2e}  max {mx:.2e}  at G{i} (r={int(radii[i])}, o={op[i]:.4f}, "
              f"|ref_i|/max={np.abs(r[i]).max() / np.abs(r).max():.2e})", flush=True)


def report(c, tag, variants=("own",)):
    """variants: own = the oracle's own forward state with the GPU images (the parity tests' setup so far);
    inject = the GPU forward's n_contrib mapped into the oracle state; fm = the same with the oracle's
    fast-math exp; spread = oracle(libm) vs oracle(fast-math exp), each on its own consistent state."""
    O.set_threads(16)
    args = Hh.oracle_args(c)
    ga = [g(a) for a in args] + [False]
    out = _C.rasterize_gaussians(*ga)
    K, color, alpha, normal, mdepth, radii = out[:6]
    H, W = c["H"], c["W"]
    gr = S.upstream_grads(H, W)
    gr["alpha"] = torch.randn(1, H, W, generator=torch.Generator().manual_seed(5)) * 1e-3
    gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gr["normal"]),
                                         alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7],
                                         out[8], out[9], c["require_depth"], False)
    gb = [t.cpu() for t in gb]
    op = c["inp"]["opacities"].numpy().reshape(-1)
    imgs = (alpha.cpu(), normal.cpu(), mdepth.cpu())
    first = True
    results = {}
    for mode in (0, 1):
        if not any(v in variants for v in (("own", "inject") if mode == 0 else ("fm", "spread"))):
            continue
        O.set_exp_mode(mode)
        t0 = time.time()
        o = O.forward(*args)
        tf = time.time() - t0
        if first:
            nc = _C.debug_n_contrib(out[8], H, W)
            print(f"== {tag}: K {K}/{o['num_rendered']} radii_eq={np.array_equal(radii.cpu().numpy(), o['radii'])} "
                  f"o>0.99: {(op > 0.99).sum()} oracle fwd {tf:.1f}s", flush=True)
            first = False
        def bwd(images):
            return O.backward(o["state"], *args[:19], gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], *images,
                              c["cam"].camera_center, o["radii"])
        if mode == 0 and "own" in variants:
            compare(gb, bwd(imgs), op, o["radii"], "oracle(libm exp) own n_contrib, GPU images")
        if mode == 1 and "spread" in variants:
            results["fm_own"] = bwd((o["alpha"], o["normal"], o["mdepth"]))
        if (mode == 0 and "inject" in variants) or (mode == 1 and "fm" in variants):
            mapped = Hh.gpu_n_contrib_for_oracle(out, o, H, W)
            own = o["state"].n_contrib()
            print(f"   n_contrib: GPU (mapped) != oracle at {(mapped != own).sum()} of {H * W} pixels", flush=True)
            o["state"].set_n_contrib(mapped)
            b = bwd(imgs)
            compare(gb, b, op, o["radii"], f"oracle({'fast-math' if mode else 'libm'} exp) GPU n_contrib + images")
        if mode == 0 and "spread" in variants:
            o2 = O.forward(*args)
            results["libm_own"] = O.backward(o2["state"], *args[:19], gr["color"], gr["mdepth"], gr["alpha"],
                                             gr["normal"], o2["alpha"], o2["normal"], o2["mdepth"],
                                             c["cam"].camera_center, o2["radii"])
    O.set_exp_mode(1)
    if "spread" in variants:
        compare([results["libm_own"][n] for n in NAMES], results["fm_own"], op, radii.cpu().numpy(),
                "SPREAD oracle(libm) vs oracle(fast-math), each on its own forward")


SMALL = [
    dict(P=40, W=40, H=24, seed=0),
    dict(P=300, W=64, H=48, seed=1),
    dict(P=500, W=100, H=70, seed=2, kernel_size=0.1),
    dict(P=400, W=61, H=53, seed=3, sgm=3, sg_degree=2),
    dict(P=300, W=64, H=48, seed=10, sgm=7, sg_degree=7),
    dict(P=400, W=64, H=48, seed=4, sh_degree=1),
    dict(P=400, W=64, H=48, seed=5, require_depth=False),
    dict(P=400, W=64, H=48, seed=6, bg=(0.3, 0.6, 0.9)),
    dict(P=10000, W=256, H=256, seed=7, log_scale=math.log(0.03)),
    dict(P=10000, W=256, H=256, seed=8, log_scale=math.log(0.03), require_depth=False),
    dict(P=2000, W=96, H=64, seed=12, flat=20.0),
    dict(P=400, W=64, H=48, seed=40, opacity_max_logit=6.0, opacity_std=3.0),
    dict(P=10000, W=256, H=256, seed=44, log_scale=math.log(0.03), opacity_max_logit=6.0, opacity_std=3.0),
    dict(P=400, W=64, H=48, seed=41, sh_degree=0, sh_max_degree=3),
    dict(P=400, W=64, H=48, seed=42, sh_degree=1, sh_max_degree=3),
    dict(P=400, W=64, H=48, seed=43, sh_degree=2, sh_max_degree=3),
]


def smoke_case():
    W, H, P = 128, 96, 2000
    return Hh.small_case(P=P, W=W, H=H, seed=0, z_range=(2.0, 5.0), log_scale=math.log(0.03), opacity_max_logit=9.0,
                         opacity_std=1.5)


def full(P, sg):
    W, H = 1920, 1080
    cam = S.make_camera(W, H)
    raw = S.make_gaussians(P, sg_degree=sg, aspect=H / W)
    inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    return dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=sg, kernel_size=0.0,
                require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))


if __name__ == "__main__":
    what = sys.argv[1:] or ["small"]
    if "small" in what:
        for case in SMALL:
            case = dict(case)
            ks = case.pop("kernel_size", 0.0)
            report(Hh.small_case(kernel_size=ks, **case), str(case))
        report(smoke_case(), "smoke")
    V = ("own", "inject", "fm", "spread")
    if "smallv" in what:
        for case in SMALL[8:13]:
            case = dict(case)
            ks = case.pop("kernel_size", 0.0)
            report(Hh.small_case(kernel_size=ks, **case), str(case), V)
    if "c3" in what:
        report(full(1_000_000, 0), "C3", V)
    if "c5" in what:
        report(full(5_000_000, 7), "C5", V)
