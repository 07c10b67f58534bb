"""Times the fused PatchMatch terms (gsr_patchmatch._Terms: reprojection, masks
and the dense NCC, pm_terms_kernel) forward and backward on the e2e scene
(1M Gaussians, 1920x1080, the bench's two orbit views), with HIP events.

    python tools/bench_pm.py [P W H] [reps]     (GSR_LIB selects a library build)

Prints one JSON line: terms forward / backward ms, the two losses and the
mask counts (so two builds can be compared on the same inputs).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]

import torch  # noqa: E402

import gsr_train  # noqa: E402
from gaussian_renderer import render, sample_depth  # noqa: E402
import gsr_patchmatch as PM  # noqa: E402


def main():
    a = sys.argv[1:]
    P, W, H = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (1_000_000, 1920, 1080)
    reps = int(a[3]) if len(a) >= 4 else 20
    step, view, nearest = gsr_train.synthetic_training_setup(P, W, H, device="cuda", seed=0)
    g = step.g
    with torch.no_grad():
        pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
        md = pkg["median_depth"].contiguous()
        M = view.R.T.contiguous()
        intr = (float(view.Fx), float(view.Fy), float(view.Cx), float(view.Cy))
        pts = PM._Lift.apply(md, view.T, M, intr)
        s = sample_depth(pts, nearest, g, step.pipe, step.kernel_size)
    md_g = md.clone().requires_grad_(True)
    nrm_g = pkg["normal"].detach().clone().requires_grad_(True)
    pin_g = s["sampled_depth"].detach().clone().requires_grad_(True)
    consts = PM._Consts(view, nearest)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd, bwd = [], []
    for r in range(reps + 3):
        ev[0].record()
        geo, ncc = PM._Terms.apply(md_g, nrm_g, pin_g, s["inside"], consts)
        ev[1].record()
        torch.autograd.grad(geo + ncc, [md_g, nrm_g, pin_g])
        ev[2].record()
        torch.cuda.synchronize()
        if r >= 3:
            fwd.append(ev[0].elapsed_time(ev[1]))
            bwd.append(ev[1].elapsed_time(ev[2]))
    fwd.sort()
    bwd.sort()
    with torch.no_grad():
        out = PM._Terms.apply(md_g, nrm_g, pin_g, s["inside"], consts)
    print(json.dumps({"lib": os.environ.get("GSR_LIB", "default"), "terms_fwd_ms": round(fwd[len(fwd) // 2], 4),
                      "terms_bwd_ms": round(bwd[len(bwd) // 2], 4), "geo": float(out[0]), "ncc": float(out[1]),
                      "P": P, "W": W, "H": H}))


if __name__ == "__main__":
    main()
