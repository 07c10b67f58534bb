"""Shared test helpers: small seeded scenes and tolerance checks."""
from __future__ import annotations

import math

import numpy as np
import torch

import gsr_scene as S


def small_case(P=40, W=40, H=24, seed=0, sh_degree=3, sg_degree=0, sgm=None, log_scale=math.log(0.12),
               opacity_max_logit=2.0, z_range=(2.0, 4.0), kernel_size=0.0, require_depth=True, cam=None,
               bg=(0.0, 0.0, 0.0), flat=1.0, opacity_std=1.0, sh_max_degree=None):
    """A small random scene plus every argument of _C.rasterize_gaussians.

    Opacity logits are capped at `opacity_max_logit` (default 2: sigmoid(2) =
    0.88, so o*G < 0.99); the clamp cases raise the cap (logit 6: o = 0.9975)
    so alpha = min(0.99, o*G) clamps and the reference's pass-through gradient
    of the clamp (render_backward.cu:931-933, 1012) is exercised.
    `sh_max_degree` > `sh_degree` gives the SH warm-up layout: 16 SH rows
    rendered at a lower active degree (train.py:130)."""
    cam = cam or S.make_camera(W, H)
    raw = S.make_gaussians(P, sh_degree=sh_degree, sg_degree=sgm if sgm is not None else sg_degree, seed=seed,
                           aspect=H / W, z_range=z_range, log_scale_mean=log_scale, log_scale_std=0.3,
                           opacity_std=opacity_std, sh_max_degree=sh_max_degree)
    raw.opacity.clamp_(max=opacity_max_logit)
    if flat != 1.0:  # surfel-like Gaussians: one axis `flat` times thinner (steep vacancy steps)
        raw.scaling[:, 2] -= math.log(flat)
    inp = S.activated_inputs(raw)
    inp = {k: v.detach().contiguous() for k, v in inp.items()}
    return dict(
        bg=torch.tensor(bg, dtype=torch.float32), inp=inp, cam=cam, W=W, H=H, sh_degree=sh_degree,
        sg_degree=sg_degree, kernel_size=kernel_size, require_depth=require_depth,
        tanx=math.tan(cam.FoVx * 0.5), tany=math.tan(cam.FoVy * 0.5), raw=raw)


def oracle_args(c, colors_precomp=None):
    inp = c["inp"]
    return (c["bg"], inp["means3D"], colors_precomp, inp["opacities"], inp["scales"], inp["rotations"], None,
            None if colors_precomp is not None else inp["shs"], inp["sg_axis"], inp["sg_sharpness"],
            inp["sg_color"], c["sh_degree"], c["sg_degree"], 1.0, c["cam"].world_view_transform,
            c["cam"].full_proj_transform, c["tanx"], c["tany"], c["kernel_size"], c["H"], c["W"],
            c["cam"].camera_center, False, c["require_depth"])


def rel_err(a, b) -> float:
    """max|a-b| / max|b| (0 if both are zero)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max() if b.size else 0.0
    num = np.abs(a - b).max() if a.size else 0.0
    return 0.0 if den == 0 and num == 0 else float(num / max(den, 1e-30))


def record_margins(fields: dict, what: str = "") -> None:
    """Parity margins: {field: (value, bar)} of one test
    case.  Prints the worst field against its bar and appends one JSON line
    per case to $GSR_MARGIN_LOG (default gpurun_out/parity_margins.jsonl at
    the repository root, when that directory can be written)."""
    import json
    import os
    if not fields:
        return
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
    worst = max(fields, key=lambda k: fields[k][0] / fields[k][1])
    v, bar = fields[worst]
    print(f"[margin] {test} {what}: worst {worst} {v:.3e} against {bar:.0e} ({bar / max(v, 1e-300):.1f}x headroom)")
    path = os.environ.get("GSR_MARGIN_LOG") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "gpurun_out", "parity_margins.jsonl")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, "what": what, "worst": worst, "value": v, "bar": bar,
                                "headroom": bar / max(v, 1e-300),
                                "fields": {k: [float(a), float(b)] for k, (a, b) in fields.items()}}) + "\n")
    except OSError:
        pass


def frac_bad(a, b, rtol, atol) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.mean(np.abs(a - b) > atol + rtol * np.abs(b)))


def gpu_n_contrib_for_oracle(out, o, H, W):
    """The GPU forward's per-pixel last contributors as positions in the
    oracle's per-tile lists.  The GPU lists are the oracle's (the reference's)
    minus the tile-culled instances, in the same order, so the
    last contributor's Gaussian is looked up in the oracle's list of its tile.
    With it (State.set_n_contrib) the oracle backward runs on exactly the GPU
    forward's state: its images and its contributor ranges."""
    from diff_gaussian_rasterization import _C

    plist, ranges = _C.debug_binning(out[7], out[9], out[0], H, W)
    last = _C.debug_n_contrib(out[8], H, W).astype(np.int64)
    ob = o["state"].binning()["point_list"].astype(np.int64)
    orng = o["state"].tile_state()["ranges"].astype(np.int64)
    gx = (W + 15) // 16
    ys, xs = np.mgrid[0:H, 0:W]
    tile = (ys // 16) * gx + (xs // 16)
    res = np.zeros((H, W), np.int64)
    has = last > 0
    g = plist.astype(np.int64)[ranges[tile[has], 0].astype(np.int64) + last[has] - 1]
    # per tile, the oracle positions of its Gaussians: search (tile, gaussian) keys in the oracle's list,
    # which is sorted per tile by depth, not id, so look up through a sorted copy
    otile = np.repeat(np.arange(orng.shape[0], dtype=np.int64), orng[:, 1] - orng[:, 0])
    okey = (otile << 32) | ob[np.concatenate([np.arange(a, b) for a, b in orng]) if len(ob) else np.zeros(0, np.int64)]
    opos = np.concatenate([np.arange(b - a) for a, b in orng]) if len(ob) else np.zeros(0, np.int64)
    srt = np.argsort(okey, kind="stable")
    want = (tile[has].astype(np.int64) << 32) | g
    at = np.searchsorted(okey[srt], want)
    assert np.array_equal(okey[srt][at], want), "GPU contributor missing from the oracle's tile list"
    res[has] = opos[srt][at] + 1
    return res.astype(np.uint32)


def free_port() -> int:
    """A free TCP port for a process group's rendezvous, outside the kernel's ephemeral range: a port picked
    by binding to port 0 is an ephemeral one, and the gloo connections an earlier multi-rank test left in
    their last states take ephemeral ports too — one was taken again between the pick and the ranks' bind
    (EADDRINUSE at the C5 8-rank test's rendezvous, round 6)."""
    import random
    import socket
    lo = 32768
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        pass
    rng = random.Random()
    for _ in range(256):
        p = rng.randrange(10000, max(10001, lo))
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
