"""Ad-hoc GPU vs oracle comparison + rough timing (development tool)."""
import os, sys, time, math
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import gsr_scene as S, helpers as Hh
from oracle import gsr_oracle as O
from diff_gaussian_rasterization import _C

def run(P, W, H, require_depth=True, seed=0, **kw):
    c = Hh.small_case(P=P, W=W, H=H, seed=seed, require_depth=require_depth, **kw)
    args = Hh.oracle_args(c)
    o = O.forward(*args)
    dev = torch.device("cuda")
    g = lambda t: None if t is None else (t.to(dev) if isinstance(t, torch.Tensor) else t)
    ga = [g(a) for a in args] + [False]
    ga = [torch.Tensor([]) if a is None else a for a in ga]
    out = _C.rasterize_gaussians(*ga)
    torch.cuda.synchronize()
    K, color, alpha, normal, mdepth, radii = out[:6]
    print(f"P={P} {W}x{H} geom={require_depth}: K gpu={K} oracle={o['num_rendered']} radii mismatch={(radii.cpu().numpy()!=o['radii']).sum()}")
    for name, gt, ot in (("color", color, o["color"]), ("alpha", alpha, o["alpha"]), ("normal", normal, o["normal"]), ("mdepth", mdepth, o["mdepth"])):
        a = gt.cpu().numpy(); b = ot
        print(f"   {name}: relmax={Hh.rel_err(a,b):.3e} frac>1e-4={Hh.frac_bad(a,b,1e-4,1e-5):.2e}")
    gr = S.upstream_grads(H, W)
    b = O.backward(o["state"], *args[:19], gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], o["alpha"], o["normal"], o["mdepth"], c["cam"].camera_center, o["radii"])
    gb = _C.rasterize_gaussians_backward(*ga[:19], g(gr["color"]), g(gr["mdepth"]), g(gr["alpha"]), g(gr["normal"]), alpha, normal, mdepth, g(c["cam"].camera_center), radii, out[6], K, out[7], out[8], out[9], require_depth, False)
    names = ["dmeans2D","dcolors","dopacity","dmeans3D","dcov3D","dsh","dsg_axis","dsg_sharpness","dsg_color","dscales","drotations"]
    for n_, t in zip(names, gb):
        a = t.cpu().numpy(); bb = b[n_]
        if a.size:
            l2 = np.linalg.norm(a.astype(np.float64) - bb) / max(np.linalg.norm(bb), 1e-30)
            print(f"   {n_}: relmax={Hh.rel_err(a,bb):.3e} relL2={l2:.3e} frac>1e-3={Hh.frac_bad(a,bb,1e-3,1e-3*np.abs(bb).max()):.2e}")

def bench(P=1_000_000, W=1920, H=1080, require_depth=True, iters=10):
    dev = torch.device("cuda")
    cam = S.make_camera(W, H).to(dev)
    raw = S.make_gaussians(P, aspect=H/W)
    inp = {k: v.to(dev).contiguous() for k, v in S.activated_inputs(raw).items()}
    gr = {k: v.to(dev) for k, v in S.upstream_grads(H, W).items()}
    bg = torch.zeros(3, device=dev)
    tanx = math.tan(cam.FoVx/2); tany = math.tan(cam.FoVy/2)
    fa = (bg, inp["means3D"], torch.Tensor([]), inp["opacities"], inp["scales"], inp["rotations"], torch.Tensor([]), inp["shs"], inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], 3, 0, 1.0, cam.world_view_transform, cam.full_proj_transform, tanx, tany, 0.0)
    def step():
        out = _C.rasterize_gaussians(*fa, H, W, cam.camera_center, False, require_depth, False)
        K, color, alpha, normal, mdepth, radii = out[:6]
        gb = _C.rasterize_gaussians_backward(*fa, gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], alpha, normal, mdepth, cam.camera_center, radii, out[6], K, out[7], out[8], out[9], require_depth, False)
        return K
    for _ in range(3): K = step()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(iters): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / iters
    print(f"bench P={P} {W}x{H} geom={require_depth}: K={K} {dt*1e3:.2f} ms/iter = {1/dt:.1f} it/s")

if __name__ == "__main__":
    _C.set_option(_C.OPT_RENDER_STATS, 1)
    _C.debug_render_stats(True)
    bench(require_depth=True, iters=1)
    st = _C.debug_render_stats(True)
    _C.set_option(_C.OPT_RENDER_STATS, 0)
    print("stats per forward (4 calls):", [v / 4 for v in st[:4]],
          "lanes/step=%.1f far-frac passes2-5=%.3f" % (st[1] / max(st[0], 1), st[3] / max(st[2], 1)))
    run(20000, 320, 240)
    for npass in (-1, 1, 2, 3, 4, 0):
        _C.set_option(_C.OPT_BISECT_PASSES, npass)
        _C.timing_enable(True)
        bench(require_depth=True, iters=5)
        _C.timing_enable(False)
        st = _C.timing_collect()
        print("bisection passes", npass, "render_fwd ms", round(st["render_fwd"][0] / max(st["render_fwd"][1], 1), 3))
    _C.set_option(_C.OPT_BISECT_PASSES, 0)
    for nopre in (1, 0):
        _C.set_option(_C.OPT_BWD_NO_PREPASS, nopre)
        _C.timing_enable(True)
        bench(require_depth=True, iters=5)
        _C.timing_enable(False)
        st = _C.timing_collect()
        print("bwd no-prepass", nopre, "render_bwd ms", round(st["render_bwd"][0] / max(st["render_bwd"][1], 1), 3))
