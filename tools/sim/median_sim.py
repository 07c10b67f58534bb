"""Development tool: median-depth root-finding strategies vs the reference
bisection on C3 contributor sets (CPU only; see median_sim.c).

python tools/sim/median_sim.py [tile_stride] [npass] [tol_rel] [maxit]"""
import ctypes, math, os, subprocess, sys
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), ROOT]
HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "median_sim.so")
subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-o", SO, os.path.join(HERE, "median_sim.c"),
                "-lm"], check=True)
import torch  # noqa: E402
import gsr_scene as S  # noqa: E402
from oracle import gsr_oracle as O  # noqa: E402
from tests import helpers as Hh  # noqa: E402

stride = int(sys.argv[1]) if len(sys.argv) > 1 else 41
if os.environ.get("SIM_CASE"):  # a tests/helpers.small_case scene, e.g. "P=600,W=16400,H=40,seed=9,log_scale=0.01"
    kw = {k: float(v) if "." in v else int(v) for k, v in (x.split("=") for x in os.environ["SIM_CASE"].split(","))}
    if "log_scale" in kw:
        kw["log_scale"] = math.log(kw["log_scale"])
    c = Hh.small_case(**kw)
    W, H, P = c["W"], c["H"], c["inp"]["means3D"].shape[0]
else:
    W, H, P = int(os.environ.get("SIM_W", 1920)), int(os.environ.get("SIM_H", 1080)), int(os.environ.get("SIM_P", 1_000_000))
    cam = S.make_camera(W, H)
    raw = S.make_gaussians(P, aspect=H / W)
    if os.environ.get('SIM_FLAT'):
        raw.scaling[:, 2] -= math.log(float(os.environ['SIM_FLAT']))
    inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    c = dict(bg=torch.zeros(3), inp=inp, cam=cam, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
             require_depth=True, tanx=math.tan(cam.FoVx / 2), tany=math.tan(cam.FoVy / 2))
O.set_threads(8)
O.set_tile_stride(100000)
o = O.forward(*Hh.oracle_args(c))
st = o["state"]
gx, gy = (W + 15) // 16, (H + 15) // 16
geo = st.geometry()
xy = np.ascontiguousarray(geo["means2D"].reshape(-1)); co = np.ascontiguousarray(geo["conic_opacity"].reshape(-1))
rp = np.ascontiguousarray(geo["ray_planes"].reshape(-1))
pl = st.binning()["point_list"]
rg = np.ascontiguousarray(st.tile_state()["ranges"].reshape(-1))
f = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
u32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
tiles = np.arange(0, gx * gy, stride, dtype=np.uint32)
sim = ctypes.CDLL(SO)
sim.sim_set_hnoise(ctypes.c_float(float(os.environ.get('SIM_HNOISE', '0'))))
sim.sim_set_halley(int(os.environ.get("SIM_HALLEY", "0")))
npass = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tol = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-6
maxit = int(sys.argv[4]) if len(sys.argv) > 4 else 10
wcost = float(os.environ.get('SIM_WCOST', '0.6'))
stats = np.zeros(64, np.float64)
sim.sim_set_pred(int(os.environ.get('SIM_SEL', '0')), ctypes.c_float(float(os.environ.get('SIM_SMAX', '1e30'))))
mr = np.zeros(len(tiles) * 256, np.float32); mn = np.zeros_like(mr)
if not os.environ.get("SIM_SKIP_RUN"):  # (a driver script may want the scene only)
    sim.sim_run(W, H, gx, len(tiles), u32(tiles), u32(rg), u32(pl), f(xy), f(co), f(rp), npass, ctypes.c_float(tol),
                maxit, ctypes.c_float(wcost), stats.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), f(mr), f(mn))
    px = stats[0]
    print(f"tiles {len(tiles)} pixels {px:.0f} in_range {stats[1]/px:.3f} mean blended {stats[10]/px:.1f} "
          f"non-ball frac {stats[11]/max(stats[10],1):.4f}")
    d = np.abs(mr.astype(np.float64) - mn)
    print(f"max|d| {d.max():.3e} rel-to-max {d.max()/np.abs(mr).max():.3e}  >1e-5: {(d > 1e-5).sum()}  "
          f"in_range mismatches {stats[8]:.0f}")
    print(f"walks mean {stats[4]/stats[1]:.2f} in-loop bisections {stats[7]:.0f} pass-fallback lanes {stats[9]:.0f}")
    print("walk hist", stats[12:28].astype(int).tolist())
    print("S bins (<=.25,.5,1,2,4,>4): lanes/fallbacks/mean walks", [(int(stats[32+3*b]), int(stats[33+3*b]), round(stats[34+3*b]/max(stats[32+3*b],1),2)) for b in range(6)])
    print(f"smooth waves {stats[50]/max(stats[51],1):.3f}")
    print(f"cost ref {stats[5]:.4e} strategy {stats[6]:.4e} ratio {stats[6]/stats[5]:.3f}")
    if os.environ.get("SIM_DUMP"):
        i = int(np.argmax(d))
        ti, rem = divmod(i, 256); wv, l = divmod(rem, 64)
        tile = int(tiles[ti]); px = (tile % gx) * 16 + (l & 15); py = (tile // gx) * 16 + wv * 4 + (l >> 4)
        print("worst pixel", px, py, "ref", mr[i], "new", mn[i])
        r = rp.reshape(-1, 4); T = 1.0; C = []
        for k in range(rg[2 * tile], rg[2 * tile + 1]):
            g = pl[k]; dx = xy[2*g]-px; dy = xy[2*g+1]-py; c4 = co[4*g:4*g+4]
            power = -0.5*(c4[0]*dx*dx+c4[2]*dy*dy)-c4[1]*dx*dy
            if power > 0: continue
            a = min(0.99, c4[3]*np.exp(power))
            if a < 1/255: continue
            if T*(1-a) < 1e-4: break
            tp = r[g,0]*dx+r[g,1]*dy+r[g,2]
            if T > 0.5: m0 = tp
            C.append((a, tp, r[g,3])); T *= 1-a
        C = np.array(C, np.float64)
        def Tv(t):
            a, tp, rs = C[:,0], C[:,1], C[:,2]; dd = (t-tp)*rs; g = np.exp(-0.5*dd*dd)
            return np.prod(np.where(t > tp, 1-a, 1-a*g)/np.sqrt(1-a*g))
        print("m0", m0, "n", len(C))
        for t in np.linspace(min(mr[i], mn[i]) - 1e-3, max(mr[i], mn[i]) + 1e-3, 15): print(f"  t={t:.6f} T={Tv(t):.6f}")
        near = np.argsort(np.abs(C[:,1]-mr[i]))[:6]
        print(C[near])
    if os.environ.get("SIM_DUMP"):
        def hd(t):
            a, tp, rs = C[:,0], C[:,1], C[:,2]; dd = (t-tp)*rs; g = np.exp(-0.5*dd*dd); ag = a*g; x = ag/(1-ag)
            before = ~(t > tp)
            A = np.prod(np.where(before, 1-ag, 1-a)); B = np.prod(1-ag)
            e = 0.5*rs*rs*x*(1-dd*dd*(1+x))
            return np.log(A)-0.5*np.log(B)+np.log(2), np.sum(-0.5*x*np.abs(dd)*rs), np.sum(np.where(before, e, -e))
        lo, hi = m0-0.4, m0+0.4
        for p in range(2):
            ts = lo + (hi-lo)/8*np.arange(9); hs = [hd(x)[0] for x in ts]
            i = 0
            for k in range(1, 8):
                if hs[k] >= 0: i = k
            print("pass", p, "h", np.round(hs, 4), "sid", i)
            lo, hi, hlo, hhi = ts[i], ts[i+1], hs[i], hs[i+1]
        t = lo + hlo/(hlo-hhi)*(hi-lo)
        for k in range(4):
            h0, d1, d2 = hd(t)
            if h0 >= 0: lo = t
            else: hi = t
            tn = t - 2*h0*d1/(2*d1*d1-h0*d2)
            print(k, t, h0, d1, d2, "->", tn, "bracket", lo, hi)
            if not (lo <= tn <= hi): tn = 0.5*(lo+hi)
            t = tn
