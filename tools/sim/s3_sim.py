"""Development tool: strategy S3 (probe walk, then Halley + two-sample verification walks) on C3
contributor sets; see median_sim.c sim_s3.  python tools/sim/s3_sim.py eps_rel [maxit]"""
import runpy, sys, ctypes, numpy as np
eps = float(sys.argv[1]); maxit = int(sys.argv[2]) if len(sys.argv) > 2 else 4
sys.argv = ["median_sim.py", "41", "2"]
g = runpy.run_path(__file__.replace("s3_sim.py", "median_sim.py"))
sim, tiles, f, u32 = g["sim"], g["tiles"], g["f"], g["u32"]
o = np.array([-0.2, -0.1, -0.05, -0.025, 0, 0.025, 0.05, 0.1, 0.2], np.float32)
out = np.zeros(32); d = np.zeros(len(tiles) * 256, np.float32)
sim.sim_s3(g["W"], g["H"], g["gx"], len(tiles), u32(tiles), u32(g["rg"]), u32(g["pl"]), f(g["xy"]), f(g["co"]),
           f(g["rp"]), len(o), f(o), ctypes.c_float(eps), maxit, ctypes.c_float(7e-6),
           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), f(d))
print(f"eps {eps}: lanes {out[0]:.0f} max|d| {out[1]:.3e} q99.9 {np.quantile(d[d>0], 0.999):.3e} fallbacks {out[2]:.0f} "
      f"mean wave rounds {out[4]/out[3]:.3f}")
print("lane rounds hist", out[5:21].astype(int).tolist())
