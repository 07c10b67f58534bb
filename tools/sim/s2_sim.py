"""Development tool: strategy S2 (one multi-sample walk around m0, then
bracketed Halley walks) on C3 contributor sets; see median_sim.c sim_s2.
python tools/sim/s2_sim.py "off1,off2,..." [tol_rel] [tol_abs] [maxit] [hnoise]"""
import runpy, sys, ctypes, numpy as np
offs = [float(x) for x in sys.argv[1].split(",")]
tol_rel = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
tol_abs = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
maxit = int(sys.argv[4]) if len(sys.argv) > 4 else 6
hnoise = float(sys.argv[5]) if len(sys.argv) > 5 else 7e-6
sys.argv = ["median_sim.py", "41", "2"]
g = runpy.run_path(__file__.replace("s2_sim.py", "median_sim.py"))
sim, tiles, f, u32 = g["sim"], g["tiles"], g["f"], g["u32"]
out = np.zeros(64)
o = np.array(sorted(offs), np.float32)
sim.sim_s2(g["W"], g["H"], g["gx"], len(tiles), u32(tiles), u32(g["rg"]), u32(g["pl"]), f(g["xy"]), f(g["co"]),
           f(g["rp"]), len(o), f(o), ctypes.c_float(tol_rel), ctypes.c_float(tol_abs), maxit, ctypes.c_float(hnoise),
           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
print(f"offsets {offs}: lanes {out[0]:.0f} in_range mismatches {out[40]:.0f} mean walks {out[1]/max(out[0]-out[2],1):.2f} "
      f"fallback lanes {out[2]:.0f} max|d| {out[3]:.3e}")
print("wave max walks hist", out[6:22].astype(int).tolist(), "mean (fallback=100 capped)",
      round(float(np.sum(np.minimum(np.arange(16), 15) * out[6:22]) / out[4]), 2))
print("lane hist", out[22:38].astype(int).tolist())
