"""Development tool: strategy S4 (grid pixels by probe walk + Halley, the others by Halley from their grid
neighbours' roots) on C3 contributor sets; see median_sim.c sim_s4.  python tools/sim/s4_sim.py [tol_rel] [maxit]"""
import os, runpy, sys, ctypes, numpy as np
tol = float(sys.argv[1]) if len(sys.argv) > 1 else 3e-5
maxit = int(sys.argv[2]) if len(sys.argv) > 2 else 4
sys.argv = ["median_sim.py", os.environ.get("SIM_STRIDE", "41"), "2"]
g = runpy.run_path(__file__.replace("s4_sim.py", "median_sim.py"))
sim, tiles, f, u32 = g["sim"], g["tiles"], g["f"], g["u32"]
import os
sim.sim_set_loose(ctypes.c_float(float(os.environ.get("SIM_LOOSE", "0"))),
                  ctypes.c_float(float(os.environ.get("SIM_TOLF", "1e-6"))))
o = np.array([float(x) for x in os.environ.get("SIM_OFFS", "-0.2,-0.1,-0.05,-0.025,0,0.025,0.05,0.1,0.2").split(",")],
             np.float32)
out = np.zeros(48)
sim.sim_s4(g["W"], g["H"], g["gx"], len(tiles), u32(tiles), u32(g["rg"]), u32(g["pl"]), f(g["xy"]), f(g["co"]),
           f(g["rp"]), len(o), f(o), ctypes.c_float(tol), maxit, ctypes.c_float(float(os.environ.get("SIM_HN", "7e-6"))),
           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
print(f"tol {tol}: lanes {out[0]:.0f} max|d| {out[1]:.3e} fallbacks {out[2]:.0f} no-guess {out[24]:.0f}")
print(f"phase-1 wave max walks {out[3]/out[4]:.2f}  phase-2 wave max walks {out[5]/out[6]:.2f} (fallback=100)")
print("phase-2 lane walks hist", out[8:24].astype(int).tolist())
print("phase-1 lane walks hist (SIM_P1)", out[25:32].astype(int).tolist())
print("phase-1 grid pixel Halley walks hist [0..7+]", out[32:40].astype(int).tolist(), "stragglers", int(out[40]), "their 2b walks", int(out[41]), "unbracketed", int(out[42]))
why = (ctypes.c_long * 11)()
sim.sim_why(why)
print("halley outcomes: ok", why[0], "ill-conditioned", why[1], "not converged", why[2], "ill D*scale log10 bins from -4:", list(why[3:11]))
