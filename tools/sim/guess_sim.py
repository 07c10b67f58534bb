"""Development tool (round 5): how good is the composite's single-splat first guess of the median depth
(median_sim.c sim_guess) against the grid-neighbour mean?  python tools/sim/guess_sim.py [tile_stride]"""
import ctypes, os, runpy, sys
import numpy as np
stride = sys.argv[1] if len(sys.argv) > 1 else "41"
sys.argv = ["median_sim.py", stride, "0"]
os.environ.setdefault("SIM_SKIP_RUN", "1")
g = runpy.run_path(__file__.replace("guess_sim.py", "median_sim.py"))
sim, tiles, f, u32 = g["sim"], g["tiles"], g["f"], g["u32"]
out = np.zeros(80)
tol, loose, curv = (float(x) for x in os.environ.get("SIM_ACC", "3e-5,2e-4,0.02").split(","))
sim.sim_guess(g["W"], g["H"], g["gx"], len(tiles), u32(tiles), u32(g["rg"]), u32(g["pl"]), f(g["xy"]), f(g["co"]),
              f(g["rp"]), ctypes.c_float(tol), ctypes.c_float(loose), ctypes.c_float(curv),
              out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
n = out[0]
print(f"in-range pixels {n:.0f}: one walk accepted from the single-splat guess {out[1]/n:.3f}, "
      f"from the neighbour mean {out[2]/n:.3f}, either {out[19]/n:.3f}; guess within the window {out[20]/n:.3f}")
print("log10 rel error bins (<-7 .. >=-1): single", out[3:11].astype(int).tolist(), "neighbour", out[11:19].astype(int).tolist())
print(f"higher-order interpolation: {out[21]:.0f} off-grid pixels, one walk accepted {out[22]/max(out[21],1):.3f}; "
      f"error bins", out[23:31].astype(int).tolist())
print(f"two-level grid: {out[31]:.0f} even-grid pixels off the 4-grid, one walk from the 4-grid interpolation accepted "
      f"{out[32]/max(out[31],1):.3f}, within two walks {(out[32]+out[33])/max(out[31],1):.3f}")
print("  by 4-grid root spread (<1e-3, <1e-2, <3e-2, <0.1, >=0.1, incomplete grid): [pixels, accepted frac]",
      [(int(out[34 + 2 * b]), round(out[35 + 2 * b] / max(out[34 + 2 * b], 1), 3)) for b in range(6)])
print("  by 4-grid m0 spread (<1e-2, <2e-2, <5e-2, <0.1, >=0.1, incomplete): [pixels, accepted frac]",
      [(int(out[46 + 2 * b]), round(out[47 + 2 * b] / max(out[46 + 2 * b], 1), 3)) for b in range(6)])
