"""Development tool (round 5): median_sim.c sim_cut — how much of a pixel's blended set the median-depth
walks must visit when the list is cut after the last contributor not far behind the first window.
python tools/sim/cut_sim.py [tile_stride] [K]"""
import ctypes, os, runpy, sys
import numpy as np
stride = sys.argv[1] if len(sys.argv) > 1 else "41"
K = float(sys.argv[2]) if len(sys.argv) > 2 else 6.5
sys.argv = ["median_sim.py", stride, "0"]
os.environ.setdefault("SIM_SKIP_RUN", "1")
g = runpy.run_path(__file__.replace("cut_sim.py", "median_sim.py"))
out = np.zeros(8)
g["sim"].sim_cut(g["W"], g["H"], g["gx"], len(g["tiles"]), g["u32"](g["tiles"]), g["u32"](g["rg"]), g["u32"](g["pl"]),
                 g["f"](g["xy"]), g["f"](g["co"]), g["f"](g["rp"]), ctypes.c_float(K),
                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
n = out[0]
print(f"in-range pixels {n:.0f}: blended {out[1]/n:.1f}, up to the cut {out[2]/n:.1f}, before the crossing "
      f"{out[3]/n:.1f}, far-behind inside the cut {out[4]/n:.1f}")
