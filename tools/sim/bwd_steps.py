"""Development tool (round 5): the render backward's walked (tile, entry) steps on the C3 scene
(median_sim.c sim_bwd_steps).  python tools/sim/bwd_steps.py [tile_stride]"""
import ctypes, os, runpy, sys
import numpy as np
stride = sys.argv[1] if len(sys.argv) > 1 else "7"
sys.argv = ["median_sim.py", stride, "0"]
os.environ.setdefault("SIM_SKIP_RUN", "1")
g = runpy.run_path(__file__.replace("bwd_steps.py", "median_sim.py"))
out = np.zeros(8)
g["sim"].sim_bwd_steps(g["W"], g["H"], g["gx"], len(g["tiles"]), g["u32"](g["tiles"]), g["u32"](g["rg"]),
                       g["u32"](g["pl"]), g["f"](g["xy"]), g["f"](g["co"]), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
n = out[0]
print(f"tiles {n:.0f}: max_contrib mean {out[1]/n:.1f}, walked steps mean {out[2]/n:.1f} "
      f"(x{len(g['tiles'])} sampled of {g['gx']*((g['H']+15)//16)} tiles), blending pixels per walked step {out[3]/max(out[2],1):.1f}")
