import runpy, sys, os
sys.argv = ["bench_sample.py", "10"]
sys.path.insert(0, "geometry-grounded-gaussian-splatting_amd")
from diff_gaussian_rasterization import _C
for d in (0, 1, 2, 3):
    _C.set_option(_C.OPT_BWD_NO_PREPASS, d)
    print("diag", d, flush=True)
    runpy.run_path("tools/bench_sample.py", run_name="__main__")
