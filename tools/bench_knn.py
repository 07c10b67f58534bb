"""distCUDA2 timing (development / DESIGN numbers): 1M points of a clustered
cloud (the shape of an SfM initialisation), one JSON line."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
import numpy as np
import torch
from simple_knn._C import distCUDA2

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
rng = np.random.default_rng(3)
for P in (1_000_000, 5_000_000):
    centers = rng.uniform(-5, 5, size=(2000, 3))
    pts = torch.from_numpy((centers[rng.integers(0, 2000, P)] + 0.05 * rng.normal(size=(P, 3))).astype(np.float32))
    pts = pts.cuda()
    for _ in range(2):
        distCUDA2(pts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        distCUDA2(pts)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"what": f"distCUDA2, {P} clustered points", "ms_per_call": round(dt * 1e3, 3),
                      "Mpoints_per_s": round(P / dt / 1e6, 1)}), flush=True)
