"""Debug: the aten ops of one e2e training iteration with their input shapes
and device time (torch.profiler), to find the torch glue left around the HIP
kernels (zero fills, gradient accumulation).  Development only.

    python tools/dbg/e2e_ops.py [P W H]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import gsr_train  # noqa: E402

a = sys.argv[1:]
P, W, H = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (1_000_000, 1920, 1080)
ts, view, nearest = gsr_train.synthetic_training_setup(P, W, H, 3, 0, device="cuda")
for _ in range(5):
    ts.step(view, nearest)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    ts.step(view, nearest)
    torch.cuda.synchronize()
keys = ("aten::zeros", "aten::zero_", "aten::fill_", "aten::add", "aten::add_", "aten::mul", "aten::copy_", "aten::cat",
        "aten::sum", "aten::neg", "aten::where", "aten::sub", "aten::div", "aten::clone", "aten::contiguous",
        "aten::zeros_like", "aten::ones_like", "aten::empty_like", "aten::sign", "aten::mean", "aten::abs")
tab = prof.key_averages(group_by_input_shape=True)
rows = [e for e in tab if e.key in keys]
rows.sort(key=lambda e: -e.device_time_total)
print(f"{'op':22s} {'calls':>5s} {'device us':>10s}  shapes")
for e in rows[:60]:
    print(f"{e.key:22s} {e.count:5d} {e.device_time_total:10.1f}  {str(e.input_shapes)[:150]}")
print()
print(prof.key_averages().table(sort_by="device_time_total", row_limit=40, max_name_column_width=60))
print()
# where the glue comes from: python call sites of the fills and elementwise ops
for e in sorted(prof.key_averages(group_by_stack_n=6), key=lambda e: -e.device_time_total):
    if e.key in ("aten::zero_", "aten::mul", "aten::add_", "aten::add", "aten::sub", "aten::where", "aten::mean",
                 "aten::sum", "aten::clone", "aten::div", "aten::neg", "aten::abs") and e.device_time_total > 4:
        print(f"{e.key:14s} {e.count:3d} {e.device_time_total:8.1f} us")
        for fr in e.stack[:6]:
            print("      ", fr)
