"""Per-component, per-kernel breakdown of the e2e training iteration.

run   (GPU box, under rocprofv3 --kernel-trace):
      python tools/e2e_breakdown.py run [steps]
      runs bench.py --e2e's TrainStep (1M Gaussians, 1080p) and launches a
      sentinel kernel (a float64 fill, which nothing else in the step uses) at
      every component boundary, so the trace splits into the components of
      gsr_train.TrainStep.COMPONENTS in stream order.
parse (anywhere):  python tools/e2e_breakdown.py parse KERNEL_TRACE_CSV [top]
      prints each component's kernel time per step with its kernels sorted
      by time (and writes the table as JSON next to the CSV)."""
import csv, json, os, re, sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SENTINEL = "FillFunctor<double>"


def run(steps: int):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    import torch
    import gsr_train

    dev = torch.device("cuda")
    ts, view, nearest = gsr_train.synthetic_training_setup(1_000_000, 1920, 1080, 3, 0, device=dev)
    for _ in range(5):
        ts.step(view, nearest)
    torch.cuda.synchronize()
    mark = torch.empty(1, dtype=torch.float64, device=dev)
    ts._mark = lambda: mark.fill_(1.0)  # noqa: E731  (the sentinel, in stream order)
    for _ in range(steps):
        ts.step(view, nearest)
    torch.cuda.synchronize()
    print(f"ran {steps} steps with sentinels")


def short(name: str) -> str:
    if "rocprim" in name:
        m = re.search(r"(onesweep_iteration|histogram|scan|reduce|lookback|init)", name)
        return "rocprim " + (m.group(1) if m else "?")
    if name.startswith("void at::native::") or name.startswith("at::native::"):
        m = re.findall(r"(\w+Functor\w*|\w+_kernel\w*|CatArray\w+|reduce_kernel|\w+Ops)", name)
        return "torch " + "/".join(dict.fromkeys(m[:3]))
    return name.split("(")[0].replace("void ", "")[:70]


def parse(path: str, top: int):
    sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    comps = ("render", "depth_normal", "patchmatch", "rgb_loss", "backward", "densify_stats", "adam")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if SENTINEL in r["Kernel_Name"]]
    per = len(comps) + 1
    steps = len(marks) // per
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    span = defaultdict(float)
    for s in range(steps):
        m = marks[s * per:(s + 1) * per]
        for c, name in enumerate(comps):
            a, b = m[c], m[c + 1]
            span[name] += (int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
            for r in rows[a + 1:b]:
                k = short(r["Kernel_Name"])
                acc[name][k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                calls[name][k] += 1
    out = {"steps": steps, "components": {}}
    for name in comps:
        ks = sorted(acc[name].items(), key=lambda kv: -kv[1])
        busy = sum(v for _, v in ks) / steps
        out["components"][name] = {"span_us": round(span[name] / steps, 1), "kernel_us": round(busy, 1),
                                   "kernels": [{"kernel": k, "us": round(v / steps, 1),
                                                "calls": calls[name][k] // steps} for k, v in ks]}
        print(f"== {name}: span {span[name] / steps:8.1f} us, kernels {busy:8.1f} us")
        for k, v in ks[:top]:
            print(f"   {v / steps:8.1f} us  x{calls[name][k] // steps:<3d} {k}")
    json.dump(out, open(os.path.splitext(path)[0] + "_e2e_breakdown.json", "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10)
    else:
        parse(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12)
