"""Print per-kernel average duration and (optional) per-call counters from tools/ktrace.sh output."""
import csv, sys
from collections import defaultdict
d = sys.argv[1]
rows = []
for r in csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")):
    rows.append((float(r["AverageNs"]) / 1e3, int(r["Calls"]), r["Name"]))
rows.sort(reverse=True)
cnt = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(set))
try:
    for r in csv.DictReader(open(f"{d}/pmc/run_counter_collection.csv")):
        k = r["Kernel_Name"][:60]
        cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]].add(r["Dispatch_Id"])
except FileNotFoundError:
    pass
for us, c, name in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    k = name[:60]
    extra = " ".join(f"{cn}={v / max(1, len(n[k][cn])):.4g}" for cn, v in cnt.get(k, {}).items())
    print(f"{us:9.1f}us x{c:>4} {name[:70]:70s} {extra}")
