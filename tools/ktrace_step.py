"""Print one step's kernel timeline from a rocprofv3 kernel trace (development tool).
python tools/ktrace_step.py TRACE_CSV [anchor_kernel_substring] [call index from the end, default -8]"""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "preprocess_fwd"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
k = int(sys.argv[3]) if len(sys.argv) > 3 else -8  # which call (from the end): -8 is inside bench.py's timed loop (the last two forwards are its K and K_live readouts)
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev = t0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    short = name.split("(")[0][-60:]
    if "rocprim" in name:
        m = re.search(r"(onesweep_iteration|histogram|scan|reduce|lookback|init)", name)
        short = "rocprim " + (m.group(1) if m else "?")
    print(f"{(s - t0) / 1000:8.1f} us  gap {(s - prev) / 1000:6.1f}  dur {(e - s) / 1000:7.1f}  {short}")
    prev = e
