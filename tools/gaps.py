"""Print one step's kernel sequence with gaps from a rocprofv3 kernel trace (development tool).
python tools/gaps.py gpurun_out/<dir>/trace/run_kernel_trace.csv [anchor-kernel-substring]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "render_fwd"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
tot_gap = 0.0
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    tot_gap += gap
    print(f"{(s - t0) / 1000:9.1f} gap {gap:7.1f} dur {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:90]}")
    prev = e
print("total gap (us)", round(tot_gap, 1))
