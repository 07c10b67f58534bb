#!/usr/bin/env python3
"""Summarise rocprofv3 output of tools/profile.sh into profiles/.

  python tools/pmc_summary.py gpurun_out/prof_r1 profiles r1 [workload_key]

Writes
  profiles/<tag>_kernel_stats.csv   (rocprofv3 --kernel-trace --stats summary, copied)
  profiles/<tag>_stages.json        per-stage average duration and HBM bytes per launch
  profiles/pmc_<workload_key>.json  same content (key: bench.py's workload key, default C3);
                                    bench.py reads `traffic` and the VALU instruction count from it

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, in KiB; on gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
(Infinity-Cache hits are included in the fabric counters.)
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def stage_of(name: str) -> str | None:
    n = name
    if "preprocess_fwd_kernel" in n:
        return "preprocess"
    if "preprocess_bwd_kernel" in n:
        return "preprocess_bwd"
    if "emit_keys_kernel" in n:
        return "emit_keys"
    if "tile_ranges_kernel" in n:
        return "tile_ranges"
    if any(k in n for k in ("rows_count_kernel", "rows_emit_kernel", "tiles_setup_kernel", "tiles_count_kernel",
                            "tiles_emit_kernel", "tiles_emit_sorted_kernel", "tiles_emit_wide_kernel", "tiles_emit_coop_kernel",
                            "list_ranges_kernel")):
        return "tile_lists"
    if "render_fwd_kernel" in n or "tile_order_kernel" in n:  # (the forward's LPT order on small grids)
        return "render_fwd"
    if "render_bwd_kernel" in n:
        return "render_bwd"
    if "bwd_prepare_kernel" in n:
        return "bwd_clear"
    if "gather_counts_kernel" in n or "live_tiles_kernel" in n or "dsort_" in n:
        return "depth_order"
    if "count_k_hist_kernel" in n:
        return "scan"
    if "radix_sort" in n or "onesweep" in n or "merge_sort" in n:
        # rocPRIM kernels are named by key/value types: the tile sort has
        # 16-bit keys (grids <= 65536 tiles), the depth sort 32-bit keys
        return "sort" if "unsigned short" in n else "depth_order"
    if "scan" in n or "reduce" in n:
        return "scan"
    return None


def per_stage_counter(path: str, counter: str, n_calls: dict) -> dict:
    tot = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st:
            tot[st] += float(r["Counter_Value"])
    return {k: v / max(1, n_calls.get(k, 1)) for k, v in tot.items()}


def launches(path: str, counter: str) -> dict:
    """Number of forward / backward calls seen in a counter pass."""
    seen = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st:
            seen[st].add(r["Dispatch_Id"])
    calls = {k: len(v) for k, v in seen.items()}
    fwd = calls.get("preprocess", 1)
    bwd = calls.get("preprocess_bwd", 1)
    out = {}
    for k in calls:
        out[k] = bwd if k in ("render_bwd", "preprocess_bwd", "bwd_clear") else fwd
    return out


def short_name(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("gsr::", "")
    return n[:60]


def per_kernel(path: str, counter: str) -> dict:
    """Per kernel (short name): the counter's average per dispatch."""
    tot, seen = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not stage_of(r["Kernel_Name"]):
            continue
        k = short_name(r["Kernel_Name"])
        tot[k] += float(r["Counter_Value"])
        seen[k].add(r["Dispatch_Id"])
    return {k: v / max(1, len(seen[k])) for k, v in tot.items()}


def kernel_table(src: str) -> dict:
    """Per-kernel average duration (trace; each kernel's first dispatch skipped) and HBM bytes per
    dispatch (separate FETCH / WRITE passes, gfx950 correction), VALU instructions per dispatch."""
    durs = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        if stage_of(r["Kernel_Name"]):
            durs[short_name(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    f = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    sq_csv = os.path.join(src, "sq", "run_counter_collection.csv")
    valu = per_kernel(sq_csv, "SQ_INSTS_VALU") if os.path.exists(sq_csv) else {}
    active = per_kernel(sq_csv, "SQ_ACTIVE_INST_VALU") if os.path.exists(sq_csv) else {}
    trans = per_kernel(sq_csv, "SQ_INSTS_VALU_TRANS_F32") if os.path.exists(sq_csv) else {}
    out = {}
    for k, lst in durs.items():
        lst = sorted(lst[1:] or lst)
        out[k] = {"dispatches": len(lst), "median_us": round(lst[len(lst) // 2] / 1e3, 2),
                  "fetch_kib": None if k not in f else round(f[k], 1),
                  "write_kib": None if k not in w else round(w[k], 1),
                  "hbm_bytes": None if k not in f or k not in w else round((2.0 * f[k] + w[k]) * 1024.0),
                  "valu_insts": None if k not in valu else round(valu[k]),
                  "valu_trans_insts": None if k not in trans else round(trans[k]),
                  "valu_active": None if k not in active else round(active[k])}
    return out


def main():
    src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    key = sys.argv[4] if len(sys.argv) > 4 else "C3"
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    # average duration per stage call from the kernel trace (skip each stage's
    # first call: one-time initialisation inside the warm-up)
    dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        st = stage_of(r["Kernel_Name"])
        if st:
            dur[st].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    fetch_csv = os.path.join(src, "fetch", "run_counter_collection.csv")
    write_csv = os.path.join(src, "write", "run_counter_collection.csv")
    nf = launches(fetch_csv, "FETCH_SIZE")
    nw = launches(write_csv, "WRITE_SIZE")
    fetch = per_stage_counter(fetch_csv, "FETCH_SIZE", nf)
    write = per_stage_counter(write_csv, "WRITE_SIZE", nw)
    sq = {}
    for sub in ("sq", "sq2"):  # the SQ passes (each holds at most 8 SQ counters + GRBM_GUI_ACTIVE)
        sq_csv = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(sq_csv):
            continue
        ns = launches(sq_csv, "GRBM_GUI_ACTIVE")
        names = sorted({r["Counter_Name"] for r in csv.DictReader(open(sq_csv))})
        for cn in names:
            for st, v in per_stage_counter(sq_csv, cn, ns).items():
                sq.setdefault(st, {})[cn if cn != "GRBM_GUI_ACTIVE" or sub == "sq" else "GRBM_GUI_ACTIVE_sq2"] = v
    # memory-path pass (optional): L2 requests / busy / tag stalls and TA busy
    mem = {}
    for sub, counters in (("tcc", ("TCC_REQ_sum", "TCC_BUSY_avr", "TCC_TAG_STALL_sum", "TCC_HIT_sum",
                                   "GRBM_GUI_ACTIVE")),
                          ("ta", ("TA_BUSY_avr", "TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE"))):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        nm = launches(path, "GRBM_GUI_ACTIVE")
        for cn in counters:
            for st, v in per_stage_counter(path, cn, nm).items():
                mem.setdefault(st, {})[cn if cn != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE_{sub}"] = v
    stages = {}
    ncalls_trace = defaultdict(int)
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        if stage_of(r["Kernel_Name"]) == "preprocess":
            ncalls_trace["fwd"] += 1
        if stage_of(r["Kernel_Name"]) == "preprocess_bwd":
            ncalls_trace["bwd"] += 1
    for st, lst in dur.items():
        lst.sort()
        n = ncalls_trace["bwd" if st in ("render_bwd", "preprocess_bwd", "bwd_clear") else "fwd"]
        per_call = max(1, len(lst) // max(1, n))
        calls = [sum(d for _, d in lst[i:i + per_call]) for i in range(0, len(lst), per_call)]
        calls.sort()
        avg_ns = calls[len(calls) // 2]  # median call: robust to one-off stalls
        f = fetch.get(st)
        w = write.get(st)
        hbm = None if f is None or w is None else (2.0 * f + w) * 1024.0
        stages[st] = {"avg_call_ms": round(avg_ns / 1e6, 4), "max_call_ms": round(calls[-1] / 1e6, 4),
                      "calls": len(calls), "dispatches_per_call": per_call,
                      "fetch_kib_per_call": f, "write_kib_per_call": w, "hbm_bytes_per_launch": hbm}
        if st in mem:
            stages[st]["mem_per_call"] = mem[st]
        if st in sq:
            c = sq[st]
            stages[st]["sq_per_call"] = c
            # VALU issue fraction at the peak rate (MI355X_MICROARCH.md per-instruction
            # constants): a wave64 VALU instruction takes 2 SIMD-32 cycles when waves
            # interleave, a transcendental 4; over the SIMD-cycles of the call:
            # 256 CUs x 4 SIMDs x GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE is summed over
            # the 8 XCDs).  `valu_busy_1wave` prices them as one wave alone (4 / 8),
            # the rounds-1-3 convention, which is not a peak (it reads > 1 on some kernels).
            if c.get("GRBM_GUI_ACTIVE"):
                simd_cycles = 256 * 4 * c["GRBM_GUI_ACTIVE"] / 8.0
                n, tr = c.get("SQ_INSTS_VALU", 0.0), c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
                stages[st]["valu_busy"] = round((2.0 * n + 2.0 * tr) / simd_cycles, 4)
                stages[st]["valu_busy_1wave"] = round((4.0 * n + 4.0 * tr) / simd_cycles, 4)
                if c.get("SQ_WAVE_CYCLES"):
                    stages[st]["wait_inst_any_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
                    stages[st]["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
    out = {"tag": tag, "workload_key": key, "source": src,
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950)", "stages": stages,
           "kernels": kernel_table(src)}
    for name in (f"{tag}_stages.json", f"pmc_{key}.json"):
        with open(os.path.join(dst, name), "w") as fh:
            json.dump(out, fh, indent=1)
    for st, v in sorted(stages.items(), key=lambda kv: -kv[1]["avg_call_ms"]):
        print(f"{st:16s} {v['avg_call_ms']:8.3f} ms  hbm/call={v['hbm_bytes_per_launch']}  valu_busy={v.get('valu_busy')}")


if __name__ == "__main__":
    main()
