#!/usr/bin/env python3
"""Per-layout rooflines from tools/gpu_prof_layouts.sh output (VERDICT r3
item 5): for each workload, the checksum kernel's rocprofv3 average
duration (trace_<w>/run_kernel_stats.csv), its algorithmic bytes per launch
(the one_workload.py line in trace_<w>.log), and its HBM bytes per launch
from the FETCH_SIZE / WRITE_SIZE passes (median per dispatch; bytes =
(2 x FETCH_SIZE + WRITE_SIZE) KB x 1024, the gfx950 correction bench.py
documents).  Writes summary.json next to them and prints a table.

    python tools/layout_rooflines.py profiles/r04/prof
"""
import csv
import json
import os
import re
import statistics
import sys

PEAK = 8.0e12
KERNELS = ("lpw_kernel", "dstr_kernel", "lpd_kernel", "slot2_kernel", "cksum_kernel", "lpa_kernel")


def main():
    d = sys.argv[1]
    out = {}
    for w in ("imixp", "imix", "ring", "1500", "64"):
        stats = os.path.join(d, f"trace_{w}", "run_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        kern, avg_ns, calls = None, None, 0
        for r in csv.DictReader(open(stats)):
            if any(k in r["Name"] for k in KERNELS):
                kern, avg_ns, calls = r["Name"], float(r["AverageNs"]), int(r["Calls"])
        m = re.search(r"algorithmic (\d+) B per launch", open(os.path.join(d, f"trace_{w}.log")).read())
        algo = int(m.group(1)) if m else None
        ctr = {}
        for c in ("fetch", "write"):
            p = os.path.join(d, f"{c}_{w}", "run_counter_collection.csv")
            if os.path.exists(p):
                for r in csv.DictReader(open(p)):
                    if kern and r["Kernel_Name"] == kern:
                        ctr.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        hbm = None
        if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
            hbm = (2 * statistics.median(ctr["FETCH_SIZE"]) + statistics.median(ctr["WRITE_SIZE"])) * 1024
        achieved = algo / (avg_ns * 1e-9) if algo and avg_ns else None
        out[w] = {"kernel": kern, "rocprof_avg_ms": avg_ns / 1e6 if avg_ns else None, "calls": calls,
                  "algorithmic_bytes": algo, "achieved_gbs": achieved / 1e9 if achieved else None,
                  "frac": achieved / PEAK if achieved else None, "hbm_bytes": hbm,
                  "traffic_over_algorithmic": hbm / algo if hbm and algo else None,
                  "hbm_frac": hbm / (avg_ns * 1e-9) / PEAK if hbm and avg_ns else None}
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(f"{'workload':8s} {'kernel':44s} {'avg ms':>8s} {'frac':>6s} {'traffic':>8s} {'HBM frac':>8s}")
    for w, r in out.items():
        print(f"{w:8s} {(r['kernel'] or '')[:44]:44s} {r['rocprof_avg_ms'] or 0:8.4f} {r['frac'] or 0:6.3f} "
              f"{r['traffic_over_algorithmic'] or 0:8.3f} {r['hbm_frac'] or 0:8.3f}")


if __name__ == "__main__":
    main()
