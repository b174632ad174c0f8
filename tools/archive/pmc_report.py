#!/usr/bin/env python3
"""Per-kernel median counter values (per dispatch and per wave) from
gpurun_out/pmc_*/run_counter_collection.csv."""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "synth" in k or "rocclr" in k:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        agg[k]["_vgpr"].append(float(r["VGPR_Count"]))
for k, c in agg.items():
    m = {n: statistics.median(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 0) or 1
    print(k[:70])
    print("  dur %.1f us  vgpr %d  waves %d" % (m["_dur_us"], m["_vgpr"], w))
    for n in sorted(m):
        if n.startswith("_") or n == "SQ_WAVES":
            continue
        extra = ""
        if "CYCLES" in n or n.startswith("SQ_WAIT") or n.startswith("SQ_ACTIVE"):
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                extra = "  (%.2f of wave cycles)" % (m[n] / wc)
        print("   %-28s %14.4g  per-wave %10.1f%s" % (n, m[n], m[n] / w, extra))
