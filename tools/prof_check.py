#!/usr/bin/env python3
"""rocprofv3 --stats average kernel duration vs bench.py's HIP-event time
per launch, for each workload's kernel (they must agree).

    python tools/prof_check.py KERNEL_STATS.csv BENCH.json
"""
import csv
import json
import sys


def main():
    stats = {r["Name"]: float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(sys.argv[1]))}
    b = json.loads(open(sys.argv[2]).read())
    rows = []
    for key, field in (("1500", "roofline"), ("64B", "roofline_64B"), ("imix", "roofline_imix")):
        if field in b:
            rows.append((key, b[field]["kernel"], b[field]["kernel_ms_hip_events"]))
    for k, v in b.get("extra", {}).items():
        if "kernel" in v and "kernel_ms" in v:
            rows.append((k, v["kernel"], v["kernel_ms"]))
    for key, kern, ev in rows:
        hits = [(n, ms) for n, ms in stats.items() if kern in n]
        if not hits:
            print(f"{key:10s} {kern:40s} not in the rocprof summary")
            continue
        n, ms = hits[0]
        print(f"{key:10s} {kern:40s} rocprof avg {ms:.4f} ms  HIP events {ev:.4f} ms  ratio {ms / ev:.3f}")


if __name__ == "__main__":
    main()
