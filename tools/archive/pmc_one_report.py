#!/usr/bin/env python3
"""Median per-dispatch counters of one kernel from tools/pmc_one.sh passes.

    python tools/pmc_one_report.py gpurun_out/pmc1_imixp_ KERNEL_SUBSTRING
"""
import csv
import glob
import statistics
import sys


def main():
    pre, kern = sys.argv[1], sys.argv[2]
    vals = {}
    for path in sorted(glob.glob(pre + "*/run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            if kern in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        print(f"{k:28s} {statistics.median(v):16.0f}")


if __name__ == "__main__":
    main()
