#!/usr/bin/env python3
"""Per-launch HBM traffic of the dominant kernel from separate rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_prof.sh), corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE (KB) reads exactly
half the bytes of a wide coalesced streaming read on gfx950, so it is
doubled; WRITE_SIZE (KB) is exact for 16-B/lane streaming stores.

    python tools/pmc_traffic.py gpurun_out/prof_fetch gpurun_out/prof_write OUT.json [BENCH.json]

With BENCH.json (a bench.py line) the kernel of each workload is the one the
dispatcher reported in that run (roofline*.kernel, extra.*.kernel).
"""
import csv
import json
import statistics
import sys

KERNELS = {
    "1500": "dstr_kernel<3, 16, true, 0>",
    "64": "lpd_kernel<2, 32, 2>",
    "imix": "lpw_kernel<true, 4, false>",
    "rss_hash": "toeplitz12x4_ab_kernel",
    "dst_cache": "dst_cache_kernel<true>",
}
# bench.py's batches: 16M packets; reads + 12 B descriptor (IMIX) + 4 B output
N = 16 << 20
IMIX_BYTES = 5944726220   # cgck_imix_bytes(16M)
ALGO = {"1500": N * 1504, "64": N * 68, "imix": IMIX_BYTES + 16 * N,
        "rss_hash": (64 << 20) * 16,            # bench.py RSS_TUPLES x (12 B read + 4 B written)
        "dst_cache": (4 * 256 * 60536 // 8) * 16}  # entries written (no input read); ~1/8 survive


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def kernels_from_bench(path):
    b = json.loads(open(path).read().strip().splitlines()[-1])
    k = dict(KERNELS)
    for key, field in (("1500", "roofline"), ("64", "roofline_64B"), ("imix", "roofline_imix")):
        if field in b and b[field].get("kernel"):
            k[key] = b[field]["kernel"]
    for key in ("rss_hash", "dst_cache"):
        v = b.get("extra", {}).get(key, {})
        if v.get("kernel"):
            k[key] = v["kernel"]
    return k


def main():
    global KERNELS
    if len(sys.argv) > 4:
        KERNELS = kernels_from_bench(sys.argv[4])
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {"method": "median per dispatch; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
           "source": [sys.argv[1], sys.argv[2]], "kernels": KERNELS}
    for key, frag in KERNELS.items():
        f = [v for k, v in fetch.items() if frag in k]
        w = [v for k, v in write.items() if frag in k]
        if not f or not w:
            continue
        fb = statistics.median(f[0]) * 1024 * 2
        wb = statistics.median(w[0]) * 1024
        res[f"bytes_per_launch_{key}"] = fb + wb
        res[f"read_bytes_{key}"] = fb
        res[f"write_bytes_{key}"] = wb
        if ALGO.get(key):
            res[f"traffic_over_algorithmic_{key}"] = (fb + wb) / ALGO[key]
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
