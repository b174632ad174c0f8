"""Toeplitz RSS row timing on one GPU: the batched
hash over dense 12-byte tuples in HBM, and the dst-cache build over a full
enumeration.  HIP events on the context stream.  Prints JSON lines.

    python tools/rss_bench.py [--n 16777216] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))

import numpy as np  # noqa: E402

import cgck  # noqa: E402

HBM_PEAK = 8.0e12
KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


def ev_time(eng, fn, reps, warm=3):
    for _ in range(warm):
        fn()
    eng.sync()
    a, b = cgck.Event(), cgck.Event()
    eng.record(a)
    for _ in range(reps):
        fn()
    eng.record(b)
    eng.sync()
    return cgck.Engine.elapsed_ms(a, b) / reps


def bench_hash(eng, n, reps):
    d = cgck.DeviceBuffer(n * 12 + 64)
    o = cgck.DeviceBuffer(4 * n)
    eng.synth_strided(d.ptr, (n * 12) // 1500, 1500, 1500, 0xC0C0)
    ms = ev_time(eng, lambda: eng.toeplitz(d.ptr, n, 12, 12, KEY, o.ptr, mask=0x7F), reps)
    algo = n * 16
    return {"kernel": "toeplitz12x4_ab_kernel<12>", "tuples": n, "ms": ms, "gtuple_s": n / ms / 1e6,
            "achieved_gbs": algo / ms / 1e6, "hbm_frac": algo / (ms * 1e-3) / HBM_PEAK}


def bench_dst(eng, nl, nf, qn, qi, cap, reps):
    key = np.frombuffer(KEY, np.uint8)
    p = cgck.Engine.dst_params((0x0A000001, 0x0A000000 + nl), (0x0A010000, 0x0A010000 + nf - 1),
                               0x5000, qn, qi, key)
    n = nl * nf * 60536
    out = cgck.DeviceBuffer(16 * min(cap, n))
    cnt = cgck.DeviceBuffer(4)
    ms = ev_time(eng, lambda: eng.dst_cache(p, out.ptr, min(cap, n), cnt.ptr), reps)
    c = np.zeros(1, np.uint32)
    cnt.download(c, stream=eng.stream)
    eng.sync()
    return {"kernel": "dst_cache_kernel<true>", "laddrs": nl, "faddrs": nf, "queue_num": qn,
            "cap": cap, "tuples": n, "written": int(c[0]), "ms": ms,
            "gtuple_s_scanned": n / ms / 1e6 if cap >= n else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64 << 20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch  # noqa: F401  (shares torch's HIP runtime, as bench.py does)
    eng = cgck.Engine(0)
    print(json.dumps({"hash": bench_hash(eng, a.n, a.reps)}), flush=True)
    print(json.dumps({"dst_full": bench_dst(eng, 4, 256, 8, 3, 1 << 31, a.reps)}), flush=True)
    print(json.dumps({"dst_default": bench_dst(eng, 1, 1, 4, 1, 100000, a.reps)}), flush=True)
    print(json.dumps({"dst_100k_of_16": bench_dst(eng, 1, 256, 16, 3, 100000, a.reps)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
