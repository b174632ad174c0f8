#!/usr/bin/env python3
"""64 B lane-per-packet kernel rate vs the relative placement of its input
(1 GiB of packets) and output (64 MiB of u32) inside one 24 GiB arena."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

G, M, K = 1 << 30, 1 << 20, 1 << 10
e = cgck.Engine(0)
big = cgck.DeviceBuffer(24 * G)
e.synth_strided(big.ptr, 24 * G // 64, 64, 64, 2)
e.sync()
a, b = cgck.Event(), cgck.Event()
n = G // 64


def krate(ip, op, reps=20):
    xs = []
    for _ in range(3):
        e.strided(ip, n, 64, 0, 64, cgck.GEN_BOTH, op)
        e.record(a)
        for _ in range(reps):
            e.strided(ip, n, 64, 0, 64, cgck.GEN_BOTH, op)
        e.record(b)
        xs.append(n * 68 / (cgck.Engine.elapsed_ms(a, b) / reps * 1e-3) / 8e12)
    return statistics.median(xs)


base = big.ptr + 2 * G
print(f"no output: {krate(base, 0):.3f}", flush=True)
for name, d in [("1G", G), ("1G+64M", G + 64 * M), ("2G", 2 * G), ("3G", 3 * G), ("8G", 8 * G),
                ("8G+256", 8 * G + 256), ("8G+4K", 8 * G + 4 * K), ("8G+64K", 8 * G + 64 * K),
                ("8G+1M", 8 * G + M), ("8G+2M", 8 * G + 2 * M), ("8G+16M", 8 * G + 16 * M),
                ("-1G", -G), ("-2G+4K", -2 * G + 4 * K), ("12G+32M", 12 * G + 32 * M)]:
    print(f"out = in + {name:8s}: {krate(base, base + d):.3f}", flush=True)
for name, d in [("in+1M", M), ("in+4K", 4 * K), ("in+256", 256)]:
    print(f"in shifted {name:6s}, out = in + 8G: {krate(base + d, base + 8 * G):.3f}", flush=True)
