#!/usr/bin/env python3
"""Does the placement of a device buffer change its streaming-read rate?
Reads 1 GiB with the plain read probe (variant 6) from: (a) a buffer that is
the process's first large allocation, (b) a buffer allocated after a 24 GiB
allocation, (c) regions carved from inside one 24 GiB arena."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

G = 1 << 30
os.environ["CGCK_KERNEL"] = os.environ.get("PROBE_VARIANT", "6")
e = cgck.Engine(0)
sink = cgck.DeviceBuffer(G // 16)
a, b = cgck.Event(), cgck.Event()


def rate(ptr, nbytes, reps=20):
    xs = []
    for _ in range(5):
        e.probe_read(ptr, nbytes, sink.ptr)
        e.record(a)
        for _ in range(reps):
            e.probe_read(ptr, nbytes, sink.ptr)
        e.record(b)
        xs.append(nbytes / (cgck.Engine.elapsed_ms(a, b) / reps * 1e-3) / 1e12)
    return statistics.median(xs)


first = cgck.DeviceBuffer(G)
e.synth_strided(first.ptr, G // 64, 64, 64, 1)
e.sync()
print(f"(a) first 1 GiB allocation: {rate(first.ptr, G):.2f} TB/s", flush=True)
big = cgck.DeviceBuffer(24 * G)
e.synth_strided(big.ptr, 24 * G // 1500, 1500, 1500, 2)
after = cgck.DeviceBuffer(G)
e.synth_strided(after.ptr, G // 64, 64, 64, 3)
e.sync()
print(f"(b) 1 GiB allocated after 24 GiB: {rate(after.ptr, G):.2f} TB/s", flush=True)
for off in (0, 8, 23):
    print(f"(c) 1 GiB at +{off} GiB inside the 24 GiB arena: {rate(big.ptr + off * G, G):.2f} TB/s", flush=True)
print(f"(d) the whole 24 GiB arena: {rate(big.ptr, 24 * G, reps=3):.2f} TB/s", flush=True)
print(f"(a') first allocation again: {rate(first.ptr, G):.2f} TB/s", flush=True)

# the 64 B lane-per-packet kernel with its u32 output, same placements
os.environ["CGCK_KERNEL"] = "auto"
k = cgck.Engine(0)
n = G // 64


def krate(ptr, optr, reps=20):
    xs = []
    for _ in range(5):
        k.strided(ptr, n, 64, 0, 64, cgck.GEN_BOTH, optr)
        k.record(a)
        for _ in range(reps):
            k.strided(ptr, n, 64, 0, 64, cgck.GEN_BOTH, optr)
        k.record(b)
        xs.append(n * 68 / (cgck.Engine.elapsed_ms(a, b) / reps * 1e-3) / 8e12)
    return statistics.median(xs)


out_small = cgck.DeviceBuffer(4 * n)
print(f"64B kernel: in=first out=after-arena      {krate(first.ptr, out_small.ptr):.3f} of peak", flush=True)
print(f"64B kernel: in=after-arena out=after-arena {krate(after.ptr, out_small.ptr):.3f}", flush=True)
print(f"64B kernel: in=arena+8G out=arena+20G      {krate(big.ptr + 8 * G, big.ptr + 20 * G):.3f}", flush=True)
print(f"64B kernel: in=first out=arena+20G         {krate(first.ptr, big.ptr + 20 * G):.3f}", flush=True)
print(f"64B kernel: in=arena+8G out=sink(first)    {krate(big.ptr + 8 * G, sink.ptr):.3f}", flush=True)
