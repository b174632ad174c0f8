#!/usr/bin/env python3
"""Streaming-read ceiling on this MI355X: probe variants x buffer sizes,
interleaved in one process (HIP events).  Variant = $CGCK_KERNEL index
passed to cgck_probe_read: 0 grid-stride x8, 1 x8 nontemporal, 2 x16
(4 blocks/CU), 3 x4 (16 blocks/CU), 4 contiguous-per-block x8, 5 x8 with 32
blocks/CU.  Also times a fixed trivial launch to price the boundary."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

sizes = [int(x) << 20 for x in os.environ.get("PROBE_MB", "64,256,1024,4096,24000").split(",")]
variants = [int(x) for x in os.environ.get("PROBE_VARIANTS", "0,1,2,3,4,5").split(",")]
engines = {}
for v in variants:
    os.environ["CGCK_KERNEL"] = str(v)
    e = cgck.Engine(0)
    engines[v] = e
L = cgck.load()
for v, e in engines.items():   # family field carries the probe variant
    pass
buf = cgck.DeviceBuffer(max(sizes))
engines[variants[0]].synth_strided(buf.ptr, max(sizes) // 1500, 1500, 1500, 7)
sink = cgck.DeviceBuffer(max(4, max(sizes) // 16))   # iso variants store a u32 per 64 B
engines[variants[0]].sync()
a, b = cgck.Event(), cgck.Event()
res = {}
for r in range(6):
    for sz in sizes:
        reps = max(3, min(50, (8 << 30) // sz))
        for v, e in engines.items():
            e.probe_read(buf.ptr, sz, sink.ptr)
            e.record(a)
            for _ in range(reps):
                e.probe_read(buf.ptr, sz, sink.ptr)
            e.record(b)
            ms = cgck.Engine.elapsed_ms(a, b) / reps
            if r:
                res.setdefault((sz, v), []).append(ms)
for (sz, v), xs in sorted(res.items()):
    ms = statistics.median(xs)
    print(f"{sz >> 20:6d} MB variant {v}: {ms * 1e3:9.1f} us  {sz / ms / 1e9:8.2f} TB/s")
