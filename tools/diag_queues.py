"""Diagnostic: does the resident burst server hold up other streams' work?
Opens the server on one context (idle exit after 1 s), then times one small
launch + synchronise on each of 12 other contexts.  A call that waits for the
server's idle exit takes ~1 s: its stream shares the server's hardware queue."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "con-gen_amd")]
import cgck  # noqa: E402

engines = [cgck.Engine(0) for _ in range(13)]
buf = cgck.DeviceBuffer(4096 * 64)
out = cgck.DeviceBuffer(4 * 4096)
for e in engines:
    e.strided(buf.ptr, 4096, 64, 0, 64, cgck.GEN_BOTH, out.ptr)
    e.sync()
engines[0].burst_open(max_pkts=256, max_bytes=1 << 20, idle_ms=1000)
x = np.zeros(64, np.uint8)
x[0] = 0x45
worst = 0.0
for i, e in enumerate(engines[1:], 1):
    t0 = time.perf_counter()
    e.strided(buf.ptr, 4096, 64, 0, 64, cgck.GEN_BOTH, out.ptr)
    e.sync()
    dt = (time.perf_counter() - t0) * 1e3
    worst = max(worst, dt)
    print(f"context {i:2d}: launch + sync {dt:8.2f} ms", flush=True)
engines[0].burst_close()
print(f"worst {worst:.2f} ms ({'BLOCKED behind the server' if worst > 500 else 'no stream waits for the server'})")
for e in engines:
    e.close()
