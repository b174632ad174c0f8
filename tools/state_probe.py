#!/usr/bin/env python3
"""Where does the per-process fast/slow state of the 64 B batch come from
?  One process, one input batch, several contexts (each its
own HIP stream, hence possibly its own hardware queue), several input batches
(separate allocations) and several output buffers; 64 B rates per
(context, input, output) cell over repeated rounds.

    python tools/state_probe.py [--engines 4] [--ins 1] [--outs 2] [--rounds 6]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--ins", type=int, default=1)
    ap.add_argument("--outs", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--aligned", action="store_true",
                    help="extra inputs: 1 GiB windows at chosen offsets inside one 3 GiB allocation")
    a = ap.parse_args()
    n = 16 << 20
    G = 1 << 30
    engines = [cgck.Engine(0) for _ in range(a.engines)]
    allocs = [cgck.DeviceBuffer(n * 64) for _ in range(a.ins)]
    bufs = [(b.ptr, f"alloc {k}") for k, b in enumerate(allocs)]
    if a.aligned:
        big = cgck.DeviceBuffer(3 * G)
        allocs.append(big)
        base = (big.ptr + G - 1) // G * G
        for off, name in ((0, "1G-aligned"), (2 << 20, "1G+2M"), (64 << 10, "1G+64K"),
                          (big.ptr - base + G // 2 if big.ptr > base else G // 2, "1G+512M")):
            if base + off + n * 64 <= big.ptr + 3 * G:
                bufs.append((base + off, name))
    for p, _ in bufs:
        engines[0].synth_strided(p, n, 64, 64, 0xC0C0)
    outs = [cgck.DeviceBuffer(4 * n) for _ in range(a.outs)]
    engines[0].sync()
    ev0, ev1 = cgck.Event(), cgck.Event()
    res = {}
    for r in range(a.rounds):
        for i, e in enumerate(engines):
            for b, (bp, _) in enumerate(bufs):
                for j, o in enumerate(outs):
                    e.strided(bp, n, 64, 0, 64, cgck.GEN_BOTH, o.ptr)
                    e.record(ev0)
                    for _ in range(a.launches):
                        e.strided(bp, n, 64, 0, 64, cgck.GEN_BOTH, o.ptr)
                    e.record(ev1)
                    ms = cgck.Engine.elapsed_ms(ev0, ev1) / a.launches
                    res.setdefault((i, b, j), []).append(n * 68 / (ms * 1e-3) / 8e12)
        print(f"round {r}: " + "  ".join(f"e{k[0]}i{k[1]}o{k[2]} {v[-1]:.3f}" for k, v in res.items()),
              flush=True)
    for (i, b, j), xs in res.items():
        print(f"engine {i} in {b} ({bufs[b][1]} @ {bufs[b][0]:#x}, 1G offset {bufs[b][0] % G:#x}) out {j}: "
              f"median {statistics.median(xs):.3f} min {min(xs):.3f} max {max(xs):.3f}")


if __name__ == "__main__":
    main()
