#!/usr/bin/env python3
"""64 B kernel rate vs allocation ORDER of its input (1 GiB) and output
(64 MiB) buffers, with and without a 24 GiB allocation alive."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

G, M = 1 << 30, 1 << 20
e = cgck.Engine(0)
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


def case(name, order):
    bufs = {}
    for what in order:
        sz = {"in": G, "out": 64 * M, "arena": 24 * G, "pad": 3 * M}[what]
        bufs[what] = cgck.DeviceBuffer(sz)
    e.synth_strided(bufs["in"].ptr, n, 64, 64, 5)
    e.sync()
    r = krate(bufs["in"].ptr, bufs["out"].ptr)
    print(f"{name:28s} in={bufs['in'].ptr:#x} out={bufs['out'].ptr:#x}: {r:.3f}", flush=True)
    for x in bufs.values():
        x.free()


for rep in range(2):
    case("in, out", ["in", "out"])
    case("out, in", ["out", "in"])
    case("arena, in, out", ["arena", "in", "out"])
    case("arena, out, in", ["arena", "out", "in"])
    case("in, arena, out", ["in", "arena", "out"])
    case("in, pad, out", ["in", "pad", "out"])
