#!/usr/bin/env python3
"""64 B fast/slow state under counters: eight 1 GiB 64 B
batches allocated in a row in one process (the allocation pattern whose last
inputs read fast and first ones slow in tools/state_probe.py), each checksummed
by the lpa kernel LAUNCHES times in input order.  Prints the HIP-event rate of
every input; run under rocprofv3 --pmc to get the counters of each dispatch
(dispatch order = input order x launches).

    python tools/state_pmc.py [--ins 8] [--launches 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ins", type=int, default=8)
    ap.add_argument("--launches", type=int, default=3)
    a = ap.parse_args()
    n = 16 << 20
    e = cgck.Engine(0)
    ins = [cgck.DeviceBuffer(n * 64) for _ in range(a.ins)]
    out = cgck.DeviceBuffer(4 * n)
    for b in ins:
        e.synth_strided(b.ptr, n, 64, 64, 0xC0C0)
    e.sync()
    ev0, ev1 = cgck.Event(), cgck.Event()
    for k, b in enumerate(ins):
        e.record(ev0)
        for _ in range(a.launches):
            e.strided(b.ptr, n, 64, 0, 64, cgck.GEN_BOTH, out.ptr)
        e.record(ev1)
        ms = cgck.Engine.elapsed_ms(ev0, ev1) / a.launches
        print(f"input {k} @ {b.ptr:#x}: {n * 68 / (ms * 1e-3) / 8e12:.3f} of HBM peak ({ms:.4f} ms)", flush=True)
    print("kernel", e.last_kernel)


if __name__ == "__main__":
    main()
