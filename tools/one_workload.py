#!/usr/bin/env python3
"""Launch one workload a few times (for rocprofv3 --pmc passes over a single
kernel): imix | imixp (packed layout hint) | ring (IMIX in 2048 B slots) | 64 | 1500.

    python tools/one_workload.py imixp [--launches 5] [--kernel FAMILY]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--packets", type=int, default=16 << 20)
    a = ap.parse_args()
    n = a.packets
    e = cgck.Engine(0)
    out = cgck.DeviceBuffer(4 * n)
    ev0, ev1 = cgck.Event(), cgck.Event()
    if a.workload == "ring":   # the IMIX frames in 2048 B ring slots at +14
        nbytes = cgck.load().cgck_imix_bytes(n)
        buf = cgck.DeviceBuffer(2048 * n)
        desc = cgck.DeviceBuffer(12 * n)
        e.synth_imix_ring(buf.ptr, desc.ptr, n, 2048, 14, 0xC0C0)
        e.set_desc_len_hint(nbytes // n)
        algo = nbytes + 16 * n

        def fn():
            e.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    elif a.workload in ("imix", "imixp"):
        nbytes = cgck.load().cgck_imix_bytes(n)
        buf = cgck.DeviceBuffer(nbytes)
        desc = cgck.DeviceBuffer(12 * n)
        e.synth_imix(buf.ptr, desc.ptr, n, 0xC0C0)
        e.set_desc_len_hint(nbytes // n)
        if a.workload == "imixp":
            e.set_desc_layout(cgck.LAYOUT_PACKED)
        algo = nbytes + 16 * n

        def fn():
            e.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    else:
        L = int(a.workload)
        buf = cgck.DeviceBuffer(n * L)
        e.synth_strided(buf.ptr, n, L, L, 0xC0C0)
        algo = n * (L + 4)

        def fn():
            e.strided(buf.ptr, n, L, 0, L, cgck.GEN_BOTH, out.ptr)
    e.sync()
    fn()
    e.record(ev0)
    for _ in range(a.launches):
        fn()
    e.record(ev1)
    ms = cgck.Engine.elapsed_ms(ev0, ev1) / a.launches
    print(f"{a.workload}: {e.last_kernel} {ms:.4f} ms  {algo / (ms * 1e-3) / 8e12:.3f} of HBM peak  "
          f"algorithmic {algo} B per launch", flush=True)


if __name__ == "__main__":
    main()
