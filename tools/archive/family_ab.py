#!/usr/bin/env python3
"""Same-process A/B of kernel families on descriptor batches (IMIX packed,
no layout hint; the same IMIX frames in ring slots): one context per family
(cgck_ctx_set_kernel), alternating blocks of launches on the same buffers,
every result checked against the oracle on a 1/64 sample.

    python tools/family_ab.py --families slot2,lpw --layouts packed,ring --rounds 5
"""
import argparse
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "con-gen_amd"), os.path.join(ROOT, "oracle")]
import cgck  # noqa: E402
import oracle  # noqa: E402

HBM = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", default="slot2,lpw")
    ap.add_argument("--layouts", default="packed,ring")
    ap.add_argument("--packets", type=int, default=16 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--stride", type=int, default=2048)
    ap.add_argument("--l3", type=int, default=14)
    ap.add_argument("--sring-len", type=int, default=576)
    a = ap.parse_args()
    n = a.packets
    P = oracle.port()
    fams = a.families.split(",")
    engs = {f: cgck.Engine(0, kernel=f) for f in fams}
    out = cgck.DeviceBuffer(4 * n)
    seed = 0xC0C0
    for lay in a.layouts.split(","):
        nbytes = cgck.load().cgck_imix_bytes(n)
        desc = cgck.DeviceBuffer(12 * n)
        if lay == "packed":
            buf = cgck.DeviceBuffer(nbytes)
            engs[fams[0]].synth_imix(buf.ptr, desc.ptr, n, seed)
        elif lay == "ring":
            buf = cgck.DeviceBuffer(n * a.stride)
            engs[fams[0]].synth_imix_ring(buf.ptr, desc.ptr, n, a.stride, a.l3, seed)
        else:  # sring: fixed-length frames of a strided batch in ring slots (cgck_strided)
            buf = cgck.DeviceBuffer(n * a.stride)
            engs[fams[0]].synth_strided(buf.ptr, n, a.stride, a.stride, seed)
            nbytes = n * a.sring_len
        algo = nbytes + (16 if lay != "sring" else 4) * n
        for e in engs.values():
            e.set_desc_len_hint(nbytes // n)
            e.sync()
        res = {f: [] for f in fams}
        kern = {}
        for r in range(a.rounds + 1):
            for f in (fams if r % 2 == 0 else fams[::-1]):
                e = engs[f]
                if lay == "sring":
                    def go(e=e):
                        e.strided(buf.ptr, n, a.stride, a.l3, a.sring_len, cgck.GEN_BOTH, out.ptr)
                else:
                    def go(e=e):
                        e.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
                go()
                e0, e1 = cgck.Event(), cgck.Event()
                e.record(e0)
                for _ in range(a.launches):
                    go()
                e.record(e1)
                e.sync()
                ms = cgck.Engine.elapsed_ms(e0, e1) / a.launches
                kern[f] = e.last_kernel
                if r > 0:
                    res[f].append(algo / (ms * 1e-3))
                if r == a.rounds:
                    o = np.zeros(n, np.uint32)
                    out.download(o, stream=e.stream)
                    e.sync()
                    if lay == "packed":
                        bad, chk = P.check_synth_imix(n, seed, cgck.GEN_BOTH, o, 64)
                    elif lay == "ring":
                        bad, chk = P.check_synth_ring(n, a.stride, a.l3, seed, cgck.GEN_BOTH, o, 64)
                    else:
                        bad, chk = 0, 0   # (random bytes at +l3: covered by the GPU tests)
                    kern[f] += f"  parity {chk - bad}/{chk}"
        for f in fams:
            m = statistics.median(res[f])
            print(f"{lay:>6} {f:>6}: {m / HBM:6.1%} of 8 TB/s (algorithmic {algo / 1e9:.2f} GB/launch)  {kern[f]}",
                  flush=True)
        buf.free()
        desc.free()


if __name__ == "__main__":
    main()
