#!/usr/bin/env python3
"""A lab kernel family against the product family it would replace and the
oracle on strided batches, in one process on the lab build:

    CGCK_LIB=con-gen_amd/libcgck_lab.so python tools/lpd_check.py [ref,cand] [small|mtu]

(default lpa,lpd on the 64 B shapes; e.g. `group,dstr mtu` for the 1500 B
LDS-DMA dense stream kernel).
For every shape and flag set the two kernels' outputs must be identical, and
GEN_BOTH batches are also checked against the referee (every 7th packet).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cgck  # noqa: E402
import oracle  # noqa: E402


def main():
    P = oracle.port()
    ref, cand = (sys.argv[1] if len(sys.argv) > 1 else "lpa,lpd").split(",")
    preset = sys.argv[2] if len(sys.argv) > 2 else "small"
    engines = {}
    for v in (ref, cand):
        os.environ["CGCK_KERNEL"] = v
        engines[v] = cgck.Engine(0)
    os.environ.pop("CGCK_KERNEL", None)
    e0 = engines[ref]
    bad_total = 0
    shapes = [(16 << 20, 64, 64), (1000003, 64, 64), (777, 64, 64), (65, 64, 64), (1, 64, 64),
              (300001, 48, 44), (100000, 32, 20), (4097, 64, 52), (64 * 2048 + 5, 64, 64)]
    if preset == "mtu":
        shapes = [(16 << 20, 1500, 1500), (1000003, 1500, 1500), (777, 1500, 1500), (5, 1500, 1500),
                  (300001, 1504, 1499), (100000, 1024, 1000), (4097, 1516, 1516), (123457, 576, 576),
                  (4099, 1520, 1520), (3, 1500, 1500), (50001, 20, 20), (9999, 1500, 40)]
    if preset == "imix":   # descriptor batches: the synthetic IMIX set (BASELINE configs[3])
        for n in (16 << 20, 100003, 4097, 65, 1):
            nbytes = cgck.load().cgck_imix_bytes(n)
            buf, desc = cgck.DeviceBuffer(nbytes), cgck.DeviceBuffer(12 * n)
            e0.synth_imix(buf.ptr, desc.ptr, n, 0xC0C0 + n)
            outs = {v: cgck.DeviceBuffer(4 * n) for v in engines}
            for name, fl in (("GEN_BOTH", cgck.GEN_BOTH), ("RAW", cgck.RAW), ("VERIFY_BSD", cgck.VERIFY_BSD)):
                got = {}
                for v, e in engines.items():
                    e.set_desc_len_hint(nbytes // n)
                    e.desc(buf.ptr, desc.ptr, n, fl, outs[v].ptr)
                    got[v] = np.zeros(n, np.uint32)
                    outs[v].download(got[v], stream=e.stream)
                    e.sync()
                    kern = e.last_kernel
                diff = int(np.count_nonzero(got[ref] != got[cand]))
                chk = ""
                if name == "GEN_BOTH":
                    bad, cnt = P.check_synth_imix(n, 0xC0C0 + n, cgck.GEN_BOTH, got[cand], 7)
                    chk = f" oracle {bad}/{cnt}"
                    diff += bad
                bad_total += diff
                print(f"imix n={n} {name}: {cand} vs {ref} mismatches {diff}{chk} ({kern})", flush=True)
            for b in list(outs.values()) + [buf, desc]:
                b.free()
        shapes = []
    flag_sets = [("GEN_BOTH", cgck.GEN_BOTH), ("RAW", cgck.RAW), ("IP", cgck.IP),
                 ("L4", cgck.L4), ("GEN_NOPSEUDO", cgck.IP | cgck.L4 | cgck.L4_NOPSEUDO)]
    for n, stride, ln in shapes:
        buf = cgck.DeviceBuffer(n * stride + 64)
        e0.synth_strided(buf.ptr, n, stride, ln, 0xC0C0 + n)
        if n == 777:   # ihl != 5 in some packets: the general (not fast) path
            host = np.zeros(n * stride + 64, np.uint8)
            buf.download(host, stream=e0.stream)
            e0.sync()
            host[0:n * stride:stride][::3] = 0x46
            buf.upload(host, stream=e0.stream)
        outs = {v: cgck.DeviceBuffer(4 * n) for v in engines}
        for name, fl in flag_sets:
            got = {}
            for v, e in engines.items():
                e.strided(buf.ptr, n, stride, 0, ln, fl, outs[v].ptr)
                got[v] = np.zeros(n, np.uint32)
                outs[v].download(got[v], stream=e.stream)
                e.sync()
                kern = e.last_kernel
            diff = int(np.count_nonzero(got[ref] != got[cand]))
            chk = ""
            if name == "GEN_BOTH" and n != 777:
                bad, cnt = P.check_synth_strided(n, stride, ln, 0xC0C0 + n, cgck.GEN_BOTH, got[cand], 7)
                chk = f" oracle {bad}/{cnt}"
                diff += bad
            bad_total += diff
            print(f"n={n} stride={stride} len={ln} {name}: {cand} vs {ref} mismatches {diff}{chk} ({kern})", flush=True)
        for o in outs.values():
            o.free()
        buf.free()
    print("TOTAL_MISMATCHES", bad_total)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
