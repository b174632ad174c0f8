#!/usr/bin/env python3
"""In-process A/B of two libcgck.so builds on the BASELINE workloads.

Processes on one box land in one of two states for the store-carrying
workloads (64 B read 69 % in some processes and 78 % in
others with the same library), so comparing builds across processes mixes
the state into the result.  This loads both builds into ONE process (two
ctypes bindings, RTLD_LOCAL, one context each) and alternates them launch
block by launch block on the same device buffers.

    python tools/ab_inproc.py --libs con-gen_amd/libcgck_base.so,con-gen_amd/libcgck.so \\
        --workloads 64,imix,1500,rss --rounds 5
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

HBM = 8.0e12
# the bench's key (bench.py RSS_KEY, the Microsoft RSS test key); $AB_KEY=seq: bytes 7..46
KEY = (bytes(range(7, 7 + 40)) if os.environ.get("AB_KEY") == "seq" else
       bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True, help="two .so paths, comma separated")
    ap.add_argument("--workloads", default="64,imix,1500,rss")
    ap.add_argument("--packets", type=int, default=16 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    args = ap.parse_args()
    paths = args.libs.split(",")
    assert len(paths) == 2
    libs = [cgck.bind(p) for p in paths]
    ctxs = []
    for L in libs:
        c = ctypes.c_void_p()
        assert L.cgck_ctx_create(0, ctypes.byref(c)) == 0, L.cgck_last_error()
        ctxs.append(c)
    n = args.packets
    e0 = cgck.Engine(0)   # data set-up only (the default build)
    out = cgck.DeviceBuffer(16 * n)
    key = (ctypes.c_uint8 * len(KEY)).from_buffer_copy(KEY)
    work = {}
    keep = []
    for w in args.workloads.split(","):
        if w in ("imix", "imixp"):
            # imixp: the packed layout hint on both contexts (lpw)
            nbytes = cgck.load().cgck_imix_bytes(n)
            buf, desc = cgck.DeviceBuffer(nbytes), cgck.DeviceBuffer(12 * n)
            e0.synth_imix(buf.ptr, desc.ptr, n, 0xC0C0)
            for L, c in zip(libs, ctxs):
                L.cgck_set_desc_len_hint(c, nbytes // n)
            layout = cgck.LAYOUT_PACKED if w == "imixp" else cgck.LAYOUT_ANY
            pre = (lambda L, c, layout=layout: L.cgck_set_desc_layout(c, layout))
            # the layout hint is per context: set on every launch (imix and imixp share the contexts)
            work[w] = (lambda L, c, buf=buf, desc=desc, pre=pre: pre(L, c) or L.cgck_desc(
                c, buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr, None, None, None), nbytes + 16 * n)
            keep += [buf, desc]
        elif w == "ring":
            # the IMIX frames in 2048 B ring slots at +14 (cgck_synth_imix_ring)
            nbytes = cgck.load().cgck_imix_bytes(n)
            buf, desc = cgck.DeviceBuffer(2048 * n), cgck.DeviceBuffer(12 * n)
            e0.synth_imix_ring(buf.ptr, desc.ptr, n, 2048, 14, 0xC0C0)
            for L, c in zip(libs, ctxs):
                L.cgck_set_desc_len_hint(c, nbytes // n)
            work[w] = (lambda L, c, buf=buf, desc=desc: L.cgck_desc(
                c, buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr, None, None, None), nbytes + 16 * n)
            keep += [buf, desc]
        elif w == "rss":
            nt = 64 << 20
            buf = cgck.DeviceBuffer(12 * nt)
            # the bench's tuples (bench_rss): 1500 B synthetic records read as 12-byte
            # tuples, so the header bytes repeat rarely (64 B records repeat them every
            # 64 bytes, and the repeated table lookups broadcast)
            e0.synth_strided(buf.ptr, 12 * nt // 1500, 1500, 1500, 0xC0C0)
            work[w] = (lambda L, c, buf=buf, nt=nt: L.cgck_toeplitz(c, buf.ptr, nt, 12, 12, ctypes.addressof(key),
                                                                     len(KEY), 0x7F, out.ptr, None),
                       16 * nt)
            keep.append(buf)
        else:
            Lb = int(w)
            buf = cgck.DeviceBuffer(n * Lb)
            e0.synth_strided(buf.ptr, n, Lb, Lb, 0xC0C0)
            work[w] = (lambda L, c, buf=buf, Lb=Lb: L.cgck_strided(c, buf.ptr, n, Lb, 0, Lb, cgck.GEN_BOTH,
                                                                    out.ptr, None, None, None),
                       n * (Lb + 4))
            keep.append(buf)
    e0.sync()
    evs = []
    for L in libs:
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        L.cgck_event_create(ctypes.byref(a))
        L.cgck_event_create(ctypes.byref(b))
        evs.append((a, b))
    res = {(w, i): [] for w in work for i in range(2)}
    for r in range(args.rounds + 1):
        for w, (fn, algo) in work.items():
            order = (0, 1) if r % 2 == 0 else (1, 0)
            for i in order:
                L, c, (a, b) = libs[i], ctxs[i], evs[i]
                assert fn(L, c) == 0, L.cgck_last_error()
                L.cgck_event_record(c, a, None)
                for _ in range(args.launches):
                    fn(L, c)
                L.cgck_event_record(c, b, None)
                ms = ctypes.c_float()
                assert L.cgck_event_elapsed_ms(a, b, ctypes.byref(ms)) == 0
                if r > 0:
                    res[(w, i)].append(algo / (ms.value / args.launches * 1e-3))
    # parity of the two builds on every workload (the same outputs, byte for byte)
    import numpy as np
    same = {}
    for w, (fn, _) in work.items():
        got = []
        for L, c in zip(libs, ctxs):
            assert fn(L, c) == 0, L.cgck_last_error()
            assert L.cgck_ctx_sync(c) == 0
            h = np.zeros(16 * n, np.uint8)
            out.download(h)
            got.append(h)
        same[w] = bool(np.array_equal(got[0], got[1]))
    table = {}
    for w in work:
        m = [statistics.median(res[(w, i)]) for i in range(2)]
        table[w] = {"A": m[0] / HBM, "B": m[1] / HBM, "B_over_A": m[1] / m[0], "same_outputs": same[w]}
        print(f"{w:>5}: A {m[0] / HBM:6.1%}  B {m[1] / HBM:6.1%}  B/A {m[1] / m[0]:.3f}  same outputs {same[w]}",
              flush=True)
    print(json.dumps({"libs": paths, "results": table}))


if __name__ == "__main__":
    main()
