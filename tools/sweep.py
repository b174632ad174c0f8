#!/usr/bin/env python3
"""In-process A/B of kernel families/variants on the BASELINE workloads.

Interleaves R rounds of K launches per (workload, variant) in ONE process on
ONE device (cdna_hip_programming.md §5.4 rule 24) and prints the median and
best HBM rate per cell.  Variants are selected through $CGCK_KERNEL at
context creation (auto | group | lpp).

    python tools/sweep.py [--packets N] [--rounds R] [--launches K]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

HBM = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=16 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--variants", default="group,lpp")
    ap.add_argument("--workloads", default="1500,64,imix")
    ap.add_argument("--flags", default="GEN_BOTH",
                    help="comma list of cgck flag names; each is a separate cell")
    ap.add_argument("--outs", default="out", help="comma list of out (u32 per packet) | none")
    args = ap.parse_args()
    n = args.packets
    flag_list = args.flags.split(",")
    out_list = args.outs.split(",")
    engines = {}
    for v in args.variants.split(","):
        os.environ["CGCK_KERNEL"] = v
        engines[v] = cgck.Engine(0)
    os.environ.pop("CGCK_KERNEL", None)
    e_probe = cgck.Engine(0)   # default family: probe variant 0 (plain streaming read)
    e0 = next(iter(engines.values()))
    work = {}
    nmax = n
    for w in args.workloads.split(","):
        if w.startswith("d"):
            # dense descriptor batch of one length: "d576" or "d576:NPACKETS"
            L, _, cnt = w[1:].partition(":")
            L, m = int(L), int(cnt) if cnt else n
            buf = cgck.DeviceBuffer(m * L)
            e0.synth_strided(buf.ptr, m, L, L, 0xC0C0)
            import numpy as np
            dh = np.zeros(m, cgck.DESC_DTYPE)
            dh["frame_off"] = np.arange(m, dtype=np.uint64) * L
            dh["ip_len"] = L
            desc = cgck.DeviceBuffer(12 * m)
            desc.upload(dh, stream=e0.stream)
            e0.sync()
            nmax = max(nmax, m)
            work[w] = (lambda e, f, o, buf=buf, desc=desc, m=m, L=L: (e.set_desc_len_hint(L),
                                                                       e.desc(buf.ptr, desc.ptr, m, f, o)),
                       m * (L + 12) + (4 * m if "out" in out_list else 0), [buf, desc])
        elif w in ("imix", "imixp"):
            # imixp: the SAME batch (same allocation: a different one can land
            # in another HBM state) with the packed layout hint;
            # imix: without it
            nbytes = cgck.load().cgck_imix_bytes(n)
            if "imix_bufs" not in locals():
                imix_bufs = (cgck.DeviceBuffer(nbytes), cgck.DeviceBuffer(12 * n))
                e0.synth_imix(imix_bufs[0].ptr, imix_bufs[1].ptr, n, 0xC0C0)
            buf, desc = imix_bufs
            algo = nbytes + 12 * n + (4 * n if "out" in out_list else 0)
            if w == "imixp":   # the packed layout hint (cgck_set_desc_layout)
                work[w] = (lambda e, f, o, buf=buf, desc=desc, h=nbytes // n: (
                    e.set_desc_len_hint(h), e.set_desc_layout(cgck.LAYOUT_PACKED), e.desc(buf.ptr, desc.ptr, n, f, o),
                    e.set_desc_layout(cgck.LAYOUT_ANY)), algo, [buf, desc])
            else:
                work[w] = (lambda e, f, o, buf=buf, desc=desc, h=nbytes // n: (
                    e.set_desc_len_hint(h), e.desc(buf.ptr, desc.ptr, n, f, o)), algo, [buf, desc])
        else:
            L = int(w)
            buf = cgck.DeviceBuffer(n * L)
            e0.synth_strided(buf.ptr, n, L, L, 0xC0C0)
            work[w] = (lambda e, f, o, buf=buf, L=L: e.strided(buf.ptr, n, L, 0, L, f, o),
                       n * L + (4 * n if "out" in out_list else 0), [buf])
    out = cgck.DeviceBuffer(4 * nmax)
    # streaming-read ceiling on the 1500 B buffer (or the first one)
    pb = work.get("1500", next(iter(work.values())))[2][0]
    sink = cgck.DeviceBuffer(4)
    work["probe"] = (lambda e, f, o, pb=pb: e.probe_read(pb.ptr, pb.nbytes, sink.ptr), pb.nbytes, [pb])
    e0.sync()
    cells = {}
    for v, e in engines.items():
        for fl in flag_list:
            for o in out_list:
                tag = v if (len(flag_list) == 1 and len(out_list) == 1) else f"{v}:{fl}:{o}"
                cells[tag] = (e, getattr(cgck, fl), out.ptr if o == "out" else 0)
    first = next(iter(cells))
    res = {(w, v): [] for w in work for v in cells if w != "probe" or v == first}
    a, b = cgck.Event(), cgck.Event()
    for r in range(args.rounds + 1):
        for w, (fn, algo, _) in work.items():
            for v, (e, fl, o) in cells.items():
                if (w, v) not in res:
                    continue
                ee = e_probe if w == "probe" else e
                fn(ee, fl, o)  # warm
                ee.record(a)
                for _ in range(args.launches):
                    fn(ee, fl, o)
                ee.record(b)
                ms = cgck.Engine.elapsed_ms(a, b) / args.launches
                if r > 0:
                    res[(w, v)].append(algo / (ms * 1e-3))
    table = {}
    for (w, v), xs in res.items():
        med, best = statistics.median(xs), max(xs)
        table[f"{w}/{v}"] = {"median_GBs": med / 1e9, "best_GBs": best / 1e9,
                             "median_frac": med / HBM}
        print(f"{w:>12} {v:>22}: median {med / 1e9:8.1f} GB/s ({med / HBM:6.1%})  best {best / 1e9:8.1f}",
              flush=True)
    print(json.dumps(table))


if __name__ == "__main__":
    main()
