"""Per-launch HIP-event trace of every bench.py leg on freshly allocated
buffers: does the 64 B, 1500 B and IMIX legs'
first ~40 launches run slower than their steady state, as RSS's did
(tools/rss_steady.py, profiles/r05/first/rss_steady.log)?  bench.py times
launches 6-25 by default (5 warm-ups, 20 steps).  One process, no torch:

  per leg: a fresh buffer pair (as bench.py allocates it), `--launches`
  launches back to back, then the frac of 8 TB/s (algorithmic bytes) by tens
  and over bench.py's window (launches 6-25) against launches 60+.

    python tools/steady.py [--launches 120] [--legs 1500,64,imix,ring]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
sys.path.insert(0, ROOT)
import cgck  # noqa: E402

HBM = 8.0e12
N = 16 << 20
SEED = 0xC0C0


def trace(eng, launch, launches):
    evs = [cgck.Event() for _ in range(launches + 1)]
    for i in range(launches):
        eng.record(evs[i])
        launch()
    eng.record(evs[launches])
    eng.sync()
    return [cgck.Engine.elapsed_ms(evs[i], evs[i + 1]) for i in range(launches)]


def show(tag, ms, algo, kernel):
    frac = [algo / (m * 1e-3) / HBM for m in ms]
    q = sorted(frac[60:]) if len(frac) > 60 else sorted(frac)
    win = frac[5:25]
    steady = q[len(q) // 2]
    print(f"{tag} [{kernel}]: bench window (launches 6-25) {sum(win) / len(win):.3f}, "
          f"steady (launches 61+, median) {steady:.3f}, window/steady {sum(win) / len(win) / steady:.3f}; "
          f"by tens {[round(sum(frac[i:i + 10]) / len(frac[i:i + 10]), 3) for i in range(0, len(frac), 10)]}",
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=120)
    ap.add_argument("--legs", default="1500,64,imix,ring")
    ap.add_argument("--repeat", type=int, default=1, help="fresh buffers per leg, one after the other")
    a = ap.parse_args()
    eng = cgck.Engine(0)
    for leg in a.legs.split(","):
        for rep in range(a.repeat):
            if leg in ("1500", "64"):
                size = int(leg)
                buf, out = cgck.DeviceBuffer(N * size), cgck.DeviceBuffer(4 * N)
                eng.synth_strided(buf.ptr, N, size, size, SEED)
                eng.sync()
                ms = trace(eng, lambda: eng.strided(buf.ptr, N, size, 0, size, cgck.GEN_BOTH, out.ptr), a.launches)
                show(f"{leg} B rep {rep}", ms, N * (size + 4), eng.last_kernel)
                buf.free()
                out.free()
            else:
                nbytes = cgck.load().cgck_imix_bytes(N)
                ring = leg == "ring"
                buf = cgck.DeviceBuffer(N * 2048 if ring else nbytes)
                desc, out = cgck.DeviceBuffer(12 * N), cgck.DeviceBuffer(4 * N)
                if ring:
                    eng.synth_imix_ring(buf.ptr, desc.ptr, N, 2048, 14, SEED)
                else:
                    eng.synth_imix(buf.ptr, desc.ptr, N, SEED)
                    eng.set_desc_layout(cgck.LAYOUT_PACKED)
                eng.set_desc_len_hint(nbytes // N)
                eng.sync()
                ms = trace(eng, lambda: eng.desc(buf.ptr, desc.ptr, N, cgck.GEN_BOTH, out.ptr), a.launches)
                show(f"IMIX {'ring' if ring else 'packed'} rep {rep}", ms, nbytes + 16 * N, eng.last_kernel)
                eng.set_desc_layout(cgck.LAYOUT_ANY)
                eng.set_desc_len_hint(1500)
                for b in (buf, desc, out):
                    b.free()


if __name__ == "__main__":
    main()
