"""Where does the batched Toeplitz hash's launch-by-launch drift come from
(187 -> 214 us over back-to-back launches in the bench's
rocprof pass)?  One process, no torch, per-launch HIP events:

  A  60 launches back to back on one input / output pair (the bench's shape)
  B  20 launches, each after 2 ms of host idle (the GPU idles between them)
  C  a second, freshly allocated pair: 60 launches back to back
  D  pair 1 again, outputs alternating between two buffers
  E  pair 1 again, 60 launches back to back (after all of the above)

    python tools/rss_steady.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

HBM = 8.0e12
KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
N = 64 << 20


def pair(eng):
    d = cgck.DeviceBuffer(N * 12 + 64)
    o = cgck.DeviceBuffer(4 * N)
    eng.synth_strided(d.ptr, (N * 12) // 1500, 1500, 1500, 0xC0C0)
    eng.sync()
    return d, o


def run(eng, d, outs, launches, idle_s=0.0):
    evs = [cgck.Event() for _ in range(launches + 1)]
    us = []
    for i in range(launches):
        eng.record(evs[i])
        eng.toeplitz(d.ptr, N, 12, 12, KEY, outs[i % len(outs)].ptr, mask=0x7F)
        if idle_s:
            eng.record(evs[i + 1])
            eng.sync()
            us.append(cgck.Engine.elapsed_ms(evs[i], evs[i + 1]) * 1e3)
            time.sleep(idle_s)
    if not idle_s:
        eng.record(evs[launches])
        eng.sync()
        us = [cgck.Engine.elapsed_ms(evs[i], evs[i + 1]) * 1e3 for i in range(launches)]
    return us


def show(tag, us):
    q = sorted(us)
    frac = [16 * N / (u * 1e-6) / HBM for u in us]
    print(f"{tag}: median {q[len(q) // 2]:.1f} us ({16 * N / (q[len(q) // 2] * 1e-6) / HBM:.3f}), "
          f"first5 {[round(u, 1) for u in us[:5]]}, last5 {[round(u, 1) for u in us[-5:]]}, "
          f"by tens {[round(sum(frac[i:i + 10]) / len(frac[i:i + 10]), 3) for i in range(0, len(frac), 10)]}",
          flush=True)


def main():
    eng = cgck.Engine(0)
    d1, o1 = pair(eng)
    show("A back-to-back, pair 1", run(eng, d1, [o1], 60))
    show("B 2 ms idle between, pair 1", run(eng, d1, [o1], 20, idle_s=0.002))
    d2, o2 = pair(eng)
    show("C back-to-back, pair 2 (fresh)", run(eng, d2, [o2], 60))
    show("D pair 1, outputs alternating", run(eng, d1, [o1, o2], 60))
    show("E back-to-back, pair 1 again", run(eng, d1, [o1], 60))
    show("F back-to-back, pair 2 again", run(eng, d2, [o2], 60))


if __name__ == "__main__":
    main()
