"""Why does bench.py's RSS leg read ~0.58-0.65 of HBM peak when
tools/ab_inproc.py reads the same kernel at ~0.74?  Time the batched hash
the bench's way (cgck events around 20 launches after 5) under the
conditions that differ between the two harnesses, one at a time, in one
process:

    python tools/rss_harness.py [torch]

  order  "do": input then output allocated (bench_rss), "od": output first
  torch  the second pass after torch.cuda is initialised (the bench imports
         it and synchronises through it)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

HBM = 8.0e12
KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
N = 64 << 20


def one(eng, order, steps=20, warmup=5):
    if order == "do":
        d = cgck.DeviceBuffer(N * 12 + 64)
        o = cgck.DeviceBuffer(4 * N)
    else:
        o = cgck.DeviceBuffer(4 * N)
        d = cgck.DeviceBuffer(N * 12 + 64)
    eng.synth_strided(d.ptr, (N * 12) // 1500, 1500, 1500, 0xC0C0)
    eng.sync()
    for _ in range(warmup):
        eng.toeplitz(d.ptr, N, 12, 12, KEY, o.ptr, mask=0x7F)
    eng.sync()
    e0, e1 = cgck.Event(), cgck.Event()
    eng.record(e0)
    for _ in range(steps):
        eng.toeplitz(d.ptr, N, 12, 12, KEY, o.ptr, mask=0x7F)
    eng.record(e1)
    eng.sync()
    ms = cgck.Engine.elapsed_ms(e0, e1) / steps
    d.free()
    o.free()
    return ms, 16 * N / (ms * 1e-3) / HBM


def main():
    eng = cgck.Engine(0)
    for order in ("do", "od", "do", "od"):
        ms, f = one(eng, order)
        print(f"no torch  order {order}: {ms:.4f} ms  {f:.3f}", flush=True)
    for steps, warm in ((10, 1), (40, 5)):
        ms, f = one(eng, "do", steps, warm)
        print(f"no torch  order do, {steps} after {warm}: {ms:.4f} ms  {f:.3f}", flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "torch":
        import torch
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
        for order in ("do", "od"):
            ms, f = one(eng, order)
            print(f"torch     order {order}: {ms:.4f} ms  {f:.3f}", flush=True)


if __name__ == "__main__":
    main()
