#!/usr/bin/env python3
"""Offline analysis of a burst-server failure dump (tests/memdiag.dump_failure):
which frame each wrong packet's values were computed from, and where its
wrong stores landed.

For every wrong packet k: its IP value v_ip = out[k] & 0xffff was stored at
a0' + 10 by the kernel (FILL) — so every place where the ring holds v_ip as a
little-endian u16 and the reference does not names a candidate a0'.  The
script matches those against the batch's frame starts (and reports the
offset from packet k's own), and recomputes packet k's values with the
oracle over every frame start of the batch to see whose bytes were read.

    python tools/analyze_failure.py gpurun_out/failures/<name>.npz [flags]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "con-gen_amd"), os.path.join(ROOT, "oracle")]


def main():
    f = np.load(sys.argv[1])
    flags = int(sys.argv[2]) if len(sys.argv) > 2 else 54
    out, exp, ver, ever, got, ref, desc = (f[k] for k in ("out", "exp", "ver", "ever", "got", "ref", "desc"))
    import cgck
    desc = desc.view(cgck.DESC_DTYPE) if desc.dtype != cgck.DESC_DTYPE else desc
    fo = desc["frame_off"].astype(np.int64) + desc["l3_off"]
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    bad_bytes = np.nonzero(got != ref)[0]
    print(f"ring at {int(f['ring_addr']):#x}; {len(bad)} wrong packets {bad[:4].tolist()}..{bad[-4:].tolist()}; "
          f"{len(bad_bytes)} wrong bytes in [{bad_bytes.min() if len(bad_bytes) else '-'}, "
          f"{bad_bytes.max() if len(bad_bytes) else '-'}]")
    # wrong bytes: in which frames, at which relative offsets
    owner = np.searchsorted(fo, bad_bytes, side="right") - 1
    rel = bad_bytes - fo[owner]
    print("wrong bytes by frame (frame: relative offsets):")
    for m in sorted(set(owner.tolist()))[:40]:
        print(f"  frame {m} (len {int(desc['ip_len'][m])}): {rel[owner == m].tolist()}")
    # per wrong packet: whose bytes give its output, and where its stores went
    gotw = got[:-1].astype(np.uint32) | (got[1:].astype(np.uint32) << 8)
    refw = ref[:-1].astype(np.uint32) | (ref[1:].astype(np.uint32) << 8)
    for k in bad[:24]:
        v = int(out[k])
        hits = [int(p) for p in np.nonzero((gotw == (v & 0xffff)) & (gotw != refw))[0]]
        cand = []
        for p in hits:
            a0 = p - 10
            m = np.nonzero(fo == a0)[0]
            cand.append((p, int(m[0]) if len(m) else None))
        # frames of the batch whose own values are these (frames do not overlap,
        # so exp[m] is what frame m's descriptor yields)
        src = np.nonzero(exp == v)[0].tolist()
        print(f"packet {k}: got {v:#010x} want {int(exp[k]):#010x}; IP value stored at {cand[:4]}; "
              f"same values from frame(s) {src[:4]}")


if __name__ == "__main__":
    main()
