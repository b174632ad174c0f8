"""Batch builders shared by the GPU parity tests of the descriptor kernels
(test_gpu_lpw.py, the lab-only test_gpu_span.py): packed (back-to-back)
frame batches of every length class, and the host-descriptor parity check
against the oracle referee."""
import numpy as np

import cgck

MIXES = {
    "imix": [64] * 7 + [576] * 4 + [1500],
    "small": list(range(0, 90)),                 # includes 0..19 (BAD_LEN) and odd lengths
    "mtu": [1500, 1499, 1514, 1480],             # 64 of them overflow one 64 KiB tile span
    "jumbo": [9000, 20000, 64, 65535, 40],       # tiles of one or two packets, the 64 KiB edge
    "wide": list(range(20, 1601, 7)),
}


def packed_batch(rng, n, lens, first_off=0):
    """Frames back to back in descriptor order: frame k+1's IPv4 header starts
    where frame k's ip_len bytes end (random l3_off inside each frame)."""
    L = rng.choice(np.asarray(lens), n)
    at = first_off
    offs = np.zeros(n, np.int64)
    for i in range(n):
        offs[i] = at
        at += int(L[i])
    buf = rng.integers(0, 256, at + 256, dtype=np.uint8)
    for i in range(n):
        o, ln = int(offs[i]), int(L[i])
        if ln < 1:
            continue
        r = rng.random()
        buf[o] = 0x40 | (5 if r < 0.7 else int(rng.integers(0, 16)))
        if ln > 9:
            buf[o + 9] = rng.choice([6, 6, 17, 1, int(rng.integers(0, 256))])
        if ln > 11 and rng.random() < 0.2:
            buf[o + 10:o + 12] = 0
        if ln >= 4:
            buf[o + 2], buf[o + 3] = (ln >> 8) & 0xFF, ln & 0xFF
    desc = np.zeros(n, cgck.DESC_DTYPE)
    l3 = np.minimum(rng.integers(0, 20, n), offs)
    desc["frame_off"] = offs - l3
    desc["l3_off"] = l3
    desc["ip_len"] = L
    return buf, desc


def run_packed(engine, port, buf, desc, flags):
    exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), len(desc), flags)
    got = buf.copy()
    out, ver = engine.run_host_desc(got, desc, flags)
    kernel = engine.last_kernel
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches, first {bad[:5]}: got {out[bad[:5]]} want {exp[bad[:5]]} "
                           f"len {desc['ip_len'][bad[:5]]}")
    return got, kernel
