#!/usr/bin/env python3
"""Where a lab kernel's outputs differ from lpa's (debug aid for A/B kernels):
    CGCK_LIB=con-gen_amd/libcgck_lab.so python tools/lpdw_debug.py REF CAND N STRIDE LEN"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))
import cgck  # noqa: E402

ref, cand, n, stride, ln = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:6])
eng = {}
for v in (ref, cand):
    os.environ["CGCK_KERNEL"] = v
    eng[v] = cgck.Engine(0)
buf = cgck.DeviceBuffer(n * stride + 64)
eng[ref].synth_strided(buf.ptr, n, stride, ln, 7)
got = {}
for v, e in eng.items():
    o = cgck.DeviceBuffer(4 * n)
    e.strided(buf.ptr, n, stride, 0, ln, cgck.GEN_BOTH, o.ptr)
    got[v] = np.zeros(n, np.uint32)
    o.download(got[v], stream=e.stream)
    e.sync()
    print(v, e.last_kernel)
bad = np.nonzero(got[ref] != got[cand])[0]
print("mismatches", len(bad))
if len(bad):
    runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
    for r in runs[:12]:
        print(f"  [{r[0]}, {r[-1]}] len {len(r)}  step {r[0] // 64}  cand {got[cand][r[0]]:#x} ref {got[ref][r[0]]:#x}")
