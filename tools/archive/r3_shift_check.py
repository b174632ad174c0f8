"""Round 3's failing values (GPUTEST_r03: test_burst_server_wide[True-600], the last
three outputs) recomputed with the oracle over page-shifted copies of the
same batch: which shift of the frames reproduces them.  Output kept in
profiles/r04/diag/r3_failure_shift.txt."""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ('tests', 'con-gen_amd', 'oracle')]
import oracle, cgck
from test_gpu_parity import random_batch
P = oracle.port()
rng = np.random.default_rng(77 + 4096 + 600)
buf, desc = random_batch(rng, 4096, 600)
size = (len(buf) + 4095) // 4096 * 4096
ring = np.zeros(size + (1 << 21), np.uint8)   # room for shifts either way
off0 = 1 << 20
ring[off0:off0 + len(buf)] = buf
got = [3420742490, 80486970, 1639029635]
for i, k in enumerate((4093, 4094, 4095)):
    d = desc[k:k + 1].copy()
    found = []
    for sh in range(-64, 65):          # shifts of whole 4 KiB pages
        dd = d.copy()
        dd["frame_off"] = np.uint64(int(d["frame_off"][0]) + off0 + sh * 4096)
        o, _ = P.batch_desc(ring.copy() if False else ring, dd.view(np.uint8), 1, 54)
        if int(o[0]) == got[i]:
            found.append(sh)
        # undo the FILL stores the oracle made on the shared ring
        ring[off0:off0 + len(buf)] = buf
        ring[:off0] = 0
        ring[off0 + len(buf):] = 0
    print("packet", k, "got", got[i], "matches FILL over the frame shifted by", [s * 4 for s in found], "KiB")
