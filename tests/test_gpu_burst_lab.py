"""Burst-server bookkeeping across the 32-bit seq wrap: runs
against libcgck_lab.so, whose cgck_lab_burst_poke restarts a server a few
seqs before the wrap with some workgroups' done words left stale (half the
seq space ahead, as a word untouched for 2^31 requests would compare).  The
first requests after it — narrow ones, which those workgroups have no slice
of — must bring every done word up to date, so the wide requests that
follow are not reported served before their slices are written; results
stay exact across the wrap.  tools/gpu_r5.sh runs it with CGCK_SERVER_OPTS=512
(every workgroup but the leader starts its slice 20 us late), so that its
control — the same run with the refresh switched off (opts 528) — fails
deterministically instead of by timing."""
import ctypes
import os

import numpy as np
import pytest

import cgck
from test_gpu_parity import check_burst, page_ring, random_batch

pytestmark = [pytest.mark.gpu, pytest.mark.lab]


@pytest.fixture(scope="module")
def lab():
    if not os.path.exists(cgck.LAB_PATH):
        pytest.skip("libcgck_lab.so not built (make -C tools lab)")
    saved = cgck.load()
    cgck._lib = cgck.bind(cgck.LAB_PATH)
    cgck._lib.cgck_lab_burst_poke.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    cgck._lib.cgck_lab_burst_stale.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    try:
        if cgck.device_count() < 1:
            pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
        e = cgck.Engine(0)
        yield e
        e.close()
    finally:
        cgck._lib = saved


@pytest.mark.parametrize("start", [0xFFFFFFF0, 0x7FFFFFF8, 1000])
def test_seq_wrap_and_stale_done_words(lab, port, start):
    L = cgck.load()
    raw, ring = page_ring(4 << 20)            # one registration: the server keeps running
    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    lab.burst_open(max_pkts=2048, max_bytes=4 << 20)
    try:
        assert L.cgck_lab_burst_poke(lab.ctx, start) == 0
        for k in range(40):                   # narrow (1 workgroup) and wide (up to 32) requests
            npk = (1, 40, 700, 2048)[k % 4]
            if k % 4 == 0 and k >= 4:
                # every workgroup but the leader left behind: the narrow
                # request next must bring their words up to date
                assert L.cgck_lab_burst_stale(lab.ctx, 1) == 0
            rng = np.random.default_rng(9100 + k + start % 977)
            buf, desc = random_batch(rng, npk, 300)
            assert len(buf) <= ring.nbytes
            flags = (cgck.GEN_BOTH, cgck.VERIFY_BSD, cgck.FILL_BOTH)[k % 3]
            ref = buf.copy()
            exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
            ring[:len(buf)] = buf
            got = ring[:len(buf)]
            out = np.full(npk, 0xDEADBEEF, np.uint32)
            ver = np.full(npk, 0xEE, np.uint8)
            lab.desc_host(got, desc, flags, out, ver)
            check_burst(out, exp, ver, ever, got, ref, f"start {start:#x} request {k} npk {npk}", 2048, ring, desc)
    finally:
        lab.burst_close()
        assert L.cgck_host_unregister(ring.ctypes.data) == 0
