"""Burst-server bookkeeping across the 32-bit seq wrap, in the
product gate: libcgck.so's test hooks (include/cgck.h) restart a server a few
seqs before the wrap (cgck_test_burst_seq) and leave some workgroups' done
words stale (cgck_test_burst_stale: half the seq space ahead, as a word
untouched for 2^31 requests would compare).  The first requests after it —
narrow ones, which those workgroups have no slice of — must bring every done
word up to date, so the wide requests that follow are not reported served
before their slices are written; results stay exact across the wrap.

tests/test_gpu_burst_lab.py runs the same body against the lab build with
every workgroup but the leader starting its slice 20 us late
(CGCK_SERVER_OPTS=512), and its control with the refresh switched off
(opts 528) fails deterministically (tools/gpu_r6.sh `lab`)."""
import ctypes

import numpy as np
import pytest

import cgck
from test_gpu_parity import check_burst, page_ring, random_batch

pytestmark = pytest.mark.gpu


def bind_hooks(L):
    L.cgck_test_burst_seq.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.cgck_test_burst_stale.argtypes = [ctypes.c_void_p, ctypes.c_uint32]


def wrap_body(eng, port, start):
    L = cgck.load()
    bind_hooks(L)
    raw, ring = page_ring(4 << 20)            # one registration: the server keeps running
    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    eng.burst_open(max_pkts=2048, max_bytes=4 << 20)
    try:
        assert L.cgck_test_burst_seq(eng.ctx, start) == 0
        for k in range(40):                   # narrow (1 workgroup) and wide (up to 32) requests
            npk = (1, 40, 700, 2048)[k % 4]
            if k % 4 == 0 and k >= 4:
                # every workgroup but the leader left behind: the narrow
                # request next must bring their words up to date
                assert L.cgck_test_burst_stale(eng.ctx, 1) == 0
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
            eng.desc_host(got, desc, flags, out, ver)
            check_burst(out, exp, ver, ever, got, ref, f"start {start:#x} request {k} npk {npk}", 2048, ring, desc)
    finally:
        eng.burst_close()
        assert L.cgck_host_unregister(ring.ctypes.data) == 0


@pytest.mark.parametrize("start", [0xFFFFFFF0, 0x7FFFFFF8, 1000])
def test_seq_wrap_and_stale_done_words(engine, port, start):
    wrap_body(engine, port, start)


def test_hooks_refuse_without_server(engine):
    L = cgck.load()
    bind_hooks(L)
    assert L.cgck_test_burst_seq(engine.ctx, 5) < 0
    assert "no open server" in cgck.last_error()
    assert L.cgck_test_burst_stale(engine.ctx, 1) < 0
