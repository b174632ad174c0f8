"""GPU tests of the per-thread windows (include/cgck.h, cgck_dropin.cpp).

RX window: a receive burst goes through cgck_rx_begin,
then the reference stack's own RX call sequence (oracle/stack_replay.c:
ip_input.c:20-112, tcp_input.c:60-85, udp_usrreq.c:53-94, ip_icmp.c:160-193;
gbtcp/inet.c:118-159, 275-352) runs over the same ring calling libcgck.so's
drop-in in_cksum / udp_cksum.  A second copy replays with the reference's
own subr.c functions (oracle/_ref; the restatement where that build is
absent).  Outcomes, the badsum counter increments, the number of checksum
calls and every byte of the ring afterwards must match, for both stacks and
every t_ip_do_incksum x t_tcp_do_incksum in {0, 1, 2} (con-gen.c:733-736).

TX window (rank 2): only registered ring memory is queued; other memory is
computed synchronously; a header or segment queued twice keeps the later call.
"""
import itertools
import threading

import numpy as np
import pytest

import cgck
import oracle
import rxcorpus

pytestmark = pytest.mark.gpu

FLAGS = list(itertools.product((0, 1), (0, 1, 2), (0, 1, 2)))   # stack, ip_in, tcp_in


def referee(port):
    R = oracle.reference()
    return R if R is not None else port


def replay_pair(port, buf, desc, stack, ip_in, tcp_in, gpu_ring=None):
    """(reference replay, GPU-window replay, window counters, served)."""
    R = referee(port)
    ref = buf.copy()
    a = port.replay_rx(*R.fn_pointers(), ref, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
    got = gpu_ring if gpu_ring is not None else buf.copy()
    if gpu_ring is not None:
        got[:len(buf)] = buf
    s0 = cgck.window_stats()
    m = cgck.rx_begin(got, desc)
    try:
        b = port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
    finally:
        served = cgck.rx_end()
    s1 = cgck.window_stats()
    return (a, ref), (b, got[:len(buf)]), m, served, [y - x for x, y in zip(s0, s1)]


@pytest.mark.parametrize("clean", [True, False])
@pytest.mark.parametrize("registered", [False, True])
def test_rx_window_replay(port, clean, registered):
    rng = np.random.default_rng(101 + clean + 2 * registered)
    frames = rxcorpus.corpus(rng, referee(port), 400, clean=clean)
    buf, desc = rxcorpus.ring(frames)
    L = cgck.load()
    raw = ring = None
    if registered:
        raw, ring, size = rxcorpus.registered_copy(buf)
        assert L.cgck_host_register(ring.ctypes.data, size) == 0
    try:
        for stack, ip_in, tcp_in in FLAGS:
            (a, ref), (b, got), m, served, d = replay_pair(port, buf, desc, stack, ip_in, tcp_in, ring)
            cell = (stack, ip_in, tcp_in)
            assert np.array_equal(a[0], b[0]), (cell, np.nonzero(a[0] != b[0])[0][:8])
            assert np.array_equal(a[1], b[1]), (cell, a[1], b[1])
            assert np.array_equal(ref, got), cell
            calls = int(b[1][4] + b[1][5])
            assert served == d[0] and served + d[1] == calls, (cell, served, d, calls)
            if clean:
                assert m == len(frames) and d[1] == 0, (cell, m, d)   # every call from the window
            else:
                assert served >= 0.9 * calls, (cell, served, calls)
            assert d[2] == 0 and d[3] == 0
    finally:
        if registered:
            L.cgck_host_unregister(ring.ctypes.data)


@pytest.mark.parametrize("nframes", [40, 400, 2500])
def test_rx_window_replay_server(port, nframes):
    """The same replay with this thread's burst server open: the window's
    burst is one server request, served by one workgroup (40 frames) or split
    over 7 / 32 of them, staged (pageable ring) and in place (registered)."""
    rng = np.random.default_rng(211 + nframes)
    frames = rxcorpus.corpus(rng, referee(port), nframes, clean=False)
    buf, desc = rxcorpus.ring(frames)
    L = cgck.load()
    cgck.burst_open(max_pkts=4096, max_bytes=8 << 20)
    try:
        for registered in (False, True):
            ring = None
            if registered:
                raw, ring, size = rxcorpus.registered_copy(buf)
                assert L.cgck_host_register(ring.ctypes.data, size) == 0
            try:
                for stack, ip_in, tcp_in in FLAGS[::2]:
                    (a, ref), (b, got), m, served, d = replay_pair(port, buf, desc, stack, ip_in, tcp_in, ring)
                    cell = (registered, stack, ip_in, tcp_in)
                    assert np.array_equal(a[0], b[0]), (cell, np.nonzero(a[0] != b[0])[0][:8])
                    assert np.array_equal(a[1], b[1]), (cell, a[1], b[1])
                    assert np.array_equal(ref, got), cell
                    calls = int(b[1][4] + b[1][5])
                    assert served == d[0] and served + d[1] == calls, (cell, served, d, calls)
                    assert served >= 0.9 * calls, (cell, served, calls)
            finally:
                if registered:
                    L.cgck_host_unregister(ring.ctypes.data)
    finally:
        cgck.burst_close()


def test_rx_window_fixture_frames(port, golden_verify):
    """The reference-made verify fixtures (tests/golden/verify.json) as one
    burst: verdicts through the window equal the fixtures' own."""
    frames = [np.frombuffer(bytes.fromhex(c["hex"]), np.uint8).copy() for c in golden_verify["cases"]]
    buf, desc = rxcorpus.ring(frames)
    for stack, ip_in, tcp_in in FLAGS:
        (a, ref), (b, got), m, served, d = replay_pair(port, buf, desc, stack, ip_in, tcp_in)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(ref, got)
    # with both flags at 1 on bsd44 every IP verdict is the fixture's bsd_ip
    (a, _), (b, _), _, _, _ = replay_pair(port, buf, desc, 0, 1, 1)
    assert int(b[1][0]) == sum(1 - c["bsd_ip"] for c in golden_verify["cases"])
    assert all((r == oracle.Port.R_DROP_IP) == (c["bsd_ip"] == 0) for r, c in zip(b[0], golden_verify["cases"]))


def test_rx_window_errors_and_reuse(port):
    rng = np.random.default_rng(7)
    buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, port, 8, clean=True))
    assert cgck.rx_begin(buf, desc) == 8
    with pytest.raises(cgck.CgckError, match="already open"):
        cgck.rx_begin(buf, desc)
    assert cgck.rx_end() == 0
    with pytest.raises(cgck.CgckError, match="no open RX window"):
        cgck.rx_end()
    bad = desc.copy()
    bad[7]["ip_len"] = 60000                        # past the ring
    with pytest.raises(cgck.CgckError, match="reaches past"):
        cgck.rx_begin(buf, bad)
    assert cgck.rx_begin(buf, desc[:0]) == 0        # empty burst
    assert cgck.rx_end() == 0
    # outside a window the same calls are synchronous and still exact
    ip = buf[rxcorpus.L2:]
    assert cgck.ip_cksum(ip, 0) == referee(port).in_cksum(ip, 0, (int(ip[0]) & 15) * 4)


def test_rx_window_threads(port):
    """Windows are per thread: four threads, four bursts, one window each."""
    errs = []

    def work(t):
        try:
            rng = np.random.default_rng(500 + t)
            buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, referee(port), 200, clean=True))
            for stack, ip_in, tcp_in in FLAGS[::3]:
                (a, ref), (b, got), m, served, d = replay_pair(port, buf, desc, stack, ip_in, tcp_in)
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(ref, got)
                assert d[1] == 0
        except Exception as e:  # noqa: BLE001 — reported below
            errs.append(repr(e))
        finally:
            cgck.thread_release()

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


# ---------------------------------------------------------------------------
# TX window
# ---------------------------------------------------------------------------

def tx_calls(row, ln, fo):
    """tcp_output.c:416-418 then ip_output.c:61-64 on the packet at row+14."""
    row[14 + 20 + fo:14 + 20 + fo + 2] = 0
    v = cgck.udp_cksum(row, 14, ln - 20)
    row[14 + 20 + fo:14 + 20 + fo + 2] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
    row[14 + 10:14 + 12] = 0
    v = cgck.ip_cksum(row, 14)
    row[14 + 10:14 + 12] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)


def expected(port, pkt, fo):
    ref = pkt.copy()
    ref[20 + fo:22 + fo] = 0
    ref[20 + fo:22 + fo] = np.frombuffer(np.uint16(port.udp_cksum(ref, 0, len(ref) - 20)).tobytes(), np.uint8)
    ref[10:12] = 0
    ref[10:12] = np.frombuffer(np.uint16(port.in_cksum(ref, 0, 20)).tobytes(), np.uint8)
    return ref


def tcp_pkt(rng, ln):
    p = rng.integers(0, 256, ln, dtype=np.uint8)
    p[0] = 0x45
    p[9] = 6
    return p


def test_tx_window_queues_only_registered_memory(port):
    """A stack-local struct packet (tcp_output.c:330-359, pkt_body) is not
    ring memory: its calls are answered synchronously inside the window and
    the flush never touches it; ring slots are queued and filled."""
    rng = np.random.default_rng(61)
    raw, ring, size = rxcorpus.registered_copy(np.zeros(64 * 2048, np.uint8))
    slots = ring[:64 * 2048].reshape(64, 2048)
    local = np.zeros((64, 2048), np.uint8)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    try:
        want = []
        for i in range(64):
            ln = int(rng.integers(40, 523))
            pkt = tcp_pkt(rng, ln)
            tgt = slots if i % 2 else local
            tgt[i, 14:14 + ln] = pkt
            want.append((tgt, i, ln, expected(port, pkt, 16)))
        s0 = cgck.window_stats()
        cgck.tx_begin()
        for tgt, i, ln, _ in want:
            tx_calls(tgt[i], ln, 16)
        s1 = cgck.window_stats()
        for tgt, i, ln, ref in want:   # synchronous ones are already final
            if tgt is local:
                assert np.array_equal(tgt[i, 14:14 + ln], ref), i
        assert cgck.tx_flush() == 64          # 32 registered packets x 2 fields
        assert s1[2] - s0[2] == 64 and s1[3] - s0[3] == 64
        for tgt, i, ln, ref in want:
            assert np.array_equal(tgt[i, 14:14 + ln], ref), i
    finally:
        L.cgck_host_unregister(ring.ctypes.data)


def test_tx_window_slot_reused_before_flush(port):
    """toy_flush reuses one struct packet (gbtcp/tcp.c:615-626): a slot that
    gets a second packet before the flush is filled for the second one."""
    rng = np.random.default_rng(62)
    raw, ring, size = rxcorpus.registered_copy(np.zeros(8 * 2048, np.uint8))
    slots = ring[:8 * 2048].reshape(8, 2048)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    try:
        cgck.tx_begin()
        first = tcp_pkt(rng, 300)
        slots[0, 14:14 + 300] = first
        tx_calls(slots[0], 300, 16)
        second = tcp_pkt(rng, 120)                 # a shorter packet in the same slot
        slots[0, 14:14 + 300] = 0
        slots[0, 14:14 + 120] = second
        tx_calls(slots[0], 120, 16)
        other = tcp_pkt(rng, 522)
        slots[1, 14:14 + 522] = other
        tx_calls(slots[1], 522, 16)
        assert cgck.tx_flush() == 4                # 2 fields x 2 distinct packets
        assert np.array_equal(slots[0, 14:14 + 120], expected(port, second, 16))
        assert not slots[0, 14 + 120:14 + 300].any()
        assert np.array_equal(slots[1, 14:14 + 522], expected(port, other, 16))
    finally:
        L.cgck_host_unregister(ring.ctypes.data)


def test_last_kernel_names(engine):
    """cgck_ctx_last_kernel reports the dispatcher's choice by the name
    rocprofv3 shows."""
    n = 4096
    buf = cgck.DeviceBuffer(n * 1500)
    out = cgck.DeviceBuffer(4 * n)
    engine.synth_strided(buf.ptr, n, 1500, 1500, 5)
    engine.strided(buf.ptr, n, 1500, 0, 1500, cgck.GEN_BOTH, out.ptr)
    assert engine.last_kernel == "dstr_kernel<3, 16, true, 0>"
    engine.strided(buf.ptr, n, 1500, 0, 1500, cgck.VERIFY_TOY, out.ptr)   # verify: group
    assert engine.last_kernel == "cksum_kernel<16, 6, 1, false, true>"
    engine.strided(buf.ptr, n, 64, 0, 64, cgck.GEN_BOTH, out.ptr)
    assert engine.last_kernel == "lpd_kernel<2, 32, 2>"
    ver = cgck.DeviceBuffer(n)
    engine.strided(buf.ptr, n, 64, 0, 64, cgck.GEN_BOTH, out.ptr, ver.ptr)   # verdicts: lpa
    assert engine.last_kernel.startswith("lpa_kernel<false, ")
    engine.sync()
    ver.free()


# ---------------------------------------------------------------------------
# Pipelined windows (cgck_rx_post / cgck_rx_begin_posted, cgck_tx_post /
# cgck_tx_complete): one burst in flight while the stack works
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("server", [False, True])
@pytest.mark.parametrize("nframes", [40, 300, 2100])
def test_rx_pipelined_replay(port, nframes, server):
    """Burst k is posted before the stack replays burst k - 1 from its
    window; every burst's outcomes, counters, call counts and ring bytes
    equal the reference replay's.  Between a post and its window a
    synchronous drop-in call runs (through the server when it is open, so a
    later request needs the posted one's slot and collects it early), and
    the rings are registered for half of the bursts."""
    R = referee(port)
    L = cgck.load()
    bursts = []
    for k in range(5):
        rng = np.random.default_rng(1300 + 10 * k + nframes)
        buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, nframes, clean=k % 2 == 0))
        if k % 2:
            raw, ring, size = rxcorpus.registered_copy(buf)
            assert L.cgck_host_register(ring.ctypes.data, size) == 0
            bursts.append((buf, desc, ring[:len(buf)], ring, raw))
        else:
            bursts.append((buf, desc, buf.copy(), None, None))
    if server:
        cgck.burst_open(max_pkts=4096, max_bytes=8 << 20)
    other = np.arange(64, dtype=np.uint8)
    try:
        for k in range(len(bursts) + 1):
            if k < len(bursts):
                buf, desc, got, _, _ = bursts[k]
                assert cgck.rx_post(got, desc) == len(desc)
                assert cgck.in_cksum(other, 3, 41) == R.in_cksum(other, 3, 41)   # a synchronous call
            if k == 0:
                continue
            buf, desc, got, _, _ = bursts[k - 1]
            for stack, ip_in, tcp_in in FLAGS[k % 3::6][:1]:
                ref = buf.copy()
                a = port.replay_rx(*R.fn_pointers(), ref, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
                s0 = cgck.window_stats()
                m = cgck.rx_begin_posted()
                try:
                    b = port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), stack, ip_in,
                                       tcp_in)
                finally:
                    served = cgck.rx_end()
                s1 = cgck.window_stats()
                cell = (k - 1, stack, ip_in, tcp_in)
                assert np.array_equal(a[0], b[0]), (cell, np.nonzero(a[0] != b[0])[0][:8])
                assert np.array_equal(a[1], b[1]), (cell, a[1], b[1])
                assert np.array_equal(ref, got), cell
                calls = int(b[1][4] + b[1][5])
                assert served == s1[0] - s0[0] and served >= 0.9 * calls, (cell, served, calls)
                assert m <= len(desc)
        with pytest.raises(cgck.CgckError, match="no burst posted"):
            cgck.rx_begin_posted()
    finally:
        if server:
            cgck.burst_close()
        for _, _, _, ring, _ in bursts:
            if ring is not None:
                L.cgck_host_unregister(ring.ctypes.data)


def test_rx_post_limits(port):
    rng = np.random.default_rng(77)
    buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, port, 16, clean=True))
    rings = [buf.copy() for _ in range(65)]
    for k in range(64):
        assert cgck.rx_post(rings[k], desc) == 16
    assert cgck.rx_pending() == 64
    with pytest.raises(cgck.CgckError, match="already posted"):
        cgck.rx_post(rings[64], desc)
    assert cgck.rx_begin_posted() == 16
    with pytest.raises(cgck.CgckError, match="already open"):
        cgck.rx_begin_posted()
    assert cgck.rx_end() == 0
    for k in range(63):
        assert cgck.rx_begin_posted() == 16
        assert cgck.rx_end() == 0
    bad = desc.copy()
    bad[3]["ip_len"] = 60000
    with pytest.raises(cgck.CgckError, match="reaches past"):
        cgck.rx_post(rings[0], bad)
    with pytest.raises(cgck.CgckError, match="no burst posted"):
        cgck.rx_begin_posted()


@pytest.mark.parametrize("server", [False, True])
def test_tx_pipelined_fill(port, server):
    """Two bursts' fills posted back to back (the GPU computes burst k while
    the stack builds burst k + 1); cgck_tx_complete writes each burst's
    fields, oldest first; the slots of the burst not yet completed keep the
    zeros the stack stored."""
    rng = np.random.default_rng(63 + server)
    raw, ring, size = rxcorpus.registered_copy(np.zeros(256 * 2048, np.uint8))
    slots = ring[:256 * 2048].reshape(256, 2048)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        bursts = []
        for k in range(3):
            want = []
            cgck.tx_begin()
            for i in range(k * 80, k * 80 + 80):
                ln = int(rng.integers(40, 1501))
                pkt = tcp_pkt(rng, ln)
                slots[i, 14:14 + ln] = pkt
                want.append((i, ln, expected(port, pkt, 16)))
                tx_calls(slots[i], ln, 16)
            assert cgck.tx_post() == 160
            bursts.append(want)
            if k >= 1:
                assert cgck.tx_complete() == 160
                for i, ln, ref in bursts[k - 1]:
                    assert np.array_equal(slots[i, 14:14 + ln], ref), (k - 1, i)
        assert cgck.tx_complete() == 160
        for i, ln, ref in bursts[2]:
            assert np.array_equal(slots[i, 14:14 + ln], ref), (2, i)
        assert cgck.tx_complete() == 0
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(ring.ctypes.data)


def expected_calls(port, pkt, fo, seg, hdr):
    """The packet's bytes after the calls the stack made on it: the segment's
    field when udp_cksum was queued, the header's when in_cksum was."""
    ref = pkt.copy()
    if seg:
        ref[20 + fo:22 + fo] = 0
        ref[20 + fo:22 + fo] = np.frombuffer(np.uint16(port.udp_cksum(ref, 0, len(ref) - 20)).tobytes(), np.uint8)
    if hdr:
        ref[10:12] = 0
        ref[10:12] = np.frombuffer(np.uint16(port.in_cksum(ref, 0, 20)).tobytes(), np.uint8)
    return ref


@pytest.mark.parametrize("mode", ["post", "flush"])
@pytest.mark.parametrize("server", [False, True])
@pytest.mark.parametrize("shape", ["header_only", "segment_only", "out_of_order", "replaced", "unregistered"])
def test_tx_pipelined_irregular(port, server, shape, mode):
    """The posted fill off the common path: packets with only their header
    queued (an ICMP reply, ip_output alone), packets with only their segment
    queued, slots queued out of address order (a ring wrap), a slot queued
    again with a shorter packet, and stack-local packets among the ring's.
    Each burst's fields equal the reference's over the packet's final bytes
    and tx_post (or the synchronous tx_flush) counts the queued fields."""
    rng = np.random.default_rng(900 + 10 * server + len(shape))
    raw, ring, size = rxcorpus.registered_copy(np.zeros(128 * 2048, np.uint8))
    slots = ring[:128 * 2048].reshape(128, 2048)
    local = np.zeros((128, 2048), np.uint8)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        for k in range(3):
            order = list(range(k * 40, k * 40 + 40))
            if shape == "out_of_order":
                order = order[20:] + order[:20]
            want, fields = {}, 0
            cgck.tx_begin()
            for j, i in enumerate(order):
                tgt = local if shape == "unregistered" and j % 3 == 1 else slots
                seg = not (shape == "header_only" and j % 4 == 2)
                hdr = not (shape == "segment_only" and j % 5 == 3)
                ln = int(rng.integers(40, 1501))
                pkt = tcp_pkt(rng, ln)
                tgt[i, 14:14 + ln] = pkt
                if seg:
                    tgt[i, 14 + 36:14 + 38] = 0
                    v = cgck.udp_cksum(tgt[i], 14, ln - 20)
                    tgt[i, 14 + 36:14 + 38] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
                if hdr:
                    tgt[i, 14 + 10:14 + 12] = 0
                    v = cgck.ip_cksum(tgt[i], 14)
                    tgt[i, 14 + 10:14 + 12] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
                if shape == "replaced" and j == 7:     # the slot gets a shorter packet before the post
                    ln2 = int(rng.integers(40, ln + 1))
                    pkt = tcp_pkt(rng, ln2)
                    tgt[i, 14:14 + ln] = 0
                    tgt[i, 14:14 + ln2] = pkt
                    ln = ln2
                    tx_calls(tgt[i], ln, 16)
                fields += (seg + hdr) if tgt is slots else 0
                want[(id(tgt), i)] = (tgt, i, ln, pkt.copy(), seg, hdr)
            if mode == "post":
                assert cgck.tx_post() == fields, (shape, k)
                assert cgck.tx_complete() == fields
            else:
                assert cgck.tx_flush() == fields, (shape, k)
            for tgt, i, ln, pkt, seg, hdr in want.values():
                ref = expected_calls(port, pkt, 16, seg, hdr)   # a field not asked for keeps its bytes
                assert np.array_equal(tgt[i, 14:14 + ln], ref), (shape, k, i, seg, hdr)
        assert cgck.tx_complete() == 0
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(ring.ctypes.data)


def test_rx_tx_pipelined_loop(port):
    """con-gen's worker loop with both windows pipelined on one thread and
    one burst server (con-gen.c:484-538): each iteration completes the
    previous TX fill before the kick, posts the next receive burst, replays
    the stack's RX calls over the previous one from its window, then builds
    and posts this iteration's TX fill.  RX outcomes and ring bytes equal the
    reference replay's and every TX field equals the reference's, with RX and
    TX requests sharing the server's two request slots."""
    R = referee(port)
    L = cgck.load()
    raw_tx, tx_ring, tx_size = rxcorpus.registered_copy(np.zeros(2 * 96 * 2048, np.uint8))
    slots = tx_ring[:2 * 96 * 2048].reshape(2, 96, 2048)
    assert L.cgck_host_register(tx_ring.ctypes.data, tx_size) == 0
    rx = []
    for k in range(6):
        rng = np.random.default_rng(4200 + k)
        buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 70 + 30 * k, clean=k % 3 != 1))
        owner, ring, size = rxcorpus.registered_copy(buf)
        assert L.cgck_host_register(ring.ctypes.data, size) == 0
        rx.append((buf, desc, ring[:len(buf)], ring, owner))
    cgck.burst_open(max_pkts=4096, max_bytes=8 << 20)
    rng = np.random.default_rng(4300)
    tx_prev = None
    try:
        for k in range(len(rx) + 1):
            if tx_prev is not None:                      # io_tx(): the previous fill, before the kick
                assert cgck.tx_complete() == 2 * len(tx_prev)
                for h, i, ln, ref in tx_prev:
                    assert np.array_equal(slots[h, i, 14:14 + ln], ref), (k, h, i)
                tx_prev = None
            if k < len(rx):
                _, desc, got, _, _ = rx[k]
                assert cgck.rx_post(got, desc) == len(desc)
            if k > 0:                                    # the receive burst of the previous iteration
                buf, desc, got, _, _ = rx[k - 1]
                stack, ip_in, tcp_in = FLAGS[(5 * k) % len(FLAGS)]
                ref = buf.copy()
                a = port.replay_rx(*R.fn_pointers(), ref, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
                cgck.rx_begin_posted()
                try:
                    b = port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), stack, ip_in,
                                       tcp_in)
                finally:
                    cgck.rx_end()
                cell = (k - 1, stack, ip_in, tcp_in)
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), cell
                assert np.array_equal(ref, got), cell
            if k == len(rx):
                break
            h = k & 1                                     # bsd_flush(): this iteration's segments
            want = []
            cgck.tx_begin()
            for i in range(40 + 10 * k):
                ln = int(rng.integers(40, 1501))
                pkt = tcp_pkt(rng, ln)
                slots[h, i, 14:14 + ln] = pkt
                want.append((h, i, ln, expected(port, pkt, 16)))
                tx_calls(slots[h, i], ln, 16)
            assert cgck.tx_post() == 2 * len(want)
            tx_prev = want
        assert tx_prev is None and cgck.tx_complete() == 0
    finally:
        cgck.burst_close()
        for _, _, _, ring, _ in rx:
            L.cgck_host_unregister(ring.ctypes.data)
        L.cgck_host_unregister(tx_ring.ctypes.data)


def test_pipelined_across_server_idle(port):
    """A posted burst or fill whose completion comes after the server idled
    out (idle_ms 20, then 100 ms of other work), and a post made while no
    server workgroup is alive: the post relaunches it, every value is exact."""
    import time
    R = referee(port)
    L = cgck.load()
    raw, tx_ring, size = rxcorpus.registered_copy(np.zeros(64 * 2048, np.uint8))
    slots = tx_ring[:64 * 2048].reshape(64, 2048)
    assert L.cgck_host_register(tx_ring.ctypes.data, size) == 0
    cgck.burst_open(max_pkts=1024, max_bytes=4 << 20, idle_ms=20)
    try:
        rng = np.random.default_rng(4400)
        for rep in range(3):
            buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 90, clean=rep != 1))
            got = buf.copy()
            assert cgck.rx_post(got, desc) == len(desc)
            want = []
            cgck.tx_begin()
            for i in range(32):
                ln = int(rng.integers(40, 1501))
                pkt = tcp_pkt(rng, ln)
                slots[i, 14:14 + ln] = pkt
                want.append((i, ln, expected(port, pkt, 16)))
                tx_calls(slots[i], ln, 16)
            assert cgck.tx_post() == 64
            time.sleep(0.1)                      # > idle_ms: the server exits once both are served
            stack, ip_in, tcp_in = FLAGS[(7 * rep) % len(FLAGS)]
            ref = buf.copy()
            a = port.replay_rx(*R.fn_pointers(), ref, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
            cgck.rx_begin_posted()
            try:
                b = port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
            finally:
                cgck.rx_end()
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(ref, got), rep
            assert cgck.tx_complete() == 64
            for i, ln, r in want:
                assert np.array_equal(slots[i, 14:14 + ln], r), (rep, i)
            time.sleep(0.1)                      # the next posts find no workgroup alive
    finally:
        cgck.burst_close()
        L.cgck_host_unregister(tx_ring.ctypes.data)


# ---------------------------------------------------------------------------
# The drain rule (include/cgck.h: cgck_rx_pending / cgck_rx_ready) and the
# burst server's bookkeeping across out-of-order collects
# ---------------------------------------------------------------------------

def replay_posted(port, R, buf, desc, got, cell):
    """Open the oldest posted burst, replay the stack over it, compare with
    the reference replay of the same bytes."""
    stack, ip_in, tcp_in = cell
    ref = buf.copy()
    a = port.replay_rx(*R.fn_pointers(), ref, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
    s0 = cgck.window_stats()
    cgck.rx_begin_posted()
    try:
        b = port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
    finally:
        served = cgck.rx_end()
    s1 = cgck.window_stats()
    assert np.array_equal(a[0], b[0]), (cell, np.nonzero(a[0] != b[0])[0][:8])
    assert np.array_equal(a[1], b[1]), (cell, a[1], b[1])
    assert np.array_equal(ref, got), cell
    return served, [y - x for x, y in zip(s0, s1)], int(b[1][4] + b[1][5])


@pytest.mark.parametrize("server", [False, True])
@pytest.mark.parametrize("nframes", [1, 3, 40, 700])
def test_rx_lone_burst_drained(port, nframes, server):
    """A burst posted with nothing after it (the last one before a quiet
    spell: con-gen.c:508-517 calls io_rx only on POLLIN) is drained in the
    iteration that follows — cgck_rx_pending says one is posted,
    cgck_rx_ready turns 1 without a wait, and the window over it replays
    bit-exact with every call answered — and every iteration with nothing
    posted finds nothing to drain."""
    import time
    R = referee(port)
    L = cgck.load()
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    rings = []
    try:
        for it in range(3):
            rng = np.random.default_rng(5100 + 10 * it + nframes)
            buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, nframes, clean=True))
            raw, ring, size = rxcorpus.registered_copy(buf)
            assert L.cgck_host_register(ring.ctypes.data, size) == 0
            rings.append((raw, ring))
            got = ring[:len(buf)]
            assert cgck.rx_pending() == 0
            with pytest.raises(cgck.CgckError, match="no burst posted"):
                cgck.rx_ready()
            assert cgck.rx_post(got, desc) == nframes       # io_rx: the burst, then a quiet spell
            assert cgck.rx_pending() == 1
            t0 = time.monotonic()
            while not cgck.rx_ready():                       # the next iteration's check (no wait)
                assert time.monotonic() - t0 < 2.0
            cell = FLAGS[(3 * it + nframes) % len(FLAGS)]
            served, d, calls = replay_posted(port, R, buf, desc, got, cell)
            # (a payload bit flip can land in a UDP length, making a call the
            # window does not hold: it is computed synchronously, still exact)
            assert served == d[0] and served + d[1] == calls and d[1] <= calls // 100, (cell, served, calls, d)
            assert cgck.rx_pending() == 0
    finally:
        if server:
            cgck.burst_close()
        for raw, ring in rings:
            L.cgck_host_unregister(ring.ctypes.data)


@pytest.mark.parametrize("gap", ["idle", "register"])
def test_burst_relaunch_after_out_of_order_collect(port, gap):
    """The pipelined loop collects out of seq order: TX fill b completes
    before the older RX burst a, whose slot the next post then needs.  The
    server then goes away — it idles out, or another range's registration
    stops it — and the next post relaunches it.  The relaunch starts after
    the latest seq collected (b), so it serves c and d; had it started after
    a, its leader would wait for b in a slot that holds d."""
    import time
    R = referee(port)
    L = cgck.load()
    raw_tx, tx_ring, tx_size = rxcorpus.registered_copy(np.zeros(64 * 2048, np.uint8))
    slots = tx_ring[:64 * 2048].reshape(64, 2048)
    assert L.cgck_host_register(tx_ring.ctypes.data, tx_size) == 0
    cgck.burst_open(max_pkts=1024, max_bytes=4 << 20, idle_ms=20)
    rng = np.random.default_rng(5200)
    bursts = [rxcorpus.ring(rxcorpus.corpus(rng, R, 50 + 20 * k, clean=True)) for k in range(2)]
    gots = [b.copy() for b, _ in bursts]
    other = None

    def fill(lo):
        want = []
        cgck.tx_begin()
        for i in range(lo, lo + 16):
            ln = int(rng.integers(40, 1501))
            pkt = tcp_pkt(rng, ln)
            slots[i, 14:14 + ln] = pkt
            want.append((i, ln, expected(port, pkt, 16)))
            tx_calls(slots[i], ln, 16)
        assert cgck.tx_post() == 32
        return want

    try:
        assert cgck.rx_post(gots[0], bursts[0][1]) == len(bursts[0][1])   # seq a
        w_b = fill(0)                                                      # seq b
        assert cgck.tx_complete() == 32                                     # collect b
        for i, ln, r in w_b:
            assert np.array_equal(slots[i, 14:14 + ln], r)
        assert cgck.rx_post(gots[1], bursts[1][1]) == len(bursts[1][1])   # collects a, posts c
        if gap == "idle":
            time.sleep(0.1)                                                # > idle_ms
        else:
            other = rxcorpus.registered_copy(np.zeros(8192, np.uint8))
            assert L.cgck_host_register(other[1].ctypes.data, other[2]) == 0
        w_d = fill(16)                                                     # seq d: relaunches
        assert cgck.tx_complete() == 32
        for i, ln, r in w_d:
            assert np.array_equal(slots[i, 14:14 + ln], r)
        for k in range(2):
            replay_posted(port, R, bursts[k][0], bursts[k][1], gots[k], FLAGS[4 + k])
    finally:
        cgck.burst_close()
        L.cgck_host_unregister(tx_ring.ctypes.data)
        if other is not None:
            L.cgck_host_unregister(other[1].ctypes.data)


def test_posted_burst_survives_unregister(port):
    """A burst posted over a registered ring, then the ring unregistered
    before its window opens: cgck_host_unregister serves the posted request
    before the mapping changes (the server never reads the range after), so
    the window's values are the ring's."""
    R = referee(port)
    L = cgck.load()
    cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        rng = np.random.default_rng(5300)
        buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 300, clean=True))
        raw, ring, size = rxcorpus.registered_copy(buf)
        assert L.cgck_host_register(ring.ctypes.data, size) == 0
        got = ring[:len(buf)]
        assert cgck.rx_post(got, desc) == 300
        assert L.cgck_host_unregister(ring.ctypes.data) == 0
        served, d, calls = replay_posted(port, R, buf, desc, got, FLAGS[7])
        assert served == d[0] and served + d[1] == calls and d[1] <= calls // 100
    finally:
        cgck.burst_close()


def test_posted_burst_not_reserved_after_mapping_change(port):
    """A burst posted over a ring; another range registered (the mapping
    change serves the posted request and stops the server); the ring's
    bytes then change; a synchronous drop-in call on the same thread posts
    the next seq and relaunches the server.  The relaunch must start after
    the request the mapping change served: served again, it would read the
    changed bytes into the burst's values."""
    R = referee(port)
    L = cgck.load()
    cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    other = None
    try:
        rng = np.random.default_rng(5310)
        buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 120, clean=True))
        raw, ring, size = rxcorpus.registered_copy(buf)
        assert L.cgck_host_register(ring.ctypes.data, size) == 0
        got = ring[:len(buf)]
        assert cgck.rx_post(got, desc) == 120
        other = rxcorpus.registered_copy(np.zeros(8192, np.uint8))
        assert L.cgck_host_register(other[1].ctypes.data, other[2]) == 0
        saved = got.copy()
        got[:] = rng.integers(0, 256, len(got), dtype=np.uint8)    # the ring reused meanwhile
        hdr = np.array([0x45, 0, 0, 20, 0, 0, 0x40, 0, 64, 6, 0, 0, 10, 0, 0, 1, 10, 0, 0, 2], np.uint8)
        assert cgck.ip_cksum(hdr) == port.in_cksum(hdr, 0, 20)        # sync call: next seq, relaunch
        got[:] = saved
        served, d, calls = replay_posted(port, R, buf, desc, got, FLAGS[7])
        assert served == d[0] and served + d[1] == calls
        L.cgck_host_unregister(ring.ctypes.data)
    finally:
        cgck.burst_close()
        if other is not None:
            L.cgck_host_unregister(other[1].ctypes.data)


@pytest.mark.parametrize("server", [False, True])
def test_pending_fill_across_many_rx_cycles(port, server):
    """One TX fill posted and left pending while 140 receive bursts are
    posted, opened and closed: the requests behind the fill's are freed out
    of order, so none reuses the fill's request slot (128 slots
    freed only from the oldest overflowed into the fill's at the 128th), and
    the completion writes the fill's own values."""
    R = referee(port)
    L = cgck.load()
    raw, ring, size = rxcorpus.registered_copy(np.zeros(16 * 2048, np.uint8))
    slots = ring[:16 * 2048].reshape(16, 2048)
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    rng = np.random.default_rng(5320 + server)
    try:
        want = []
        cgck.tx_begin()
        for i in range(4):
            ln = int(rng.integers(40, 1501))
            pkt = tcp_pkt(rng, ln)
            slots[i, 14:14 + ln] = pkt
            want.append((i, ln, expected(port, pkt, 16)))
            tx_calls(slots[i], ln, 16)
        assert cgck.tx_post() == 8
        buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 6, clean=True))
        raw2, ring2, size2 = rxcorpus.registered_copy(buf)
        assert L.cgck_host_register(ring2.ctypes.data, size2) == 0
        got = ring2[:len(buf)]
        try:
            for it in range(140):
                got[:] = buf
                assert cgck.rx_post(got, desc) == 6
                served, d, calls = replay_posted(port, R, buf, desc, got, FLAGS[(it * 5) % len(FLAGS)])
                assert served == d[0], it
            assert cgck.tx_pending() == 1
        finally:
            L.cgck_host_unregister(ring2.ctypes.data)
        assert cgck.tx_complete() == 8
        for i, ln, r in want:
            assert np.array_equal(slots[i, 14:14 + ln], r), i
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(ring.ctypes.data)


@pytest.mark.parametrize("server", [False, True])
def test_tx_post_beyond_queue_completes_oldest(port, server):
    """64 fills posted and a 65th window closed: cgck_tx_post completes the
    oldest first (its fields written), so no queued field is dropped."""
    rng = np.random.default_rng(5400 + server)
    raw, ring, size = rxcorpus.registered_copy(np.zeros(130 * 2048, np.uint8))
    slots = ring[:130 * 2048].reshape(130, 2048)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        fills = []
        for k in range(65):
            want = []
            cgck.tx_begin()
            for i in range(2 * k, 2 * k + 2):
                ln = int(rng.integers(40, 1501))
                pkt = tcp_pkt(rng, ln)
                slots[i, 14:14 + ln] = pkt
                want.append((i, ln, expected(port, pkt, 16)))
                tx_calls(slots[i], ln, 16)
            assert cgck.tx_post() == 4
            fills.append(want)
        assert cgck.tx_pending() == 64
        for i, ln, ref in fills[0]:                      # written by the 65th post
            assert np.array_equal(slots[i, 14:14 + ln], ref), (0, i)
        for k in range(1, 65):
            assert cgck.tx_complete() == 4
            for i, ln, ref in fills[k]:
                assert np.array_equal(slots[i, 14:14 + ln], ref), (k, i)
        assert cgck.tx_complete() == 0
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(ring.ctypes.data)


# ---------------------------------------------------------------------------
# The TX window across the whole loop iteration: replies built while the
# stack processes a receive burst (tcp_respond RSTs, icmp_error, echo
# replies) and keepalives at check_timers are queued, not computed one call
# at a time
# ---------------------------------------------------------------------------

def ka_records(rng, n):
    ka = np.zeros(n, oracle.Port.KA_DTYPE)
    for f, hi in (("laddr", 2 ** 32), ("faddr", 2 ** 32), ("rcv_nxt", 2 ** 32), ("snd_una", 2 ** 32)):
        ka[f] = rng.integers(0, hi, n, dtype=np.uint64)
    ka["lport"] = rng.integers(0, 2 ** 16, n)
    ka["fport"] = rng.integers(0, 2 ** 16, n)
    ka["hiwat"] = rng.integers(0, 2 ** 20, n)
    ka["scale"] = rng.integers(0, 9, n)
    return ka


class Iteration:
    """One side (reference functions, or libcgck's drop-ins inside the
    windows) of thread_process iterations over one pool: the receive burst
    with its replies, then check_timers' keepalives, replies built into the
    transmit slots in order."""

    def __init__(self, port, fns, pool, tx_base, tx_stride, cap):
        self.port, self.fns, self.pool = port, fns, pool
        self.tx_base, self.tx_stride, self.cap = tx_base, tx_stride, cap
        self.local = np.zeros(2048 * 1200, np.uint8)   # room for every reply (the ring full from the start)
        self.used = self.nlocal = 0
        self.ip_id = 4242
        self.sent = np.zeros(4, np.int64)

    def _run(self, desc, n, ip_in, tcp_in, ka):
        tx = self.pool[self.tx_base + self.used * self.tx_stride:]
        loc = self.local[self.nlocal * 2048:]
        res, ctr, txs, self.ip_id = self.port.replay_rx_rsp(
            self.fns[0], self.fns[1], self.pool, desc.view(np.uint8), n, ip_in, tcp_in, tx, self.tx_stride,
            max(self.cap - self.used, 0), loc, rxcorpus.LADDR, ka, self.ip_id)
        self.used += int(txs[0])
        self.nlocal += int(txs[1])
        self.sent += txs[2:].astype(np.int64)
        return res, ctr

    def burst(self, desc, ip_in, tcp_in):
        return self._run(desc, len(desc), ip_in, tcp_in, None)

    def timers(self, ka):
        return self._run(np.zeros(0, cgck.DESC_DTYPE), 0, 0, 0, ka)


@pytest.mark.parametrize("mode", ["sync", "pipelined"])
@pytest.mark.parametrize("ring", ["room", "full"])
def test_rsp_iteration_tx_window(port, mode, ring):
    """con-gen's loop with the TX window open from the kick to the flush:
    io_tx, then the receive burst through the RX window (cgck_rx_begin, or
    pipelined: post burst k, replay burst k - 1, drain the last one), the
    stack's replies to it and check_timers' keepalives, then the flush (or
    cgck_tx_post, completed before the next kick).  The corpus draws RSTs,
    net / port unreachables and echo replies (oracle_replay_rx_rsp).  RX
    outcomes, counters and the whole pool — receive frames and replies —
    equal the reference replay's byte for byte; every reply call in ring
    memory is queued (window_stats[3] = 0 with room in the ring) and no
    received frame's verify call is (the replay would count it bad).  With
    the ring full the replies built in pkt_body are computed synchronously
    (window_stats[3] > 0) and are exact too."""
    R = referee(port)
    L = cgck.load()
    rng = np.random.default_rng(6100 + (mode == "pipelined") + 2 * (ring == "full"))
    nb = 4
    bursts = [rxcorpus.rsp_corpus(rng, R, 60 + 70 * k) for k in range(nb)]
    frames = [f for b in bursts for f in b]
    kas = [ka_records(rng, 6) for _ in range(nb)]
    cap = 1200 if ring == "room" else 40             # transmit slots (rxcorpus.pool(frames, 1200))
    buf, desc_all, tx_base, tx_stride = rxcorpus.pool(frames, 1200)
    descs, at = [], 0
    for b in bursts:
        descs.append(desc_all[at:at + len(b)])
        at += len(b)
    ref = buf.copy()
    raw, got, size = rxcorpus.registered_copy(buf)
    assert L.cgck_host_register(got.ctypes.data, size) == 0
    got = got[:len(buf)]
    A = Iteration(port, R.fn_pointers(), ref, tx_base, tx_stride, cap)
    B = Iteration(port, cgck.fn_pointers(), got, tx_base, tx_stride, cap)
    cgck.burst_open(max_pkts=4096, max_bytes=8 << 20)
    s0 = cgck.window_stats()
    try:
        for k in range(nb + (mode == "pipelined")):
            flags = FLAGS[(7 * k + 3) % 9]           # bsd44 cells
            if mode == "pipelined":
                cgck.tx_complete()                   # before io_tx (con-gen.c:493)
            cgck.tx_begin()
            if mode == "sync":
                cgck.rx_begin(got, descs[k])
                todo = k
            else:
                if k < nb:
                    cgck.rx_post(got, descs[k])
                todo = k - 1
                if k == nb:                          # nothing received: the drain rule
                    assert cgck.rx_pending() == 1
            if todo >= 0:
                if mode == "pipelined":
                    cgck.rx_begin_posted()
                try:
                    rb = B.burst(descs[todo], flags[1], flags[2])
                finally:
                    cgck.rx_end()
                ra = A.burst(descs[todo], flags[1], flags[2])
                assert np.array_equal(ra[0], rb[0]), (k, np.nonzero(ra[0] != rb[0])[0][:8])
                assert np.array_equal(ra[1], rb[1]), (k, ra[1], rb[1])
                A.timers(kas[todo])
                B.timers(kas[todo])
            if mode == "sync":
                cgck.tx_flush()
            else:
                cgck.tx_post()
        if mode == "pipelined":
            cgck.tx_complete()
            assert cgck.tx_complete() == 0 and cgck.rx_pending() == 0
        s1 = cgck.window_stats()
    finally:
        cgck.burst_close()
        L.cgck_host_unregister(got.ctypes.data)
    d = [y - x for x, y in zip(s0, s1)]
    assert A.used == B.used and A.nlocal == B.nlocal and np.array_equal(A.sent, B.sent)
    assert A.used + A.nlocal <= 1200
    assert min(A.sent) > 0, A.sent
    assert np.array_equal(ref, got), np.nonzero(ref != got)[0][:16]
    assert np.array_equal(A.local[:A.nlocal * 2048], B.local[:B.nlocal * 2048])
    tx_calls = 2 * int(A.sent.sum())
    if ring == "room":
        assert d[3] == 0 and d[2] == tx_calls, (d, tx_calls)
    else:
        assert d[3] == 2 * B.nlocal and d[2] == 2 * B.used, (d, B.used, B.nlocal)


# ---------------------------------------------------------------------------
# Coalesced posting: bursts and fills posted while an earlier request is on
# the burst server go out together as one request when it is back
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("server", [False, True])
def test_rx_coalesced_small_bursts(port, server):
    """Sixty bursts of 1..6 frames over one registered pool, posted and
    opened on a random schedule (up to 40 outstanding), with a synchronous
    drop-in call now and then (it takes a server slot): every burst's
    window replays bit-exact, oldest first, and cgck_rx_ready never says
    ready for a burst whose values are not in."""
    R = referee(port)
    L = cgck.load()
    rng = np.random.default_rng(7100 + server)
    sizes = [int(rng.integers(1, 7)) for _ in range(60)]
    frames = rxcorpus.corpus(rng, R, sum(sizes), clean=True)
    buf, desc_all = rxcorpus.ring(frames)
    raw, pool, size = rxcorpus.registered_copy(buf)
    assert L.cgck_host_register(pool.ctypes.data, size) == 0
    got = pool[:len(buf)]
    descs, at = [], 0
    for s in sizes:
        descs.append(desc_all[at:at + s].copy())
        at += s
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    other = np.arange(64, dtype=np.uint8)
    ref = buf.copy()                                # the reference replay's ring, burst after burst
    posted = opened = 0
    try:
        while opened < len(sizes):
            k = int(rng.integers(0, 4))
            for _ in range(k):
                if posted < len(sizes) and posted - opened < 40:
                    assert cgck.rx_post(got, descs[posted]) == sizes[posted]
                    posted += 1
            if rng.random() < 0.1:
                assert cgck.in_cksum(other, 3, 41) == R.in_cksum(other, 3, 41)
            if posted > opened and rng.random() < 0.5:
                r = cgck.rx_ready()
                assert r in (0, 1)
                stack, ip_in, tcp_in = cell = FLAGS[(opened * 5) % len(FLAGS)]
                d = descs[opened]
                a = port.replay_rx(*R.fn_pointers(), ref, d.view(np.uint8), len(d), stack, ip_in, tcp_in)
                cgck.rx_begin_posted()
                try:
                    b = port.replay_rx(*cgck.fn_pointers(), got, d.view(np.uint8), len(d), stack, ip_in, tcp_in)
                finally:
                    cgck.rx_end()
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (opened, cell, a, b)
                assert np.array_equal(ref, got), (opened, cell)   # the ring as the reference left it
                opened += 1
            assert cgck.rx_pending() == posted - opened
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(pool.ctypes.data)


@pytest.mark.parametrize("server", [False, True])
def test_tx_coalesced_fills(port, server):
    """Forty small fills posted back to back with none completed (a
    transport holding each fill's slots back until it completes), then
    completed as cgck_tx_ready reports them in: every field equals the
    reference's, fills complete in post order, and a fill's slots keep the
    stack's zeros until then."""
    rng = np.random.default_rng(7200 + server)
    raw, ring, size = rxcorpus.registered_copy(np.zeros(200 * 2048, np.uint8))
    slots = ring[:200 * 2048].reshape(200, 2048)
    L = cgck.load()
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    if server:
        cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        fills, at = [], 0
        for k in range(40):
            want = []
            cgck.tx_begin()
            for i in range(at, at + int(rng.integers(1, 6))):
                ln = int(rng.integers(40, 600))
                pkt = tcp_pkt(rng, ln)
                slots[i, 14:14 + ln] = pkt
                want.append((i, ln, expected(port, pkt, 16)))
                tx_calls(slots[i], ln, 16)
            at += len(want)
            assert cgck.tx_post() == 2 * len(want)
            fills.append(want)
        assert cgck.tx_pending() == 40
        import time
        t0 = time.monotonic()
        done = 0
        while done < 40:
            if cgck.tx_ready() == 1 or time.monotonic() - t0 > 1.0:
                assert cgck.tx_complete() == 2 * len(fills[done])
                for i, ln, ref in fills[done]:
                    assert np.array_equal(slots[i, 14:14 + ln], ref), (done, i)
                done += 1
                if done < 40:                   # the next fill's fields are still the zeros
                    i, ln, _ = fills[done][0]
                    if cgck.tx_ready() == 0:
                        assert not slots[i, 14 + 10:14 + 12].any()
        assert cgck.tx_pending() == 0 and cgck.tx_complete() == 0
    finally:
        if server:
            cgck.burst_close()
        L.cgck_host_unregister(ring.ctypes.data)


def test_rx_tx_fused_coalesced(port):
    """Receive bursts and TX fills posted over ONE registered pool on a random
    schedule, both queues deep: what waits in both queues when the server
    answers goes out as one two-part request (the frames with the RX flags,
    the fill's packets with the TX flags).  Every burst replays bit-exact
    against the reference, every fill's fields equal the reference's, in
    post order on each side."""
    R = referee(port)
    L = cgck.load()
    rng = np.random.default_rng(7300)
    sizes = [int(rng.integers(1, 5)) for _ in range(70)]
    frames = rxcorpus.corpus(rng, R, sum(sizes), clean=True)
    buf, desc_all, tx_base, tx_stride = rxcorpus.pool(frames, 400)
    raw, pool, size = rxcorpus.registered_copy(buf)
    assert L.cgck_host_register(pool.ctypes.data, size) == 0
    got = pool[:len(buf)]
    ref = buf.copy()
    descs, at = [], 0
    for s in sizes:
        descs.append(desc_all[at:at + s].copy())
        at += s
    slot = lambda j: got[tx_base + j * tx_stride:tx_base + j * tx_stride + 2048]
    cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
    posted = opened = 0
    fills, completed, next_tx = [], 0, 0
    try:
        while opened < len(sizes) or completed < len(fills):
            if posted < len(sizes) and posted - opened < 60 and rng.random() < 0.6:
                assert cgck.rx_post(got, descs[posted]) == sizes[posted]
                posted += 1
            if next_tx < 380 and len(fills) - completed < 60 and rng.random() < 0.6:
                want = []
                cgck.tx_begin()
                for _ in range(int(rng.integers(1, 4))):
                    ln = int(rng.integers(40, 600))
                    pkt = tcp_pkt(rng, ln)
                    row = slot(next_tx)
                    row[14:14 + ln] = pkt
                    want.append((next_tx, ln, expected(port, pkt, 16)))
                    tx_calls(row, ln, 16)
                    next_tx += 1
                assert cgck.tx_post() == 2 * len(want)
                fills.append(want)
            if posted > opened and (rng.random() < 0.3 or posted == len(sizes)):
                stack, ip_in, tcp_in = cell = FLAGS[(opened * 7) % len(FLAGS)]
                d = descs[opened]
                a = port.replay_rx(*R.fn_pointers(), ref, d.view(np.uint8), len(d), stack, ip_in, tcp_in)
                cgck.rx_begin_posted()
                try:
                    b = port.replay_rx(*cgck.fn_pointers(), got, d.view(np.uint8), len(d), stack, ip_in, tcp_in)
                finally:
                    cgck.rx_end()
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (opened, cell)
                opened += 1
            if len(fills) > completed and (rng.random() < 0.3 or next_tx >= 380):
                assert cgck.tx_complete() == 2 * len(fills[completed])
                for j, ln, r in fills[completed]:
                    assert np.array_equal(slot(j)[14:14 + ln], r), (completed, j)
                completed += 1
        assert cgck.rx_pending() == 0 and cgck.tx_pending() == 0
        # the receive frames as the reference left them (the transmit slots differ by design)
        for d in descs:
            for o, l3, ln in d.tolist():
                assert np.array_equal(got[o:o + l3 + ln], ref[o:o + l3 + ln])
    finally:
        cgck.burst_close()
        L.cgck_host_unregister(pool.ctypes.data)


def test_coalesced_threads_with_mapping_changes(port):
    """Three worker threads, each with its own pool, burst server and both
    coalesced queues deep, while the main thread keeps registering and
    unregistering a range of its own (each change stops every server, after
    serving what is posted): every burst replays bit-exact and every fill's
    fields are the reference's on every thread."""
    import time
    R = referee(port)
    L = cgck.load()
    errs, stop = [], threading.Event()

    def work(t):
        try:
            rng = np.random.default_rng(7500 + t)
            sizes = [int(rng.integers(1, 6)) for _ in range(40)]
            frames = rxcorpus.corpus(rng, R, sum(sizes), clean=True)
            buf, desc_all, tx_base, tx_stride = rxcorpus.pool(frames, 200)
            raw, pool, size = rxcorpus.registered_copy(buf)
            assert L.cgck_host_register(pool.ctypes.data, size) == 0
            got, ref = pool[:len(buf)], buf.copy()
            descs, at = [], 0
            for s in sizes:
                descs.append(desc_all[at:at + s].copy())
                at += s
            cgck.burst_open(max_pkts=1024, max_bytes=4 << 20)
            try:
                fills, nxt = [], 0
                for k in range(len(sizes)):
                    assert cgck.rx_post(got, descs[k]) == sizes[k]
                    want = []
                    cgck.tx_begin()
                    for _ in range(2):
                        ln = int(rng.integers(40, 400))
                        pkt = tcp_pkt(rng, ln)
                        row = got[tx_base + nxt * tx_stride:tx_base + nxt * tx_stride + 2048]
                        row[14:14 + ln] = pkt
                        want.append((nxt, ln, expected(port, pkt, 16)))
                        tx_calls(row, ln, 16)
                        nxt += 1
                    assert cgck.tx_post() == 4
                    fills.append(want)
                    if k % 3 == 2:          # open three bursts, complete three fills
                        for j in range(k - 2, k + 1):
                            stack, ip_in, tcp_in = FLAGS[(j * 5 + t) % len(FLAGS)]
                            d = descs[j]
                            a = port.replay_rx(*R.fn_pointers(), ref, d.view(np.uint8), len(d), stack, ip_in,
                                               tcp_in)
                            cgck.rx_begin_posted()
                            try:
                                b = port.replay_rx(*cgck.fn_pointers(), got, d.view(np.uint8), len(d), stack,
                                                   ip_in, tcp_in)
                            finally:
                                cgck.rx_end()
                            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (t, j)
                            assert cgck.tx_complete() == 4
                            for s_, ln, r in fills[j]:
                                row = got[tx_base + s_ * tx_stride:tx_base + s_ * tx_stride + 2048]
                                assert np.array_equal(row[14:14 + ln], r), (t, j, s_)
                    time.sleep(0.0005)
                while cgck.rx_pending():
                    cgck.rx_begin_posted()
                    cgck.rx_end()
                while cgck.tx_pending():
                    cgck.tx_complete()
            finally:
                cgck.burst_close()
                L.cgck_host_unregister(pool.ctypes.data)
        except Exception as e:  # noqa: BLE001 — reported below
            errs.append(repr(e))
        finally:
            cgck.thread_release()

    th = [threading.Thread(target=work, args=(t,)) for t in range(3)]
    for x in th:
        x.start()
    cycles = 0
    while any(x.is_alive() for x in th):
        raw, other, size = rxcorpus.registered_copy(np.zeros(16384, np.uint8))
        assert L.cgck_host_register(other.ctypes.data, size) == 0
        time.sleep(0.002)
        assert L.cgck_host_unregister(other.ctypes.data) == 0
        del other, raw
        cycles += 1
    for x in th:
        x.join()
    assert not errs, errs
    assert cycles > 0


def test_verify_outside_rx_window_counted(port):
    """include/cgck.h: with the TX window open, a received frame verified
    outside an RX window looks like a transmit call and is queued (the stack
    gets 0).  cgck_window_stats_n's [4] counts such calls on the headers of
    the last closed RX window's frames, and nothing else."""
    R = referee(port)
    L = cgck.load()
    rng = np.random.default_rng(5330)
    buf, desc = rxcorpus.ring(rxcorpus.corpus(rng, R, 24, clean=True))
    raw, ring, size = rxcorpus.registered_copy(np.concatenate([buf, np.zeros(4 * 2048, np.uint8)]))
    assert L.cgck_host_register(ring.ctypes.data, size) == 0
    got = ring[:len(buf)]
    tx = ring[len(buf):len(buf) + 4 * 2048].reshape(4, 2048)
    try:
        cgck.tx_begin()
        s0 = cgck.window_stats_n()
        assert len(s0) == 5
        cgck.rx_begin(got, desc)
        try:
            port.replay_rx(*cgck.fn_pointers(), got, desc.view(np.uint8), len(desc), 0, 2, 2)
        finally:
            cgck.rx_end()
        s1 = cgck.window_stats_n()
        assert s1[4] == s0[4]                          # inside the window: answered, not counted
        for k in range(3):                             # the missed path: verified after rx_end
            off = int(desc[k]["frame_off"]) + 14
            got[off + 10:off + 12] = 0
            assert cgck.ip_cksum(got, off) == 0        # queued (the hazard itself)
        for i in range(2):                             # a genuine transmit slot: not counted
            pkt = tcp_pkt(rng, 200)
            tx[i, 14:214] = pkt
            tx_calls(tx[i], 200, 16)
        s2 = cgck.window_stats_n()
        assert s2[4] - s1[4] == 3 and s2[2] - s1[2] == 3 + 4, (s1, s2)
        cgck.tx_flush()
    finally:
        L.cgck_host_unregister(ring.ctypes.data)


def test_thread_bind(port):
    """cgck_thread_bind picks the device of a worker's drop-in context before
    its first use (con-gen.c:1062-1100: workers bound by queue
    id modulo the devices); a binding to another device after the context
    exists is refused, and survives cgck_thread_release."""
    nd = cgck.device_count()
    errs = []

    def worker(q):
        try:
            dev = q % nd
            assert cgck.thread_bind(dev) == 0
            assert cgck.thread_device() == dev
            rng = np.random.default_rng(5340 + q)
            for _ in range(20):
                pkt = tcp_pkt(rng, int(rng.integers(40, 1501)))
                pkt[10:12] = 0
                assert cgck.ip_cksum(pkt) == port.in_cksum(pkt, 0, 20)
            if nd > 1:
                with pytest.raises(cgck.CgckError, match="already on device"):
                    cgck.thread_bind((dev + 1) % nd)
            with pytest.raises(cgck.CgckError, match="cgck_thread_bind: device"):
                cgck.thread_bind(nd)
            cgck.thread_release()
            assert cgck.thread_device() == dev
        except Exception as e:          # noqa: BLE001 - reported below
            errs.append((q, repr(e)))

    ths = [threading.Thread(target=worker, args=(q,)) for q in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs


def test_first_request_after_open(port):
    """The first request right after cgck_burst_open is served at once, cycle
    after cycle: the server's device-memory doorbell is zeroed by the host
    before the open returns (an asynchronous zeroing still in flight once
    wiped request 1's doorbell, which then waited out the 2 s bound)."""
    import time
    rng = np.random.default_rng(5350)
    worst = 0.0
    for k in range(60):
        cgck.burst_open(max_pkts=64, max_bytes=1 << 16)
        try:
            pkt = tcp_pkt(rng, int(rng.integers(40, 1501)))
            pkt[10:12] = 0
            t0 = time.monotonic()
            assert cgck.ip_cksum(pkt) == port.in_cksum(pkt, 0, 20), k
            worst = max(worst, time.monotonic() - t0)
        finally:
            cgck.burst_close()
    assert worst < 0.5, worst
