"""CPU tests of the RX-window test infrastructure and of the drop-in failure
path (no GPU needed).

* oracle/stack_replay.c restates the reference stacks' RX call sequences;
  here it is checked against the reference's own rules (ip_input.c:45-58,
  tcp_input.c:75-85, udp_usrreq.c:86-94, ip_icmp.c:187-193,
  gbtcp/inet.c:142-153, 319-330) on crafted frames, and the restated
  checksum functions against the reference build through it.
* cgck_set_error_handler: a drop-in call that cannot reach a device calls
  the handler (con-gen's panic3 in production); without one it aborts.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import cgck
import oracle
import rxcorpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = oracle.Port


def replay(port, fns, frames, stack, ip_in, tcp_in):
    buf, desc = rxcorpus.ring(frames)
    res, ctr = port.replay_rx(fns[0], fns[1], buf, desc.view(np.uint8), len(desc), stack, ip_in, tcp_in)
    return res, ctr, buf


def ctr_dict(ctr):
    return dict(zip(P.COUNTERS, (int(x) for x in ctr)))


def test_replay_policy_rules(port):
    """The 0/1/2 flag semantics and the zero-field conventions, frame by frame."""
    rng = np.random.default_rng(3)
    fns = port.fn_pointers()
    good = rxcorpus.frame(rng, port, 6, 100)
    bad_ip = good.copy()
    bad_ip[10] ^= 1
    bad_tcp = good.copy()
    bad_tcp[-1] ^= 1

    # bsd ip_input.c:50-56: any nonzero flag counts and drops
    for f in (1, 2):
        res, ctr, _ = replay(port, fns, [bad_ip], 0, f, 2)
        assert res[0] == P.R_DROP_IP and ctr_dict(ctr)["ips_badsum"] == 1
    res, ctr, buf = replay(port, fns, [bad_ip], 0, 0, 2)
    assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["ips_badsum"] == 0 and ctr_dict(ctr)["in_calls"] == 0
    assert buf[rxcorpus.L2 + 10] == 0 and buf[rxcorpus.L2 + 11] == 0   # :49 zeroed, not recomputed
    # gbtcp inet.c:321-328: 1 counts, 2 drops; the field is restored when not dropped
    res, ctr, buf = replay(port, fns, [bad_ip], 1, 1, 2)
    assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["ips_badsum"] == 1
    assert np.array_equal(buf[rxcorpus.L2:rxcorpus.L2 + len(bad_ip)], bad_ip)
    res, ctr, _ = replay(port, fns, [bad_ip], 1, 2, 2)
    assert res[0] == P.R_DROP_IP and ctr_dict(ctr)["ips_badsum"] == 1
    # tcp_input.c:79-83 / inet.c:146-150: 1 counts, 2 drops
    for stack in (0, 1):
        res, ctr, _ = replay(port, fns, [bad_tcp], stack, 1, 1)
        assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["tcps_rcvbadsum"] == 1
        res, ctr, _ = replay(port, fns, [bad_tcp], stack, 1, 2)
        assert res[0] == P.R_DROP_L4 and ctr_dict(ctr)["tcps_rcvbadsum"] == 1
        res, ctr, _ = replay(port, fns, [good], stack, 2, 2)
        assert res[0] == P.R_ACCEPT and sum(ctr[:4]) == 0 and ctr_dict(ctr)["udp_calls"] == 1

    # ip_sum 0x0000 where the computed value is 0xFFFF: bsd maps it (:46-48), gbtcp does not
    # (retune ip_id so the header's word sum is a multiple of 65535)
    p = rxcorpus.frame(rng, port, 6, 40)
    rxcorpus.le16(p, 10, 0)
    s = sum(int(p[k]) | int(p[k + 1]) << 8 for k in range(0, 20, 2)) % 65535
    rxcorpus.le16(p, 4, ((int(p[4]) | int(p[5]) << 8) - s) % 65535)
    assert port.in_cksum(p, 0, 20) == 0xFFFF              # ip_sum stays stored as 0
    rxcorpus.le16(p, 20 + 16, 0)
    rxcorpus.le16(p, 20 + 16, port.udp_cksum(p, 0, 40))
    res, ctr, _ = replay(port, fns, [p], 0, 2, 2)
    assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["ips_badsum"] == 0
    res, ctr, _ = replay(port, fns, [p], 1, 2, 2)
    assert res[0] == P.R_DROP_IP and ctr_dict(ctr)["ips_badsum"] == 1

    # udp_usrreq.c:86: uh_sum == 0 is not checked
    u = rxcorpus.frame(rng, port, 17, 64)
    rxcorpus.le16(u, 26, 0)
    rxcorpus.le16(u, 10, 0)
    rxcorpus.le16(u, 10, port.in_cksum(u, 0, 20))
    res, ctr, _ = replay(port, fns, [u], 0, 2, 2)
    assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["udp_calls"] == 0
    u[30] ^= 4                                            # payload change, still unchecked
    res, ctr, _ = replay(port, fns, [u], 0, 2, 2)
    assert res[0] == P.R_ACCEPT and ctr_dict(ctr)["udps_badsum"] == 0
    # ip_icmp.c:189-192: a bad ICMP checksum counts and drops (no flag)
    c = rxcorpus.frame(rng, port, 1, 64)
    c[40] ^= 1
    res, ctr, _ = replay(port, fns, [c], 0, 0, 0)
    assert res[0] == P.R_DROP_L4 and ctr_dict(ctr)["icps_checksum"] == 1 and ctr_dict(ctr)["in_calls"] == 1


def test_replay_reference_vs_restatement(port):
    """The same replay with the reference's in_cksum/udp_cksum (oracle/_ref)
    and with the restatement: identical outcomes, counters and bytes over a
    corpus of every edge shape."""
    R = oracle.reference()
    if R is None:
        pytest.skip("reference build absent (oracle/_ref)")
    rng = np.random.default_rng(11)
    frames = rxcorpus.corpus(rng, R, 600)
    for stack in (0, 1):
        for ip_in, tcp_in in ((0, 0), (1, 1), (2, 2), (1, 2), (2, 1)):
            a = replay(port, R.fn_pointers(), frames, stack, ip_in, tcp_in)
            b = replay(port, port.fn_pointers(), frames, stack, ip_in, tcp_in)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
            if ip_in and tcp_in:
                assert a[1][4] > 0 and a[1][5] > 0


def _run(code):
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                          timeout=120)


PRELUDE = ("import os, sys\n"
           "sys.path.insert(0, 'con-gen_amd')\n"
           "import numpy as np, cgck\n"
           "if cgck.device_count() > 0:\n"
           "    os._exit(99)\n")


def test_error_handler_receives_dropin_failure():
    """No device: in_cksum cannot produce a value and calls the handler with
    what failed and why (con-gen passes one that ends in panic3)."""
    r = _run(PRELUDE +
             "def h(what, msg):\n"
             "    print('HANDLER|' + what + '|' + msg, flush=True)\n"
             "    os._exit(7)\n"
             "cgck.set_error_handler(h)\n"
             "cgck.in_cksum(np.zeros(20, np.uint8), 0, 20)\n")
    if r.returncode == 99:
        pytest.skip("a device is visible")
    assert r.returncode == 7, r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("HANDLER|")][0]
    _, what, msg = line.split("|", 2)
    assert "no gfx950 context" in what and "no HIP device" in msg


def test_dropin_failure_aborts_without_handler():
    r = _run(PRELUDE + "cgck.udp_cksum(np.zeros(64, np.uint8), 0, 44)\n")
    if r.returncode == 99:
        pytest.skip("a device is visible")
    assert r.returncode == -6 and "libcgck:" in r.stderr and "no HIP device" in r.stderr


def test_thread_ctx_and_rx_begin_without_device():
    if cgck.device_count() > 0:
        pytest.skip("a device is visible")
    L = cgck.load()
    assert not L.cgck_thread_ctx()
    assert b"no HIP device" in L.cgck_last_error()
    buf, desc = rxcorpus.ring([np.zeros(40, np.uint8)])
    with pytest.raises(cgck.CgckError, match="no HIP device"):
        cgck.rx_begin(buf, desc)
    assert cgck.window_stats() == [0, 0, 0, 0]


# ---------------------------------------------------------------------------
# bsd44 with the packets RX processing sends back (oracle_replay_rx_rsp)
# ---------------------------------------------------------------------------

def rsp_replay(port, fns, buf, desc, tx_base, tx_stride, cap, ip_in, tcp_in, ka=None, ip_id=77):
    local = np.zeros(2048 * 64, np.uint8)
    tx = buf[tx_base:]
    res, ctr, txs, idn = port.replay_rx_rsp(fns[0], fns[1], buf, desc.view(np.uint8), len(desc), ip_in, tcp_in,
                                            tx, tx_stride, cap, local, rxcorpus.LADDR, ka, ip_id)
    return res, ctr, txs, idn, local


def keepalives(rng, n):
    ka = np.zeros(n, P.KA_DTYPE)
    ka["laddr"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    ka["faddr"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    ka["lport"] = rng.integers(0, 2 ** 16, n)
    ka["fport"] = rng.integers(0, 2 ** 16, n)
    ka["rcv_nxt"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    ka["snd_una"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    ka["hiwat"] = rng.integers(0, 2 ** 20, n)
    ka["scale"] = rng.integers(0, 9, n)
    return ka


def test_rsp_replay_reference_vs_restatement(port):
    """The response replay over the reference's own in_cksum / udp_cksum and
    over the restatement: outcomes, counters, replies sent and every byte of
    both rings equal; every reply carries checksums that verify."""
    R = oracle.reference()
    if R is None:
        pytest.skip("reference build absent")
    rng = np.random.default_rng(81)
    frames = rxcorpus.rsp_corpus(rng, R, 600)
    buf, desc, tx_base, tx_stride = rxcorpus.pool(frames, 700)
    ka = keepalives(rng, 20)
    a = rsp_replay(port, R.fn_pointers(), buf.copy(), desc, tx_base, tx_stride, 700, 1, 1, ka)
    b_buf = buf.copy()
    b = rsp_replay(port, port.fn_pointers(), b_buf, desc, tx_base, tx_stride, 700, 1, 1, ka)
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    txs = b[2]
    assert txs[1] == 0 and txs[0] == txs[2:].sum()
    assert min(txs[2:]) > 0, txs                      # RSTs, ICMP errors, echo replies, keepalives
    assert sum(1 for r in b[0] if r == P.R_NOTOURS) > 0
    # each reply's checksums verify (zero the field, recompute, compare)
    for j in range(int(txs[0])):
        ip = b_buf[tx_base + j * tx_stride + 14:]
        hl = (int(ip[0]) & 15) * 4
        tot = int(ip[2]) << 8 | int(ip[3])
        h = ip[:hl].copy()
        stored = h[10:12].copy()
        h[10:12] = 0
        assert np.frombuffer(np.uint16(port.in_cksum(h, 0, hl)).tobytes(), np.uint8).tolist() == stored.tolist()
        pkt = ip[:tot].copy()
        if pkt[9] == 6:
            st = pkt[hl + 16:hl + 18].copy()
            pkt[hl + 16:hl + 18] = 0
            assert np.uint16(port.udp_cksum(pkt, 0, tot - hl)).tobytes() == st.tobytes(), j
        else:
            assert pkt[9] == 1
            st = pkt[hl + 2:hl + 4].copy()
            pkt[hl + 2:hl + 4] = 0
            assert np.uint16(port.in_cksum(pkt, hl, tot - hl)).tobytes() == st.tobytes(), j


def test_rsp_replay_ring_full_uses_pkt_body(port):
    """With the transmit ring full the replies are built in pkt_body
    (netmap_init_tx_packet, netmap.c:74-83): same bytes either way."""
    rng = np.random.default_rng(82)
    frames = rxcorpus.rsp_corpus(rng, port, 120)
    buf, desc, tx_base, tx_stride = rxcorpus.pool(frames, 130)
    fns = port.fn_pointers()
    full = rsp_replay(port, fns, buf.copy(), desc, tx_base, tx_stride, 130, 2, 2)
    part_buf = buf.copy()
    part = rsp_replay(port, fns, part_buf, desc, tx_base, tx_stride, 16, 2, 2)
    assert part[2][0] == 16 and part[2][1] == full[2][0] - 16
    assert np.array_equal(full[0], part[0]) and np.array_equal(full[1], part[1])
    # the packets past the ring equal the ring-built ones of the full replay
    full_buf = buf.copy()
    rsp_replay(port, fns, full_buf, desc, tx_base, tx_stride, 130, 2, 2)
    for j in range(16, int(full[2][0])):
        want = full_buf[tx_base + j * tx_stride:tx_base + j * tx_stride + 1514]
        got = part[4][(j - 16) * 2048:(j - 16) * 2048 + 1514]
        ln = 14 + (int(want[16]) << 8 | int(want[17]))
        assert np.array_equal(want[:ln], got[:ln]), j
