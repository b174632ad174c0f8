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
