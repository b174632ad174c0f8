"""CPU tests of the oracle (the referee): its C restatement of subr.c:119-223
against the golden fixtures generated from the reference's own checksum unit,
and against that reference build directly where it is present."""
import numpy as np
import pytest

import oracle


def hexa(s):
    return np.frombuffer(bytes.fromhex(s), np.uint8).copy()


def test_kat_ipv4_header(port, golden_basic):
    kat = golden_basic["kat_ipv4"]
    a = hexa(kat["hex"])
    v = port.in_cksum(a, 0, 20)
    assert v == kat["in_cksum"]
    # stored verbatim into the header the bytes read b8 61
    assert np.array([v], "<u2").tobytes() == b"\xb8\x61"


def test_zero_classes(port, golden_basic):
    for z in golden_basic["zero_class"]["fills"]:
        a = np.full(max(z["len"], 1), z["fill"], np.uint8)
        assert port.in_cksum(a, 0, z["len"]) == z["in_cksum"]
        if z["fill"] == 0 or z["len"] % 2 == 0:   # S == 0 or S == k*65535
            assert z["in_cksum"] == 0xFFFF
    for c in golden_basic["zero_class"]["crafted"]:
        a = hexa(c["hex"])
        assert port.in_cksum(a, 0, len(a)) == c["in_cksum"] == 0xFFFF


def test_length_offset_grid(port, golden_basic):
    g = golden_basic["len_off_grid"]
    buf = hexa(g["buf_hex"])
    for off in range(16):
        got = [port.in_cksum(buf, off, n) for n in g["lens"]]
        assert got == g["in_cksum"][off], f"offset {off}"


def test_udp_frames(port, golden_basic):
    for f in golden_basic["udp_frames"]:
        fr = hexa(f["frame_hex"])
        assert port.udp_cksum(fr, 14, f["l4len"]) == f["udp_cksum"]


@pytest.mark.parametrize("name", ["64", "1500"])
def test_synth_strided_sets(port, golden_synth, name):
    s = golden_synth["sets"][name]
    seed = golden_synth["seed"]
    for k, (ip, tcp) in enumerate(s["expect"]):
        pkt = port.synth_packet(k, s["stride"], s["ip_len"], seed)
        if k < len(s["raw_hex"]):
            assert pkt.tobytes().hex() == s["raw_hex"][k]
        assert port.in_cksum(pkt, 0, 20) == ip
        assert port.udp_cksum(pkt, 0, s["ip_len"] - 20) == tcp


def test_synth_imix_set(port, golden_synth):
    s = golden_synth["sets"]["imix"]
    seed = golden_synth["seed"]
    for k, ((off, ln), (ip, tcp)) in enumerate(zip(s["desc"], s["expect"])):
        assert port.imix_desc(k) == (off, ln)
        pkt = port.stream_bytes(off, ln, seed)
        port.stamp_header(pkt, 0, ln)
        if k < len(s["raw_hex"]):
            assert pkt.tobytes().hex() == s["raw_hex"][k]
        assert (port.in_cksum(pkt, 0, 20), port.udp_cksum(pkt, 0, ln - 20)) == (ip, tcp)


def test_batch_referee_matches_fixture(port, golden_synth):
    """The batch referee (used against the GPU) reproduces the fixture."""
    s = golden_synth["sets"]["1500"]
    n = 512
    buf = np.concatenate([port.synth_packet(k, 1500, 1500, golden_synth["seed"]) for k in range(n)])
    out, ver = port.batch_strided(buf, n, 1500, 0, 1500, oracle_flags("GEN_BOTH"))
    exp = np.array(s["expect"][:n], np.uint32)
    assert np.array_equal(out & 0xFFFF, exp[:, 0])
    assert np.array_equal(out >> 16, exp[:, 1])
    assert not ver.any()
    bad, chk = port.check_synth_strided(n, 1500, 1500, golden_synth["seed"],
                                        oracle_flags("GEN_BOTH"), out)
    assert (bad, chk) == (0, n)


def oracle_flags(name):
    import cgck
    return getattr(cgck, name)


def test_call_site_verdicts(port, golden_verify):
    """Call-site semantics a11-a14, a16 against the reference-derived verdicts."""
    for c in golden_verify["cases"]:
        p = hexa(c["hex"])
        hl = (int(p[0]) & 15) * 4
        l4 = c["ip_len"] - hl
        assert port.lib.oracle_bsd_ip_input_verify(p.copy().ctypes.data) == c["bsd_ip"], c["kind"]
        assert port.lib.oracle_toy_ip_verify(p.copy().ctypes.data) == c["toy_ip"], c["kind"]
        if c["proto"] == 6:
            assert port.lib.oracle_bsd_tcp_input_verify(p.copy().ctypes.data, l4) == c["bsd_l4"]
            assert port.lib.oracle_toy_tcp_verify(p.copy().ctypes.data, l4) == c["toy_l4"]
        else:
            assert port.lib.oracle_bsd_udp_input_verify(p.copy().ctypes.data, l4) == c["bsd_l4"]


def test_batch_referee_verify_flags(port, golden_verify):
    """oracle_packet's VERIFY flags reproduce the call-site verdicts."""
    import cgck
    for c in golden_verify["cases"]:
        p = hexa(c["hex"])
        o = np.zeros(1, np.uint32)
        v = port.lib.oracle_packet(p.ctypes.data, c["ip_len"], cgck.VERIFY_BSD,
                                   o.ctypes.data_as(oracle._u32p))
        assert (v & 1) == (1 - c["bsd_ip"]), c["kind"]
        assert ((v >> 1) & 1) == (1 - c["bsd_l4"]), c["kind"]
        if c["proto"] == 6:
            v = port.lib.oracle_packet(p.ctypes.data, c["ip_len"], cgck.VERIFY_TOY,
                                       o.ctypes.data_as(oracle._u32p))
            assert (v & 1) == (1 - c["toy_ip"]) and ((v >> 1) & 1) == (1 - c["toy_l4"])


def test_fill_matches_call_sites(port):
    """FILL (STORE) in the referee == tcp_output.c:416-418 + ip_output.c:61-64."""
    import cgck
    rng = np.random.default_rng(3)
    for i in range(200):
        ln = int(rng.integers(40, 1501))
        p = rng.integers(0, 256, ln, dtype=np.uint8)
        p[0] = 0x45
        p[9] = 6
        a = p.copy()
        port.lib.oracle_tcp_output_fill(a.ctypes.data, ln - 20)
        port.lib.oracle_ip_output_fill(a.ctypes.data)
        b = p.copy()
        o = np.zeros(1, np.uint32)
        port.lib.oracle_packet(b.ctypes.data, ln, cgck.FILL_BOTH, o.ctypes.data_as(oracle._u32p))
        assert np.array_equal(a, b)


@pytest.mark.skipif(oracle.reference() is None, reason="reference build absent")
def test_port_vs_reference_random():
    """Differential: restatement vs the reference's own subr.c unit."""
    P, R = oracle.port(), oracle.reference()
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    for _ in range(20000):
        off = int(rng.integers(0, 16))
        n = int(rng.integers(0, 1700))
        assert P.in_cksum(buf, off, n) == R.in_cksum(buf, off, n)
        o2 = int(rng.integers(0, 16))
        buf[o2] = (int(buf[o2]) & 0xF0) | int(rng.integers(0, 16))
        hl = (int(buf[o2]) & 15) * 4
        n2 = int(rng.integers(0, 4096 - o2 - hl))
        assert P.udp_cksum(buf, o2, n2) == R.udp_cksum(buf, o2, n2)
