"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own
checksum unit (oracle/_ref/libref_cksum.so, built by oracle/build_ref.sh from
/root/reference/subr.c:119-223).  Run in the build container:

    make -C oracle && python tests/golden/make_golden.py

The reference has no tests, fixtures or known-answer vectors of its own
(SURVEY §4), so these files are what pins parity.  Every expected value below
is produced by calling the reference's in_cksum/udp_cksum; call-site verdicts
follow the reference call sites line by line (cited), with only the checksum
calls delegated to the reference build.  Packet bytes for the synthetic sets
come from the splitmix64 stream of SURVEY §8(d) (oracle.Port.stream_bytes);
the first 64 packets of each set are also stored raw, in hex, so the fixture
does not depend on the generator.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

SEED = 0xC0C0


def u16le(a, off):
    return int(a[off]) | (int(a[off + 1]) << 8)


def put16le(a, off, v):
    a[off] = v & 0xFF
    a[off + 1] = (v >> 8) & 0xFF


def main():
    R = oracle.reference()
    if R is None:
        sys.exit("make_golden: oracle/_ref/libref_cksum.so missing (run make -C oracle)")
    P = oracle.port()
    out = {}

    # (i) Textbook IPv4 header KAT (RFC 1071 style example): stored bytes b8 61.
    kat = np.frombuffer(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"), np.uint8).copy()
    out["kat_ipv4"] = {"hex": kat.tobytes().hex(), "in_cksum": R.in_cksum(kat, 0, 20)}

    # (ii) zero classes: all-0x00 (S == 0) and all-0xFF (S == k*65535), and
    # non-trivial regions whose sum is a multiple of 65535.
    zc = []
    for n in (0, 1, 2, 3, 7, 8, 20, 64, 1500):
        for fill in (0x00, 0xFF):
            a = np.full(max(n, 1), fill, np.uint8)
            zc.append({"fill": fill, "len": n, "in_cksum": R.in_cksum(a, 0, n)})
    rng = np.random.default_rng(7)
    crafted = []
    for n in (20, 44, 64, 100, 1480):
        a = rng.integers(0, 256, n, dtype=np.uint8)
        s = sum(u16le(a, i) for i in range(0, n - 1, 2)) % 65535
        v = (u16le(a, 0) - s) % 65535   # force S == 0 (mod 65535), S != 0
        put16le(a, 0, v)
        crafted.append({"hex": a.tobytes().hex(), "in_cksum": R.in_cksum(a, 0, n)})
    out["zero_class"] = {"fills": zc, "crafted": crafted}

    # (iii) every length 0..64 and the MTU-edge lengths at start offsets 0..15
    # of one fixed random buffer.
    buf = np.random.default_rng(11).integers(0, 256, 1600, dtype=np.uint8)
    lens = list(range(65)) + [575, 576, 1479, 1480, 1499, 1500, 1513, 1514]
    grid = [[R.in_cksum(buf, off, n) for n in lens] for off in range(16)]
    out["len_off_grid"] = {"buf_hex": buf.tobytes().hex(), "lens": lens, "in_cksum": grid}

    # udp_cksum at frame offset 14, ihl 5..15, random segments (tcp_output
    # style l4 length), odd lengths included.
    ug = []
    rng = np.random.default_rng(13)
    for i in range(256):
        frame = rng.integers(0, 256, 2048, dtype=np.uint8)
        ihl = 5 if i % 4 else int(rng.integers(5, 16))
        frame[14] = 0x40 | ihl
        l4 = int(rng.integers(0, 2048 - 14 - 4 * ihl))
        ug.append({"frame_hex": frame[: 14 + 4 * ihl + l4].tobytes().hex(), "l4len": l4,
                   "udp_cksum": R.udp_cksum(frame, 14, l4)})
    out["udp_frames"] = ug
    with open(os.path.join(HERE, "basic.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))

    # (iv) synthetic batches: expected (ip, tcp) for 4096 packets of 64 B,
    # 1500 B (stride = length, dense) and IMIX, checksum fields zeroed.
    synth = {"seed": SEED, "sets": {}}
    for name, stride, ln in (("64", 64, 64), ("1500", 1500, 1500)):
        exp, raw = [], []
        for k in range(4096):
            pkt = P.synth_packet(k, stride, ln, SEED)
            exp.append([R.in_cksum(pkt, 0, 20), R.udp_cksum(pkt, 0, ln - 20)])
            if k < 64:
                raw.append(pkt.tobytes().hex())
        synth["sets"][name] = {"stride": stride, "ip_len": ln, "expect": exp, "raw_hex": raw}
    exp, raw, desc = [], [], []
    for k in range(4096):
        off, ln = P.imix_desc(k)
        pkt = P.stream_bytes(off, ln, SEED)
        P.stamp_header(pkt, 0, ln)
        exp.append([R.in_cksum(pkt, 0, 20), R.udp_cksum(pkt, 0, ln - 20)])
        desc.append([off, ln])
        if k < 64:
            raw.append(pkt.tobytes().hex())
    synth["sets"]["imix"] = {"desc": desc, "expect": exp, "raw_hex": raw}
    with open(os.path.join(HERE, "synth.json"), "w") as f:
        json.dump(synth, f, separators=(",", ":"))

    # (v) verify-verdict vectors.  Packets are finalized the way the TX path
    # does it (tcp_output.c:416-418 then ip_output.c:61-64; udp_usrreq.c:186-190),
    # then corrupted; verdicts follow the RX call sites exactly.
    def tx_fill(p, proto, l4len):
        hl = (p[0] & 15) * 4
        fo = 16 if proto == 6 else 6
        put16le(p, hl + fo, 0)
        put16le(p, hl + fo, R.udp_cksum(p, 0, l4len))
        put16le(p, 10, 0)
        put16le(p, 10, R.in_cksum(p, 0, hl))

    def bsd_ip_input(p):  # ip_input.c:45-58
        q = p.copy()
        s = u16le(q, 10)
        s = 0xFFFF if s == 0 else s
        put16le(q, 10, 0)
        return int(R.in_cksum(q, 0, (q[0] & 15) * 4) == s)

    def bsd_tcp_input(p, l4len):  # tcp_input.c:75-85
        q = p.copy()
        hl = (q[0] & 15) * 4
        s = u16le(q, hl + 16)
        put16le(q, hl + 16, 0)
        return int(R.udp_cksum(q, 0, l4len) == s)

    def bsd_udp_input(p, l4len):  # udp_usrreq.c:86-94
        q = p.copy()
        hl = (q[0] & 15) * 4
        s = u16le(q, hl + 6)
        if s == 0:
            return 1
        put16le(q, hl + 6, 0)
        return int(R.udp_cksum(q, 0, l4len) == s)

    def toy_ip(p):  # gbtcp/inet.c:319-330
        q = p.copy()
        s = u16le(q, 10)
        put16le(q, 10, 0)
        return int(R.in_cksum(q, 0, (q[0] & 15) * 4) == s)

    def toy_tcp(p, l4len):  # gbtcp/inet.c:142-153
        q = p.copy()
        hl = (q[0] & 15) * 4
        s = u16le(q, hl + 16)
        put16le(q, hl + 16, 0)
        return int(R.udp_cksum(q, 0, l4len) == s)

    rng = np.random.default_rng(17)
    cases = []

    def add(kind, p, proto, l4len):
        e = {"kind": kind, "hex": p.tobytes().hex(), "proto": proto, "ip_len": len(p),
             "bsd_ip": bsd_ip_input(p), "toy_ip": toy_ip(p)}
        if proto == 6:
            e["bsd_l4"] = bsd_tcp_input(p, l4len)
            e["toy_l4"] = toy_tcp(p, l4len)
        else:
            e["bsd_l4"] = bsd_udp_input(p, l4len)
        cases.append(e)

    for i in range(64):
        proto = 6 if i % 4 else 17
        ln = int(rng.choice([40, 41, 64, 99, 576, 1500]))
        p = rng.integers(0, 256, ln, dtype=np.uint8)
        ihl = 5 if i % 8 else 6
        p[0] = 0x40 | ihl
        p[9] = proto
        p[2], p[3] = ln >> 8, ln & 0xFF
        l4 = ln - 4 * ihl
        tx_fill(p, proto, l4)
        add("good", p, proto, l4)
        q = p.copy()
        j = int(rng.integers(4 * ihl, ln))
        q[j] ^= 1 << int(rng.integers(0, 8))
        add("payload_flip", q, proto, l4)
        q = p.copy()
        q[int(rng.choice([1, 4, 5, 8, 12, 19]))] ^= 0x10
        add("header_flip", q, proto, l4)
        if proto == 17:
            q = p.copy()
            put16le(q, 4 * ihl + 6, 0)
            add("udp_zero_sum", q, proto, l4)
    # stored ip_sum 0x0000 where the correct value is 0xFFFF: craft a header
    # whose word sum is a multiple of 65535 (then in_cksum == 0xFFFF).
    for i in range(8):
        p = rng.integers(0, 256, 60, dtype=np.uint8)
        p[0] = 0x45
        p[9] = 6
        p[2], p[3] = 0, 60
        tx_fill(p, 6, 40)
        put16le(p, 10, 0)
        s = sum(u16le(p, k) for k in range(0, 20, 2)) % 65535
        put16le(p, 4, (u16le(p, 4) - s) % 65535)   # retune ip_id
        assert R.in_cksum(p, 0, 20) == 0xFFFF
        tx_fill(p, 6, 40)                          # L4 again (pseudo unchanged), ip_sum = 0xFFFF
        add("ip_sum_ffff", p.copy(), 6, 40)
        q = p.copy()
        put16le(q, 10, 0)
        add("ip_sum_zero_for_ffff", q, 6, 40)
    with open(os.path.join(HERE, "verify.json"), "w") as f:
        json.dump({"cases": cases}, f, separators=(",", ":"))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
