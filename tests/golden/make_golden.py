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


if __name__ == "__main__" and len(sys.argv) == 1:
    main()
    rss_main()


# ---------------------------------------------------------------------------
# Toeplitz RSS fixtures: tests/golden/rss.json.
#     python tests/golden/make_golden.py rss
# Expected hashes come from the reference's own toeplitz_hash / rss_hash4
# (oracle/_ref/libref_rss.so, built from subr.c:29-35, 482-530).  The
# dst-cache sets run the loop of con-gen.c:291-360 (restated in
# oracle/rss_oracle.c) with the REFERENCE's rss_hash4 as its hash, and store
# the count, a SHA-256 of the entries and the first/last 32 entries.
# ---------------------------------------------------------------------------

MS_RSS = [  # Microsoft RSS verification suite, default key: (dst, dport, src, sport, ipv4, ipv4+tcp)
    ("161.142.100.80", 1766, "66.9.149.187", 2794, 0x323e8fc2, 0x51ccc178),
    ("65.69.140.83", 4739, "199.92.111.2", 14230, 0xd718262a, 0xc626b0ea),
    ("12.22.207.184", 38024, "24.19.198.95", 12898, 0xd2d0a5de, 0x5c2b394a),
    ("209.142.163.6", 2217, "38.27.205.30", 48228, 0x82989176, 0xafc7327f),
    ("202.188.127.2", 1303, "153.39.163.191", 44251, 0x5d1809c5, 0x10e828a2),
]


def ip4(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def htonl(x):
    return int.from_bytes(x.to_bytes(4, "big"), "little")


def htons(x):
    return int.from_bytes(x.to_bytes(2, "big"), "little")


DST_SETS = [  # name, laddr range, faddr range, port, queue_num, queue_id, key, cap
    ("default_q4", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.1", 80, 4, 1, "freebsd", 100000),
    ("straddle_q8", "10.0.0.1", "10.0.0.2", "10.1.0.1", "10.1.0.3", 8080, 8, 7, "freebsd", 5000),
    ("no_filter_id128", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.2", 80, 4, 128, "freebsd", 70000),
    ("no_filter_num1", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.9", 443, 1, 0, "freebsd", 1000),
    ("id_above_num", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.1", 80, 4, 5, "freebsd", 100000),
    ("many_tiles_q16", "10.0.0.1", "10.0.0.1", "10.2.0.0", "10.2.0.199", 80, 16, 3, "freebsd", 100000),
    ("nf63_q2", "192.168.0.1", "192.168.0.2", "172.16.0.1", "172.16.0.63", 80, 2, 0, "freebsd", 1 << 22),
    ("nf64_q3", "192.168.0.1", "192.168.0.1", "172.16.0.0", "172.16.0.63", 80, 3, 2, "freebsd", 1 << 22),
    ("nf65_q5", "192.168.0.1", "192.168.0.1", "172.16.0.0", "172.16.0.64", 53, 5, 4, "freebsd", 1 << 22),
    ("nf130_q7", "192.168.0.1", "192.168.0.1", "172.16.0.0", "172.16.0.129", 53, 7, 0, "freebsd", 1 << 22),
    ("key52_q3", "10.0.0.1", "10.0.0.3", "10.1.0.1", "10.1.0.4", 80, 3, 2, "random52", 300000),
    ("key16_q12", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.4", 80, 12, 11, "random16", 20000),
    ("cap1", "10.0.0.1", "10.0.0.1", "10.1.0.1", "10.1.0.1", 80, 4, 1, "freebsd", 1),
    ("full_range_zero_n", "0.0.0.0", "255.255.255.255", "10.1.0.1", "10.1.0.1", 80, 4, 1, "freebsd", 100),
    ("wrapped_n", "10.0.0.0", "10.0.255.255", "10.1.0.0", "10.1.0.255", 80, 2, 1, "freebsd", 200000),
]


def rss_main():
    import hashlib
    RR = oracle.reference_rss()
    if RR is None:
        sys.exit("make_golden: oracle/_ref/libref_rss.so missing (run make -C oracle)")
    P = oracle.port()
    key = RR.key
    rng = np.random.default_rng(23)
    keys = {"freebsd": key, "random52": rng.integers(0, 256, 52, dtype=np.uint8),
            "random16": rng.integers(0, 256, 16, dtype=np.uint8)}
    out = {"freebsd_rss_key": key.tobytes().hex(),
           "keys": {k: v.tobytes().hex() for k, v in keys.items()}}

    # Published vectors, checked against the reference build here.
    ms = []
    for dst, dp, src, sp, h2, h4 in MS_RSS:
        d4 = np.frombuffer(ip4(src).to_bytes(4, "big") + ip4(dst).to_bytes(4, "big")
                           + sp.to_bytes(2, "big") + dp.to_bytes(2, "big"), np.uint8)
        assert RR.toeplitz_hash(d4, key) == h4 and RR.toeplitz_hash(d4[:8], key) == h2
        r4 = RR.rss_hash4(htonl(ip4(dst)), htonl(ip4(src)), htons(dp), htons(sp), key)
        ms.append({"data_hex": d4.tobytes().hex(), "ipv4": h2, "ipv4_tcp": h4, "rss_hash4": r4,
                   "laddr": htonl(ip4(dst)), "faddr": htonl(ip4(src)), "lport": htons(dp),
                   "fport": htons(sp)})
    out["ms_vectors"] = ms

    # toeplitz_hash over random data: every cnt 0..48 and 100, 1500 for a set
    # of key sizes (key_size < 4 still reads key[0..3], subr.c:489).
    buf = rng.integers(0, 256, 1600, dtype=np.uint8)
    kbuf = rng.integers(0, 256, 64, dtype=np.uint8)
    cnts = list(range(49)) + [100, 1500]
    ksz = [2, 4, 5, 12, 16, 40, 52, 64]
    grid = [[RR.toeplitz_hash(buf, kbuf, c, ks) for c in cnts] for ks in ksz]
    out["toeplitz_grid"] = {"data_hex": buf.tobytes().hex(), "key_hex": kbuf.tobytes().hex(),
                            "cnts": cnts, "key_sizes": ksz, "hash": grid}

    # 4096 random 12-byte tuples (dense records) with the default key.
    tup = rng.integers(0, 256, 4096 * 12, dtype=np.uint8)
    out["tuples12"] = {"data_hex": tup.tobytes().hex(),
                       "hash": [RR.toeplitz_hash(tup[12 * k:12 * k + 12], key) for k in range(4096)]}

    dsets = []
    ref_fn = RR.fn_rss_hash4()
    for name, l0, l1, f0, f1, port, qn, qi, kname, cap in DST_SETS:
        k = keys[kname]
        ents = P.dst_cache(ip4(l0), ip4(l1), ip4(f0), ip4(f1), htons(port), qn, qi, k, cap,
                           hash_fn=ref_fn)
        dsets.append({"name": name, "laddr": [ip4(l0), ip4(l1)], "faddr": [ip4(f0), ip4(f1)],
                      "fport": htons(port), "queue_num": qn, "queue_id": qi, "key": kname,
                      "cap": cap, "count": len(ents),
                      "sha256": hashlib.sha256(ents.tobytes()).hexdigest(),
                      "head": ents[:32].tobytes().hex(), "tail": ents[-32:].tobytes().hex()})
        print(f"  dst set {name}: {len(ents)} entries")
    out["dst_sets"] = dsets
    with open(os.path.join(HERE, "rss.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("rss fixtures written to", HERE)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "rss":
    rss_main()
