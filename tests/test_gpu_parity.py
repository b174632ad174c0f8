"""GPU parity: the gfx950 kernels (through the C-ABI) against the golden
fixtures made from the reference's own subr.c checksum unit and against the
oracle referee on the same bytes.  Integer work: every comparison is
bit-exact.  Run on an MI355X with `pytest -m gpu`."""
import ctypes

import numpy as np
import pytest

import cgck
import memdiag

pytestmark = pytest.mark.gpu

SEED = 0xC0C0


def hexa(s):
    return np.frombuffer(bytes.fromhex(s), np.uint8).copy()


# ---------------------------------------------------------------------------
# Drop-in symbols (subr.h:373-374) against the reference-made fixtures
# ---------------------------------------------------------------------------

def test_dropin_kat(engine, golden_basic):
    kat = golden_basic["kat_ipv4"]
    a = hexa(kat["hex"])
    assert cgck.in_cksum(a, 0, 20) == kat["in_cksum"]
    assert cgck.ip_cksum(a, 0) == kat["in_cksum"]


def test_dropin_zero_classes(engine, golden_basic):
    for z in golden_basic["zero_class"]["fills"]:
        a = np.full(max(z["len"], 1), z["fill"], np.uint8)
        assert cgck.in_cksum(a, 0, z["len"]) == z["in_cksum"], z
    for c in golden_basic["zero_class"]["crafted"]:
        a = hexa(c["hex"])
        assert cgck.in_cksum(a, 0, len(a)) == c["in_cksum"]


def test_dropin_length_offset_grid(engine, golden_basic):
    g = golden_basic["len_off_grid"]
    buf = hexa(g["buf_hex"])
    for off in range(16):
        got = [cgck.in_cksum(buf, off, n) for n in g["lens"]]
        assert got == g["in_cksum"][off], f"offset {off}"


def test_dropin_udp_frames(engine, golden_basic):
    for f in golden_basic["udp_frames"]:
        fr = hexa(f["frame_hex"])
        assert cgck.udp_cksum(fr, 14, f["l4len"]) == f["udp_cksum"]
        assert cgck.tcp_cksum(fr, 14, f["l4len"]) == f["udp_cksum"]


# ---------------------------------------------------------------------------
# Batched, device-resident synthetic sets against the fixtures
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("name", ["64", "1500"])
def test_synth_strided_fixture(engine, golden_synth, name):
    s = golden_synth["sets"][name]
    n, stride, ln = len(s["expect"]), s["stride"], s["ip_len"]
    buf = cgck.DeviceBuffer(n * stride)
    out = cgck.DeviceBuffer(4 * n)
    engine.synth_strided(buf.ptr, n, stride, ln, golden_synth["seed"])
    engine.strided(buf.ptr, n, stride, 0, ln, cgck.GEN_BOTH, out.ptr)
    host = np.zeros(len(s["raw_hex"]) * stride, np.uint8)
    o = np.zeros(n, np.uint32)
    buf.download(host, stream=engine.stream)
    out.download(o, stream=engine.stream)
    engine.sync()
    for k, h in enumerate(s["raw_hex"]):
        assert host[k * stride:k * stride + ln].tobytes().hex() == h, f"device bytes, packet {k}"
    exp = np.array(s["expect"], np.uint32)
    assert np.array_equal(o & 0xFFFF, exp[:, 0])
    assert np.array_equal(o >> 16, exp[:, 1])


def test_synth_imix_fixture(engine, golden_synth):
    s = golden_synth["sets"]["imix"]
    n = len(s["expect"])
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    engine.synth_imix(buf.ptr, desc.ptr, n, golden_synth["seed"])
    engine.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    d = np.zeros(n, cgck.DESC_DTYPE)
    o = np.zeros(n, np.uint32)
    host = np.zeros(nbytes, np.uint8)
    desc.download(d, stream=engine.stream)
    out.download(o, stream=engine.stream)
    buf.download(host, stream=engine.stream)
    engine.sync()
    assert [[int(a), int(b)] for a, b in zip(d["frame_off"], d["ip_len"])] == s["desc"]
    assert not d["l3_off"].any()
    for k, h in enumerate(s["raw_hex"]):
        off, ln = s["desc"][k]
        assert host[off:off + ln].tobytes().hex() == h
    exp = np.array(s["expect"], np.uint32)
    assert np.array_equal(o & 0xFFFF, exp[:, 0])
    assert np.array_equal(o >> 16, exp[:, 1])


# ---------------------------------------------------------------------------
# Randomised differential tests against the oracle referee, every flag set
# and every kernel shape (G = 4 / 16 / 64 lanes per packet)
# ---------------------------------------------------------------------------

FLAG_SETS = [
    cgck.RAW,
    cgck.IP,
    cgck.L4,
    cgck.GEN_BOTH,
    cgck.L4 | cgck.L4_NOPSEUDO,
    cgck.GEN_BOTH | cgck.ZERO_FIELDS,
    cgck.FILL_BOTH,
    cgck.IP | cgck.ZERO_FIELDS | cgck.STORE,
    cgck.VERIFY_BSD,
    cgck.VERIFY_TOY,
    cgck.IP | cgck.L4 | cgck.L4_NOPSEUDO | cgck.VERIFY,
    cgck.VERIFY_BSD | cgck.STORE,
]


def random_batch(rng, n, max_len, odd=True):
    """Packets at random (also odd) offsets of one host buffer, random ihl,
    protocols and lengths, some checksum fields 0 / 0xFFFF / correct."""
    lens = rng.integers(0, max_len + 1, n)
    lens[rng.random(n) < 0.05] = 0
    gaps = rng.integers(0, 40, n)
    if not odd:
        gaps &= ~1
        lens &= ~1
    offs = np.zeros(n, np.int64)
    at = 32
    for i in range(n):
        offs[i] = at
        at += int(lens[i]) + int(gaps[i]) + 64
    buf = rng.integers(0, 256, at + 128, dtype=np.uint8)
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        r = rng.random()
        ihl = 5 if r < 0.7 else int(rng.integers(0, 16))
        buf[o] = 0x40 | ihl
        buf[o + 9] = rng.choice([6, 6, 17, 1, int(rng.integers(0, 256))])
        if rng.random() < 0.2:
            buf[o + 10:o + 12] = 0
        if rng.random() < 0.1:
            buf[o + 10:o + 12] = 0xFF
        if ln >= 2:
            buf[o + 2], buf[o + 3] = (ln >> 8) & 0xFF, ln & 0xFF
    desc = np.zeros(n, cgck.DESC_DTYPE)
    l3 = rng.integers(0, 20, n)
    desc["frame_off"] = offs - l3
    desc["l3_off"] = l3
    desc["ip_len"] = lens
    return buf, desc


@pytest.mark.parametrize("hint", [64, 256, 1500, 4000])
@pytest.mark.parametrize("flags", FLAG_SETS)
def test_fuzz_desc_vs_oracle(engine, port, flags, hint):
    rng = np.random.default_rng(flags * 131 + hint)
    max_len = {64: 80, 256: 300, 1500: 1600, 4000: 5000}[hint]
    n = 700
    buf, desc = random_batch(rng, n, max_len)
    ref_buf = buf.copy()
    exp, ever = port.batch_desc(ref_buf, desc.view(np.uint8), n, flags)
    engine.set_desc_len_hint(hint)
    got_buf = buf.copy()
    out, ver = engine.run_host_desc(got_buf, desc, flags)
    engine.set_desc_len_hint(1500)
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches, first {bad[:5]}: got {out[bad[:5]]} "
                           f"{ver[bad[:5]]} want {exp[bad[:5]]} {ever[bad[:5]]} "
                           f"len {desc['ip_len'][bad[:5]]}")
    assert np.array_equal(got_buf, ref_buf), "STORE bytes differ"


STRIDED = [  # (stride, l3_off, ip_len) — covers every launch shape and alignment
    (64, 0, 64), (64, 0, 60), (72, 14, 54), (61, 3, 58), (80, 0, 80),
    (128, 14, 100), (256, 0, 255), (300, 1, 256),
    (1500, 0, 1500), (1514, 14, 1500), (2048, 14, 1500), (1501, 0, 1501), (1600, 7, 1590),
    (2048, 14, 2000), (9000, 0, 9000), (4000, 1, 3999),
]


@pytest.mark.parametrize("stride,l3,ln", STRIDED)
@pytest.mark.parametrize("flags", [cgck.GEN_BOTH, cgck.RAW, cgck.FILL_BOTH, cgck.VERIFY_BSD])
def test_fuzz_strided_vs_oracle(engine, port, stride, l3, ln, flags):
    rng = np.random.default_rng(stride * 7 + ln)
    n = 333
    buf = rng.integers(0, 256, n * stride + l3 + ln + 64, dtype=np.uint8)
    for k in range(n):
        o = k * stride + l3
        buf[o] = 0x45 if k % 5 else (0x40 | int(rng.integers(5, 16)))
        buf[o + 9] = (6, 17, 1, 6, 99)[k % 5]
    ref = buf.copy()
    exp, ever = port.batch_strided(ref, n, stride, l3, ln, flags)
    got = buf.copy()
    out, ver = engine.run_host_strided(got, n, stride, l3, ln, flags)
    assert np.array_equal(out, exp)
    assert np.array_equal(ver, ever)
    assert np.array_equal(got, ref)


# Every kernel family forced through $CGCK_KERNEL (read at context creation),
# on the strided shapes each one accepts; a family falls back to the group
# kernel where its preconditions fail, so every cell is a valid comparison.
FAMILIES = ["group", "lpp", "lpa", "lpd", "slot2", "lpw", "dstr"]   # every family libcgck.so dispatches to
FAMILY_SHAPES = [  # (stride, l3_off, ip_len, packets); odd counts: every ip_hl = 5
    (64, 0, 64, 3000), (64, 0, 64, 4097), (64, 16, 64, 999), (64, 0, 48, 333), (32, 0, 20, 333), (128, 16, 64, 333), (72, 2, 60, 333),
    (256, 0, 255, 333), (1500, 0, 1500, 3000), (1504, 4, 1500, 333), (1520, 0, 1517, 333),
    (1500, 0, 1000, 333), (1500, 14, 1486, 333),
]


@pytest.fixture(scope="module")
def family_engines():
    engines = {f: cgck.Engine(0, kernel=f) for f in FAMILIES}
    yield engines
    for e in engines.values():
        e.close()


@pytest.mark.parametrize("family", FAMILIES)
@pytest.mark.parametrize("stride,l3,ln,n", FAMILY_SHAPES)
@pytest.mark.parametrize("flags", [cgck.GEN_BOTH, cgck.RAW, cgck.IP, cgck.L4 | cgck.L4_NOPSEUDO,
                                   cgck.VERIFY_TOY])
def test_family_strided_vs_oracle(family_engines, port, family, stride, l3, ln, n, flags):
    rng = np.random.default_rng(stride * 13 + ln + n)
    buf = rng.integers(0, 256, n * stride + l3 + ln + 64, dtype=np.uint8)
    for k in range(n):
        o = k * stride + l3
        buf[o] = 0x45 if (k % 7 or n % 2) else (0x40 | int(rng.integers(5, 16)))
        buf[o + 9] = (6, 17, 1, 6, 99, 6, 6)[k % 7]
    ref = buf.copy()
    exp, ever = port.batch_strided(ref, n, stride, l3, ln, flags)
    got = buf.copy()
    # lpd takes batches without a verdict array (it falls back to lpa with one):
    # its cells compare the outputs, and the kernel it ran
    e = family_engines[family]
    out, ver = e.run_host_strided(got, n, stride, l3, ln, flags, want_verdict=family != "lpd")
    bad = np.nonzero((out != exp) | ((ver if ver is not None else ever) != ever))[0]
    assert len(bad) == 0, f"{family}: {len(bad)} mismatches, first {bad[:5]}"
    assert np.array_equal(got, ref)
    if family == "lpd" and stride <= 64 and (stride | l3) % 16 == 0 and 20 <= ln <= 64:
        assert e.last_kernel.startswith("lpd_kernel<"), e.last_kernel
    if family == "dstr" and stride <= 1520 and (stride | l3) % 4 == 0 and not flags & cgck.VERIFY:
        assert e.last_kernel.startswith("dstr_kernel<"), e.last_kernel


def test_edges(engine, port):
    # empty batch
    engine.strided(0, 0, 64, 0, 64, cgck.GEN_BOTH)
    engine.sync()
    # zero-length and maximal regions in one descriptor batch
    buf = np.random.default_rng(9).integers(0, 256, 70000, dtype=np.uint8)
    buf[16] = 0x45
    desc = np.zeros(4, cgck.DESC_DTYPE)
    desc[0] = (0, 16, 0)
    desc[1] = (0, 16, 65535)
    desc[2] = (1, 16, 19)    # too short for a header: BAD_LEN
    desc[3] = (3, 0, 40000)
    for flags in (cgck.RAW, cgck.GEN_BOTH, cgck.VERIFY_TOY):
        exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), 4, flags)
        out, ver = engine.run_host_desc(buf.copy(), desc, flags)
        assert np.array_equal(out, exp) and np.array_equal(ver, ever), flags
    assert cgck.in_cksum(buf, 0, 0) == 0xFFFF


def test_bad_counters(engine, port, golden_verify):
    cases = golden_verify["cases"]
    buf, desc = pack_cases(cases)
    d = cgck.DeviceBuffer(buf.nbytes)
    dd = cgck.DeviceBuffer(desc.nbytes)
    bad = cgck.DeviceBuffer(8)
    d.upload(buf, stream=engine.stream)
    dd.upload(desc, stream=engine.stream)
    cgck.load().cgck_memset(bad.ptr, 0, 8, engine.stream)
    ver = cgck.DeviceBuffer(len(cases))
    engine.desc(d.ptr, dd.ptr, len(cases), cgck.VERIFY_BSD, None, ver.ptr, bad.ptr)
    b = np.zeros(2, np.uint32)
    v = np.zeros(len(cases), np.uint8)
    bad.download(b, stream=engine.stream)
    ver.download(v, stream=engine.stream)
    engine.sync()
    assert b[0] == sum(1 - c["bsd_ip"] for c in cases)
    assert b[1] == sum(1 - c["bsd_l4"] for c in cases)
    assert b[0] == int(((v & 1) != 0).sum()) and b[1] == int(((v & 2) != 0).sum())


def pack_cases(cases, align=1):
    parts, descs, at = [], [], 0
    for c in cases:
        p = hexa(c["hex"])
        pad = (-at) % align + 3
        parts.append(np.zeros(pad, np.uint8))
        at += pad
        parts.append(p)
        descs.append((at, 0, len(p)))
        at += len(p)
    parts.append(np.zeros(64, np.uint8))
    desc = np.zeros(len(descs), cgck.DESC_DTYPE)
    for i, d in enumerate(descs):
        desc[i] = d
    return np.concatenate(parts), desc


@pytest.mark.parametrize("align", [1, 2, 16])
def test_verify_fixture_verdicts(engine, golden_verify, align):
    """RX verify modes reproduce the reference call sites' verdicts:
    bsd44 ip_input.c:45-58 + tcp_input.c:75-85 / udp_usrreq.c:86-94 and
    gbtcp/inet.c:319-330 + 142-153."""
    cases = golden_verify["cases"]
    buf, desc = pack_cases(cases, align)
    out, ver = engine.run_host_desc(buf.copy(), desc, cgck.VERIFY_BSD)
    for c, v in zip(cases, ver):
        assert (v & 1) == 1 - c["bsd_ip"], c["kind"]
        assert ((v >> 1) & 1) == 1 - c["bsd_l4"], c["kind"]
    tcp = [c for c in cases if c["proto"] == 6]
    buf, desc = pack_cases(tcp, align)
    out, ver = engine.run_host_desc(buf.copy(), desc, cgck.VERIFY_TOY)
    for c, v in zip(tcp, ver):
        assert (v & 1) == 1 - c["toy_ip"] and ((v >> 1) & 1) == 1 - c["toy_l4"], c["kind"]


def burst_slices(n, max_pkts, per=64, max_wg=32):
    """The server's split of an n-packet request (burst_wgs, cgck_internal.h):
    W workgroups, packet i in slice j = the j with n*j//W <= i < n*(j+1)//W."""
    K = 1 if max_pkts <= 64 else min((max_pkts + per - 1) // per, max_wg)
    W = 1 if n <= 64 else min((n + per - 1) // per, K)
    return W, [n * j // W for j in range(W + 1)]


def check_burst(out, exp, ver, ever, got, ref, what, max_pkts, ring=None, desc=None, vm=None):
    """Bit-exact outputs, verdicts and bytes; on a mismatch the message names
    the packets, their server slices, the ring's address and size, and the
    frames' offsets, so a failure on a box nobody can log into still says
    where it went wrong."""
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    bad_bytes = np.nonzero(got != ref)[0]
    if len(bad) == 0 and len(bad_bytes) == 0:
        return
    W, edges = burst_slices(len(out), max_pkts)
    slices = sorted({int(np.searchsorted(edges, int(i), side="right")) - 1 for i in bad})
    msg = [f"{what}: {len(bad)} packets wrong, {len(bad_bytes)} bytes wrong; W {W}"]
    if len(bad):
        msg.append(f"indices {bad[:8].tolist()}..{bad[-8:].tolist()} slices {slices[:16]} "
                   f"got {out[bad[:4]].tolist()} want {exp[bad[:4]].tolist()} "
                   f"verdict got {ver[bad[:4]].tolist()} want {ever[bad[:4]].tolist()}")
        if desc is not None:
            fo = desc["frame_off"].astype(np.int64) + desc["l3_off"]
            msg.append(f"frame offsets {fo[bad[:4]].tolist()} lens {desc['ip_len'][bad[:4]].tolist()}")
    if len(bad_bytes):
        msg.append(f"byte offsets {bad_bytes[:8].tolist()}..{bad_bytes[-4:].tolist()} "
                   f"got {got[bad_bytes[:8]].tolist()} want {ref[bad_bytes[:8]].tolist()} "
                   f"4 KiB pages {sorted(set((bad_bytes // 4096).tolist()))[:16]}")
    if ring is not None:
        msg.append(f"ring {ring.ctypes.data:#x} + {ring.nbytes}")
        msg.append(f"mappings {memdiag.vma_info(ring.ctypes.data, ring.nbytes)}")
    if vm is not None:
        msg.append(f"vmstat over the request {memdiag.vmstat_delta(vm, memdiag.vmstat())}")
    path = memdiag.dump_failure(what, out=out, exp=exp, ver=ver, ever=ever, got=got, ref=ref,
                                desc=desc if desc is not None else np.zeros(0, cgck.DESC_DTYPE),
                                ring_addr=np.uint64(ring.ctypes.data if ring is not None else 0))
    msg.append(f"arrays in {path}")
    raise AssertionError("; ".join(msg))


def page_ring(nbytes):
    """A ring of nbytes (rounded up to pages) in an anonymous mapping of its
    own, as a transport's pool is (cgck_host_register refuses the brk heap):
    (owner, view)."""
    import mmap
    size = (nbytes + 4095) // 4096 * 4096
    m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    return m, np.frombuffer(m, np.uint8)


@pytest.mark.parametrize("npk,registered", [(500, False), (3000, False), (500, True), (3000, True)])
def test_host_resident_batch(engine, port, npk, registered):
    """cgck_desc_host's three ways in: a small pageable burst (pinned staging,
    500 packets), a large pageable batch (DMA, 3000 packets > 512 KiB), and
    ring memory registered with cgck_host_register (read where it lies)."""
    rng = np.random.default_rng(21 + npk)
    buf, desc = random_batch(rng, npk, 1500)
    L = cgck.load()
    if registered:
        raw, ring = page_ring(len(buf))
        assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    try:
        for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD):
            ref = buf.copy()
            exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
            if registered:
                ring[:len(buf)] = buf
                got = ring[:len(buf)]
            else:
                got = buf.copy()
            out = np.zeros(len(desc), np.uint32)
            ver = np.zeros(len(desc), np.uint8)
            engine.desc_host(got, desc, flags, out, ver)
            check_burst(out, exp, ver, ever, got, ref, f"npk {npk} flags {flags}", 1,
                        ring if registered else None, desc)
    finally:
        if registered:
            L.cgck_host_unregister(ring.ctypes.data)


@pytest.mark.parametrize("registered", [False, True])
def test_burst_server_desc_host(engine, port, registered):
    """cgck_desc_host through the resident burst server (cgck_burst_open): the
    same bytes, results and verdicts as the referee, staged or in place; a
    batch larger than the server's capacity takes the launch path."""
    L = cgck.load()
    engine.burst_open(max_pkts=1024, max_bytes=1 << 20)
    try:
        for npk in (1, 37, 700, 1500):          # 1500 packets: over max_pkts, launch path
            rng = np.random.default_rng(31 + npk)
            buf, desc = random_batch(rng, npk, 1500)
            if registered:
                raw, ring = page_ring(len(buf))
                assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
            try:
                for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD, cgck.VERIFY_TOY):
                    ref = buf.copy()
                    exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
                    if registered:
                        ring[:len(buf)] = buf
                        got = ring[:len(buf)]
                    else:
                        got = buf.copy()
                    out = np.zeros(len(desc), np.uint32)
                    ver = np.zeros(len(desc), np.uint8)
                    engine.desc_host(got, desc, flags, out, ver)
                    check_burst(out, exp, ver, ever, got, ref, f"npk {npk} flags {flags}", 1024,
                                ring if registered else None, desc)
            finally:
                if registered:
                    L.cgck_host_unregister(ring.ctypes.data)
    finally:
        engine.burst_close()


@pytest.mark.parametrize("max_len", [80, 600])
@pytest.mark.parametrize("registered", [False, True])
def test_burst_server_wide(engine, port, registered, max_len):
    """Requests split over the server's workgroups (burst_wgs: one up to 64
    packets, then one per 64, up to 32): slice edges at 64 / 65 / 130 / 2047 /
    2048 / 4096 packets, staged or in place, generate / fill / verify,
    against the referee; a second server of 2 workgroups (max_pkts 128)
    takes uneven slices of 65 / 127 / 128 packets."""
    L = cgck.load()
    for max_pkts, sizes in ((4096, (64, 65, 130, 2047, 2048, 4096)), (128, (65, 127, 128))):
        engine.burst_open(max_pkts=max_pkts, max_bytes=4 << 20)
        try:
            for npk in sizes:
                rng = np.random.default_rng(77 + npk + max_len)
                buf, desc = random_batch(rng, npk, max_len)
                ring = None
                if registered:
                    raw, ring = page_ring(len(buf))
                    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
                try:
                    for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD):
                        ref = buf.copy()
                        exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
                        if registered:
                            ring[:len(buf)] = buf
                            got = ring[:len(buf)]
                        else:
                            got = buf.copy()
                        out = np.zeros(len(desc), np.uint32)
                        ver = np.zeros(len(desc), np.uint8)
                        vm = memdiag.vmstat()
                        engine.desc_host(got, desc, flags, out, ver)
                        check_burst(out, exp, ver, ever, got, ref, f"max_pkts {max_pkts} npk {npk} flags {flags}",
                                    max_pkts, ring, desc, vm)
                finally:
                    if registered:
                        L.cgck_host_unregister(ring.ctypes.data)
        finally:
            engine.burst_close()


def test_burst_server_reregister_cycles(engine, port):
    """register ring A, serve, unregister and unmap it,
    register a larger ring B and FILL through a 32-workgroup server, checking
    every packet, byte and verdict; sixteen cycles, two frame sizes.  (Round
    3's test carved its rings out of the brk heap, where the allocator
    returns and re-faults pages under a registration: the GPU then read and
    wrote some pages 64 or 128 KiB off; cgck_host_register refuses the heap,
    test_host_register_refuses_brk_heap.)"""
    L = cgck.load()
    engine.burst_open(max_pkts=4096, max_bytes=4 << 20)
    try:
        for cycle in range(16):
            max_len = 600 if cycle % 2 else 80
            for npk in (2048, 4096):
                rng = np.random.default_rng(900 + 17 * cycle + npk)
                buf, desc = random_batch(rng, npk, max_len)
                raw, ring = page_ring(len(buf))
                assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
                try:
                    for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD):
                        ref = buf.copy()
                        exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
                        ring[:len(buf)] = buf
                        got = ring[:len(buf)]
                        out = np.zeros(npk, np.uint32)
                        ver = np.zeros(npk, np.uint8)
                        vm = memdiag.vmstat()
                        engine.desc_host(got, desc, flags, out, ver)
                        check_burst(out, exp, ver, ever, got, ref, f"cycle {cycle} npk {npk} flags {flags}",
                                    4096, ring, desc, vm)
                finally:
                    assert L.cgck_host_unregister(ring.ctypes.data) == 0
                del ring, got, raw
    finally:
        engine.burst_close()


def test_host_register_refuses_brk_heap(engine):
    """A buffer of the brk heap ([heap] in /proc/self/maps) is refused with
    -EINVAL; the same bytes in a mapping of their own register."""
    L = cgck.load()
    small = [np.zeros(16384, np.uint8) for _ in range(8)]   # small arrays come from the heap
    heap = [a for a in small if memdiag.in_brk_heap(a.ctypes.data, a.nbytes)]
    if not heap:
        pytest.skip("no numpy buffer landed in the brk heap in this process")
    assert L.cgck_host_register(heap[0].ctypes.data, heap[0].nbytes) == -22
    assert "brk heap" in cgck.last_error()
    raw, ring = page_ring(16384)
    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    assert L.cgck_host_unregister(ring.ctypes.data) == 0


@pytest.mark.parametrize("npk", [40, 700])
def test_burst_request_range_refused(engine, port, npk):
    """cgck_burst_request: the server itself checks every descriptor against
    the request's range (registered memory read in place) — one frame past
    the range fails the request with -EIO, nothing read out of range, nothing
    stored; the same batch inside the range is exact (one workgroup at 40
    packets, eleven slices at 700)."""
    L = cgck.load()
    rng = np.random.default_rng(4242 + npk)
    buf, desc = random_batch(rng, npk, 600)
    raw, ring = page_ring(len(buf))
    ring[:len(buf)] = buf
    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    engine.burst_open(max_pkts=1024, max_bytes=4 << 20)
    try:
        dev = cgck.host_device_ptr(ring)
        ends = desc["frame_off"].astype(np.int64) + desc["l3_off"] + desc["ip_len"]
        rng_bytes = int(ends.max())
        out = np.zeros(npk, np.uint32)
        ver = np.zeros(npk, np.uint8)
        # the exact range: served
        assert engine.burst_request(dev, rng_bytes, desc, cgck.FILL_BOTH, out, ver) == 0
        ref = buf.copy()
        exp, ever = port.batch_desc(ref, desc.view(np.uint8), npk, cgck.FILL_BOTH)
        check_burst(out, exp, ver, ever, ring[:len(buf)], ref, "in range", 1024, ring, desc)
        # one byte short of the farthest frame: refused on the device
        ring[:len(buf)] = buf
        assert engine.burst_request(dev, rng_bytes - 1, desc, cgck.FILL_BOTH, out, ver) == -5   # -EIO
        assert "refused" in cgck.last_error()
        # a frame offset far past the range (it would fault if it were read)
        bad = desc.copy()
        bad["frame_off"][npk // 2] = 1 << 40
        assert engine.burst_request(dev, ring.nbytes, bad, cgck.FILL_BOTH, out, ver) == -5
        # the refused requests stored nothing (the slices that checked first
        # may have served: only a wholly refused slice is untouched, so
        # compare only the frames of a one-workgroup request)
        if npk <= 64:
            assert np.array_equal(ring[:len(buf)], buf)
        # and the server still serves
        ring[:len(buf)] = buf
        assert engine.burst_request(dev, ring.nbytes, desc, cgck.GEN_BOTH, out, ver) == 0
        exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), npk, cgck.GEN_BOTH)
        check_burst(out, exp, ver, ever, ring[:len(buf)], buf, "after refusal", 1024, ring, desc)
    finally:
        engine.burst_close()
        assert L.cgck_host_unregister(ring.ctypes.data) == 0


def test_burst_server_idle_relaunch(engine, port):
    """The server exits after idle_ms without a request and the next request
    relaunches it; close is idempotent."""
    import time
    engine.burst_open(max_pkts=256, max_bytes=1 << 20, idle_ms=20)
    try:
        for rep in range(4):
            rng = np.random.default_rng(41 + rep)
            buf, desc = random_batch(rng, 64 if rep % 2 == 0 else 256, 1500)   # one / four workgroups
            exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), len(desc), cgck.VERIFY_BSD)
            out, ver = np.zeros(len(desc), np.uint32), np.zeros(len(desc), np.uint8)
            engine.desc_host(buf.copy(), desc, cgck.VERIFY_BSD, out, ver)
            assert np.array_equal(out, exp) and np.array_equal(ver, ever), rep
            time.sleep(0.1)                      # > idle_ms: the server has exited
    finally:
        engine.burst_close()
    engine.burst_close()


def test_burst_server_dropin_and_tx(port):
    """The drop-in symbols and the deferred TX window on this thread's context
    with its burst server open (cgck_burst_open(NULL, ...))."""
    cgck.burst_open(max_pkts=512, max_bytes=1 << 20)
    try:
        rng = np.random.default_rng(5)
        for n in (0, 1, 19, 20, 21, 64, 1479, 1480, 1500):
            for off in (0, 1, 7):
                buf = rng.integers(0, 256, off + n + 64, dtype=np.uint8)
                assert cgck.in_cksum(buf, off, n) == port.in_cksum(buf, off, n), (n, off)
        for ln in (20, 40, 64, 576, 1500):
            pkt = rng.integers(0, 256, ln + 16, dtype=np.uint8)
            pkt[0] = 0x45
            pkt[9] = 6
            assert cgck.udp_cksum(pkt, 0, ln - 20) == port.udp_cksum(pkt, 0, ln - 20), ln
        ring = np.zeros((64, 2048), np.uint8)
        want = []
        for i in range(64):
            ln = int(rng.integers(40, 1501))
            pkt = rng.integers(0, 256, ln, dtype=np.uint8)
            pkt[0] = 0x45
            pkt[9] = 6
            pkt[36:38] = 0
            pkt[10:12] = 0
            ring[i, 14:14 + ln] = pkt
            ref = pkt.copy()
            ref[36:38] = np.frombuffer(np.uint16(port.udp_cksum(ref, 0, ln - 20)).tobytes(), np.uint8)
            ref[10:12] = np.frombuffer(np.uint16(port.in_cksum(ref, 0, 20)).tobytes(), np.uint8)
            want.append((ln, ref))
        cgck.tx_begin()
        for i, (ln, ref) in enumerate(want):
            row = ring[i]
            v = cgck.udp_cksum(row, 14, ln - 20)
            row[14 + 36:14 + 38] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
            v = cgck.ip_cksum(row, 14)
            row[14 + 10:14 + 12] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
        # the ring is not registered: every call was answered synchronously
        # (through the server) and nothing is left for the flush
        assert cgck.tx_flush() == 0
        for i, (ln, ref) in enumerate(want):
            assert np.array_equal(ring[i, 14:14 + ln], ref), i
    finally:
        cgck.burst_close()


def test_host_resident_desc_past_buffer(engine):
    """A descriptor that reaches past the given bytes is refused (-EINVAL),
    not read."""
    buf = np.zeros(4096, np.uint8)
    desc = np.zeros(2, cgck.DESC_DTYPE)
    desc[0] = (0, 0, 1500)
    desc[1] = (3000, 14, 1500)
    with pytest.raises(cgck.CgckError):
        engine.desc_host(buf, desc, cgck.GEN_BOTH, np.zeros(2, np.uint32), np.zeros(2, np.uint8))


@pytest.mark.parametrize("registered", [False, True])
def test_deferred_tx_fill(engine, port, registered):
    """Deferred TX window: the stack's own call pattern (tcp_output.c:416-418
    then ip_output.c:61-64, each storing the return value) inside
    cgck_tx_begin/flush yields the same bytes as the synchronous reference
    sequence — queued and read in place from a registered ring, or answered
    synchronously when the memory is not registered."""
    rng = np.random.default_rng(23)
    raw, flat = page_ring(256 * 2048)
    ring = flat.reshape(256, 2048)   # netmap-like slots, IP at +14
    if registered:
        assert cgck.load().cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    want = []
    for i in range(256):
        ln = int(rng.integers(40, 523))       # MTU 522 (con-gen.c:741)
        pkt = rng.integers(0, 256, ln, dtype=np.uint8)
        pkt[0] = 0x45
        pkt[9] = 6 if i % 3 else 17
        ring[i, 14:14 + ln] = pkt
        ref = pkt.copy()
        hl = 20
        fo = 16 if pkt[9] == 6 else 6
        ref[hl + fo:hl + fo + 2] = 0
        ref[hl + fo:hl + fo + 2] = np.frombuffer(
            np.uint16(port.udp_cksum(ref, 0, ln - hl)).tobytes(), np.uint8)
        ref[10:12] = 0
        ref[10:12] = np.frombuffer(np.uint16(port.in_cksum(ref, 0, hl)).tobytes(), np.uint8)
        want.append((ln, ref, fo))
    cgck.tx_begin()
    for i, (ln, ref, fo) in enumerate(want):
        row = ring[i]
        row[14 + 20 + fo:14 + 20 + fo + 2] = 0                 # tcp_template zeroes th_sum
        v = cgck.udp_cksum(row, 14, ln - 20)                   # th->th_sum = tcp_cksum(...)
        row[14 + 20 + fo:14 + 20 + fo + 2] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
        row[14 + 10:14 + 12] = 0                                # ip->ip_sum = 0
        v = cgck.ip_cksum(row, 14)                              # ip->ip_sum = ip_cksum(ip)
        row[14 + 10:14 + 12] = np.frombuffer(np.uint16(v).tobytes(), np.uint8)
    try:
        assert cgck.tx_flush() == (2 * len(want) if registered else 0)
    finally:
        if registered:
            cgck.load().cgck_host_unregister(ring.ctypes.data)
    for i, (ln, ref, fo) in enumerate(want):
        assert np.array_equal(ring[i, 14:14 + ln], ref), i


# ---------------------------------------------------------------------------
# Full BASELINE.json sizes: 100 % at 16M x 64 B, 1/64 sample at 16M x 1500 B
# and IMIX, plus size-independent round trips (fill -> verify -> corrupt).
# ---------------------------------------------------------------------------

@pytest.mark.slow
@pytest.mark.parametrize("stride,every", [(64, 1), (1500, 64)])
def test_full_size_strided(engine, port, stride, every):
    n = 16 << 20
    buf = cgck.DeviceBuffer(n * stride)
    out = cgck.DeviceBuffer(4 * n)
    engine.synth_strided(buf.ptr, n, stride, stride, SEED)
    engine.strided(buf.ptr, n, stride, 0, stride, cgck.GEN_BOTH, out.ptr)
    o = np.zeros(n, np.uint32)
    out.download(o, stream=engine.stream)
    engine.sync()
    bad, chk = port.check_synth_strided(n, stride, stride, SEED, cgck.GEN_BOTH, o, every)
    assert bad == 0 and chk == (n + every - 1) // every
    # round trip: fill both fields in place, then every packet verifies clean
    ver = cgck.DeviceBuffer(n)
    badc = cgck.DeviceBuffer(8)
    cgck.load().cgck_memset(badc.ptr, 0, 8, engine.stream)
    engine.strided(buf.ptr, n, stride, 0, stride, cgck.FILL_BOTH, None)
    engine.strided(buf.ptr, n, stride, 0, stride, cgck.VERIFY_BSD, out.ptr, ver.ptr, badc.ptr)
    o2 = np.zeros(n, np.uint32)
    b = np.zeros(2, np.uint32)
    out.download(o2, stream=engine.stream)
    badc.download(b, stream=engine.stream)
    engine.sync()
    assert np.array_equal(o2, o), "verify recomputation differs from generation"
    assert b.tolist() == [0, 0]
    # corrupt one payload byte in 1000 random packets: exactly those fail L4
    rng = np.random.default_rng(31)
    ks = np.unique(rng.integers(0, n, 1000))
    one = np.array([0x5A], np.uint8)
    for k in ks:
        pos = int(k) * stride + int(rng.integers(40, stride))
        cur = np.zeros(1, np.uint8)
        cgck.load().cgck_memcpy(cur.ctypes.data, buf.ptr + pos, 1, engine.stream)
        engine.sync()
        cur ^= one
        cgck.load().cgck_memcpy(buf.ptr + pos, cur.ctypes.data, 1, engine.stream)
    cgck.load().cgck_memset(badc.ptr, 0, 8, engine.stream)
    engine.strided(buf.ptr, n, stride, 0, stride, cgck.VERIFY_BSD, None, ver.ptr, badc.ptr)
    v = np.zeros(n, np.uint8)
    ver.download(v, stream=engine.stream)
    badc.download(b, stream=engine.stream)
    engine.sync()
    assert b.tolist() == [0, len(ks)]
    assert np.array_equal(np.nonzero(v)[0], ks)


@pytest.mark.slow
def test_full_size_imix(engine, port):
    n = 16 << 20
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    engine.synth_imix(buf.ptr, desc.ptr, n, SEED)
    engine.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    o = np.zeros(n, np.uint32)
    out.download(o, stream=engine.stream)
    engine.sync()
    bad, chk = port.check_synth_imix(n, SEED, cgck.GEN_BOTH, o, 64)
    assert bad == 0 and chk == n // 64


# ---------------------------------------------------------------------------
# Shared-nothing worker threads (con-gen.c:1092-1100): every thread calls the
# drop-in symbols on its own context at the same time; results stay exact.
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("server", [False, True])
def test_dropin_concurrent_threads(engine, golden_basic, server):
    """Eight threads on their own drop-in contexts; with `server`, each keeps
    its own resident burst server (eight polling workgroups at once)."""
    import threading
    g = golden_basic["len_off_grid"]
    buf = hexa(g["buf_hex"])
    frames = golden_basic["udp_frames"][:32]
    errors = []

    def worker(tid):
        try:
            if server:
                cgck.burst_open(max_pkts=64, max_bytes=1 << 16)
            for rep in range(3):
                off = (tid + rep) % 16
                got = [cgck.in_cksum(buf, off, n) for n in g["lens"][::7]]
                if got != g["in_cksum"][off][::7]:
                    errors.append(f"thread {tid}: in_cksum at offset {off}")
                for f in frames:
                    fr = hexa(f["frame_hex"])
                    if cgck.udp_cksum(fr, 14, f["l4len"]) != f["udp_cksum"]:
                        errors.append(f"thread {tid}: udp_cksum")
                        break
        finally:
            cgck.thread_release()

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors[:5]


def thp_ring(nbytes):
    """A ring in an anonymous mapping advised MADV_HUGEPAGE, 2 MiB aligned
    and never written yet: (owner, view).  The pages come in on the first
    write after cgck_host_register — the trigger DESIGN.md §0 named for the
    round-3/4 wrong-address reads."""
    import mmap
    al = 2 << 20
    size = (nbytes + al - 1) // al * al
    m = mmap.mmap(-1, size + al, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    whole = np.frombuffer(m, np.uint8)
    start = (-whole.ctypes.data) % al
    m.madvise(mmap.MADV_HUGEPAGE, start, size)
    return m, whole[start:start + size]


@pytest.mark.parametrize("cycle", range(3))
def test_thp_ring_first_touch_after_register(engine, port, cycle):
    """a ring advised MADV_HUGEPAGE, registered before
    any of its pages exist, then written for the first time; GEN, FILL and
    VERIFY through a 32-workgroup server (4096 packets, every index, byte
    and verdict checked), then once more after the frames are rewritten in
    place.  The smaps entry (AnonHugePages) and the THP counters of the
    request go into the failure message."""
    L = cgck.load()
    rng = np.random.default_rng(7700 + cycle)
    npk = 4096
    buf, desc = random_batch(rng, npk, 600 if cycle % 2 else 1500)
    raw, ring = thp_ring(len(buf))
    vm0 = memdiag.vmstat()
    assert L.cgck_host_register(ring.ctypes.data, ring.nbytes) == 0
    engine.burst_open(max_pkts=4096, max_bytes=8 << 20)
    try:
        for rep in range(2):
            for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD):
                ref = buf.copy()
                exp, ever = port.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
                ring[:len(buf)] = buf                         # rep 0: the first touch of every page
                got = ring[:len(buf)]
                out = np.zeros(npk, np.uint32)
                ver = np.zeros(npk, np.uint8)
                vm = memdiag.vmstat()
                engine.desc_host(got, desc, flags, out, ver)
                check_burst(out, exp, ver, ever, got, ref,
                            f"THP cycle {cycle} rep {rep} flags {flags} {memdiag.vma_info(ring.ctypes.data, 4096)} "
                            f"thp since register {memdiag.vmstat_delta(vm0, memdiag.vmstat())}",
                            4096, ring, desc, vm)
    finally:
        engine.burst_close()
        assert L.cgck_host_unregister(ring.ctypes.data) == 0
