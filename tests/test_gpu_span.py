"""Packed-span kernel (cgck_span.hip, an A/B family of libcgck_lab.so, forced
as variant 12 by $CGCK_KERNEL=span): bit-exact against the oracle referee
(oracle/cksum_oracle.c) on packed batches of every length class and
alignment, on batches that are NOT packed (its gap / lane-per-packet
fallbacks must stay exact whatever the layout), and on the full-size IMIX
batch (BASELINE configs[3]).  The module runs against the lab build: it swaps
the binding for its own duration."""
import os

import numpy as np
import pytest

import cgck
from test_gpu_parity import FLAG_SETS, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not os.path.exists(cgck.LAB_PATH):
        pytest.skip("libcgck_lab.so not built (make -C tools lab)")
    saved = cgck.load()
    cgck._lib = cgck.bind(cgck.LAB_PATH)
    try:
        if cgck.device_count() < 1:
            pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
        os.environ["CGCK_KERNEL"] = "span"
        try:
            e = cgck.Engine(0)
        finally:
            os.environ.pop("CGCK_KERNEL", None)
        yield e
        e.close()
    finally:
        cgck._lib = saved

MIXES = {
    "imix": [64] * 7 + [576] * 4 + [1500],
    "small": list(range(0, 90)),                 # includes 0..19 (BAD_LEN) and odd lengths
    "mtu": [1500, 1499, 1514, 1480],             # 64 of them overflow one 64 KiB tile span
    "jumbo": [9000, 20000, 64, 65535, 40],       # tiles of one or two packets, the 64 KiB edge
    "wide": list(range(20, 1601, 7)),
}


def packed_batch(rng, n, lens, first_off=0):
    """Frames back to back in descriptor order: frame k+1's IPv4 header starts
    where frame k's ip_len bytes end (random l3_off inside each frame)."""
    L = rng.choice(np.asarray(lens), n)
    at = first_off
    offs = np.zeros(n, np.int64)
    for i in range(n):
        offs[i] = at
        at += int(L[i])
    buf = rng.integers(0, 256, at + 256, dtype=np.uint8)
    for i in range(n):
        o, ln = int(offs[i]), int(L[i])
        if ln < 1:
            continue
        r = rng.random()
        buf[o] = 0x40 | (5 if r < 0.7 else int(rng.integers(0, 16)))
        if ln > 9:
            buf[o + 9] = rng.choice([6, 6, 17, 1, int(rng.integers(0, 256))])
        if ln > 11 and rng.random() < 0.2:
            buf[o + 10:o + 12] = 0
        if ln >= 4:
            buf[o + 2], buf[o + 3] = (ln >> 8) & 0xFF, ln & 0xFF
    desc = np.zeros(n, cgck.DESC_DTYPE)
    l3 = np.minimum(rng.integers(0, 20, n), offs)
    desc["frame_off"] = offs - l3
    desc["l3_off"] = l3
    desc["ip_len"] = L
    return buf, desc


def run_packed(engine, port, buf, desc, flags):
    exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), len(desc), flags)
    got = buf.copy()
    out, ver = engine.run_host_desc(got, desc, flags)
    kernel = engine.last_kernel
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches, first {bad[:5]}: got {out[bad[:5]]} want {exp[bad[:5]]} "
                           f"len {desc['ip_len'][bad[:5]]}")
    return got, kernel


@pytest.mark.parametrize("mix", sorted(MIXES))
@pytest.mark.parametrize("flags", [f for f in FLAG_SETS if not f & cgck.STORE])
def test_packed_batches(engine, port, mix, flags):
    rng = np.random.default_rng(hash(mix) % 1000 + flags)
    n = 40 if mix == "jumbo" else 3000
    buf, desc = packed_batch(rng, n, MIXES[mix], first_off=int(rng.integers(0, 16)))
    got, kernel = run_packed(engine, port, buf, desc, flags)
    assert kernel.startswith("span_kernel<")
    assert np.array_equal(got, buf)


@pytest.mark.parametrize("flags", [cgck.FILL_BOTH, cgck.VERIFY_BSD | cgck.STORE])
def test_packed_hint_with_store_uses_other_family(engine, port, flags):
    """STORE batches do not take the span kernel (in-place field stores would
    race with neighbours' span reads) and stay exact."""
    rng = np.random.default_rng(5 + flags)
    buf, desc = packed_batch(rng, 2000, MIXES["imix"])
    exp_buf = buf.copy()
    exp, ever = port.batch_desc(exp_buf, desc.view(np.uint8), len(desc), flags)
    got = buf.copy()
    out, ver = engine.run_host_desc(got, desc, flags)
    assert not engine.last_kernel.startswith("span_kernel")
    assert np.array_equal(out, exp) and np.array_equal(ver, ever) and np.array_equal(got, exp_buf)


@pytest.mark.parametrize("max_len", [80, 600, 1600])
def test_packed_hint_on_unpacked_batches(engine, port, max_len):
    """Gapped, odd-offset batches (random_batch) and a 2048-byte-slot ring
    under the packed hint: the span's gap handling and the lane-per-packet
    tiles must be exact too."""
    rng = np.random.default_rng(max_len)
    buf, desc = random_batch(rng, 1500, max_len)
    for flags in (cgck.GEN_BOTH, cgck.VERIFY_BSD, cgck.RAW):
        run_packed(engine, port, buf, desc, flags)
    n = 700
    ring = rng.integers(0, 256, n * 2048 + 64, dtype=np.uint8)
    rd = np.zeros(n, cgck.DESC_DTYPE)
    rd["frame_off"] = np.arange(n) * 2048
    rd["l3_off"] = 14
    rd["ip_len"] = rng.integers(20, max_len + 1, n)
    for k in range(n):
        ring[k * 2048 + 14] = 0x45
        ring[k * 2048 + 14 + 9] = 6
    for flags in (cgck.GEN_BOTH, cgck.VERIFY_TOY):
        run_packed(engine, port, ring, rd, flags)


def test_packed_reversed_and_overlapping(engine, port):
    """Order and overlap cost efficiency only: descriptors walking a packed
    buffer backwards, and pairs of descriptors over the same bytes."""
    rng = np.random.default_rng(77)
    buf, desc = packed_batch(rng, 2000, MIXES["imix"])
    run_packed(engine, port, buf, desc[::-1].copy(), cgck.GEN_BOTH)
    dup = np.repeat(desc, 2)
    run_packed(engine, port, buf, dup, cgck.VERIFY_BSD)


@pytest.mark.slow
def test_full_size_imix_packed(engine, port):
    """BASELINE configs[3] (16M IMIX packets, packed by cgck_synth_imix)
    through the span kernel: every 64th packet against the referee, plus the
    same batch through the default (slot2) path compared in full."""
    n = 16 << 20
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    ref = cgck.DeviceBuffer(4 * n)
    engine.synth_imix(buf.ptr, desc.ptr, n, 0xC0C0)
    engine.set_desc_len_hint(nbytes // n)
    ref_engine = cgck.Engine(0)   # the default (slot2) path
    ref_engine.set_desc_len_hint(nbytes // n)
    ref_engine.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, ref.ptr)
    ref_engine.sync()
    ref_engine.close()
    engine.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    assert engine.last_kernel.startswith("span_kernel<")
    engine.set_desc_len_hint(1500)
    o = np.zeros(n, np.uint32)
    r = np.zeros(n, np.uint32)
    out.download(o, stream=engine.stream)
    ref.download(r, stream=engine.stream)
    engine.sync()
    for b in (buf, desc, out, ref):
        b.free()
    bad, chk = port.check_synth_imix(n, 0xC0C0, cgck.GEN_BOTH, o, 64)
    assert bad == 0 and chk == n // 64
    assert np.array_equal(o, r)
