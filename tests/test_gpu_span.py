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
from batches import MIXES, packed_batch, run_packed
from test_gpu_parity import FLAG_SETS, random_batch

pytestmark = [pytest.mark.gpu, pytest.mark.lab]


@pytest.fixture(scope="module")
def engine():
    if not os.path.exists(cgck.LAB_PATH):
        pytest.skip("libcgck_lab.so not built (make -C tools lab)")
    saved = cgck.load()
    cgck._lib = cgck.bind(cgck.LAB_PATH)
    try:
        if cgck.device_count() < 1:
            pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
        e = cgck.Engine(0, kernel="span")
        yield e
        e.close()
    finally:
        cgck._lib = saved

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
    same batch through the slot2 kernel compared in full."""
    n = 16 << 20
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    ref = cgck.DeviceBuffer(4 * n)
    engine.synth_imix(buf.ptr, desc.ptr, n, 0xC0C0)
    engine.set_desc_len_hint(nbytes // n)
    ref_engine = cgck.Engine(0, kernel="slot2")   # a second kernel's results
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
