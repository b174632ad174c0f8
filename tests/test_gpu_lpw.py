"""The packed-buffer streaming kernel (lpw_kernel, cgck_lane.hip): descriptor
batches of mixed lengths under cgck_set_desc_layout(CGCK_LAYOUT_PACKED).
Bit-exact against the oracle referee (oracle/cksum_oracle.c) on packed
batches of every length class and alignment, on batches that are NOT packed
(gapped, reversed, overlapping: its frame-by-frame steps must stay exact
whatever the hint says), through the dispatcher's own choice, and on the
full-size IMIX batch (BASELINE configs[3]) packed and in 2048 B ring slots,
against the slot2 kernel's results."""
import numpy as np
import pytest

import cgck
from test_gpu_parity import FLAG_SETS, random_batch
from batches import MIXES, packed_batch

pytestmark = pytest.mark.gpu
LPW = ("lpw_kernel<", "lpx_kernel<")   # lpx: the lab build's two-rounds-in-flight form ($CGCK_LPW_X)


@pytest.fixture(scope="module")
def lpw():
    """An engine pinned to the lpw family (cgck_ctx_set_kernel)."""
    e = cgck.Engine(0, kernel="lpw")
    e.set_desc_layout(cgck.LAYOUT_PACKED)
    yield e
    e.close()


def run(engine, port, buf, desc, flags):
    exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), len(desc), flags)
    got = buf.copy()
    out, ver = engine.run_host_desc(got, desc, flags)
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    assert len(bad) == 0, (f"{len(bad)} mismatches, first {bad[:5]}: got {out[bad[:5]]} want {exp[bad[:5]]} "
                           f"len {desc['ip_len'][bad[:5]]}")
    return got, engine.last_kernel


@pytest.mark.parametrize("mix", sorted(MIXES))
@pytest.mark.parametrize("flags", [f for f in FLAG_SETS if not f & cgck.STORE])
def test_packed_batches(lpw, port, mix, flags):
    rng = np.random.default_rng(hash(mix) % 1000 + flags + 7)
    n = 40 if mix == "jumbo" else 3000
    buf, desc = packed_batch(rng, n, MIXES[mix], first_off=int(rng.integers(0, 16)))
    got, kernel = run(lpw, port, buf, desc, flags)
    assert kernel.startswith(LPW)
    assert np.array_equal(got, buf)


@pytest.mark.parametrize("flags", [cgck.FILL_BOTH, cgck.VERIFY_BSD | cgck.STORE])
def test_store_takes_other_family(lpw, port, flags):
    """In-place stores are not lpw's (it reads the bytes it would rewrite
    through LDS copies): those batches go to the group kernel, exact."""
    rng = np.random.default_rng(15 + flags)
    buf, desc = packed_batch(rng, 2000, MIXES["imix"])
    exp_buf = buf.copy()
    exp, ever = port.batch_desc(exp_buf, desc.view(np.uint8), len(desc), flags)
    got = buf.copy()
    out, ver = lpw.run_host_desc(got, desc, flags)
    assert not lpw.last_kernel.startswith("lpw_kernel")
    assert np.array_equal(out, exp) and np.array_equal(ver, ever) and np.array_equal(got, exp_buf)


@pytest.mark.parametrize("max_len", [80, 600, 1600])
def test_unpacked_batches(lpw, port, max_len):
    """Gapped, odd-offset batches and a 2048-byte-slot ring under the packed
    hint: every step is computed frame by frame, exact."""
    rng = np.random.default_rng(max_len + 3)
    buf, desc = random_batch(rng, 1500, max_len)
    for flags in (cgck.GEN_BOTH, cgck.VERIFY_BSD, cgck.RAW):
        run(lpw, port, buf, desc, flags)
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
        run(lpw, port, ring, rd, flags)


@pytest.mark.parametrize("total", [0, 511, 512, 513, 1024, 8191, 8192, 8193, 12000])
def test_gathered_window_edges(lpw, port, total):
    """Scattered steps (frames in slots, not back to back) whose chunk-run
    list totals `total` chunks: exactly one / two windows, one over, the
    16-window limit and past it (computed frame by frame from global memory);
    frames at odd offsets, empty frames among them, then a whole empty step,
    then the same step again: the owner table's marks, carries and row edges."""
    rng = np.random.default_rng(total + 11)
    n = 64
    # split `total` chunks over 64 frames (some empty), each frame in its own slot
    cuts = np.sort(rng.integers(0, total + 1, n - 1)) if total else np.zeros(n - 1, np.int64)
    nch = np.diff(np.concatenate([[0], cuts, [total]]))
    q = rng.integers(0, 16, n)
    lens = np.where(nch > 0, np.maximum(16 * nch - q - rng.integers(0, 16, n), 1), 0)
    lens = np.where((nch > 0) & (lens <= 16 * (nch - 1) - q), 16 * (nch - 1) - q + 1, lens)
    lens = np.minimum(lens, 65535)
    slot = int(max(16 * nch.max() + 64, 128)) if total else 128
    frames = np.concatenate([np.arange(n), np.arange(n)])          # two steps of the same frames
    buf = rng.integers(0, 256, 3 * n * slot + 64, dtype=np.uint8)
    desc = np.zeros(3 * n, cgck.DESC_DTYPE)
    for i in range(3 * n):
        k = i % n
        if n <= i < 2 * n:                      # the middle step: empty frames
            desc[i] = (2 * n * slot, 0, 0)
            continue
        base = (k + (n if i >= 2 * n else 0)) * slot
        o = base + int(q[k])
        if lens[k]:
            buf[o] = 0x45
            buf[o + 9] = 6 if lens[k] > 9 else buf[o + 9]
        desc[i] = (base, int(q[k]), int(lens[k]))
    del frames
    for flags in (cgck.GEN_BOTH, cgck.RAW):
        _, k = run(lpw, port, buf, desc, flags)
        assert k.startswith(LPW), k


def test_reversed_overlapping_and_mixed_steps(lpw, port):
    """Descriptors walking a packed buffer backwards, pairs over the same
    bytes, and packed and unpacked 64-frame steps interleaved in one batch."""
    rng = np.random.default_rng(78)
    buf, desc = packed_batch(rng, 2000, MIXES["imix"])
    run(lpw, port, buf, desc[::-1].copy(), cgck.GEN_BOTH)
    run(lpw, port, buf, np.repeat(desc, 2), cgck.VERIFY_BSD)
    mixed = desc.copy()
    for s in range(0, len(mixed) - 64, 192):   # every third step reversed
        mixed[s:s + 64] = mixed[s:s + 64][::-1]
    run(lpw, port, buf, mixed, cgck.GEN_BOTH)


def test_dispatcher_picks_lpw_for_mid_lengths(engine, port):
    """The default dispatch: typical length 256 B .. 1 KiB -> lpw with or
    without CGCK_LAYOUT_PACKED (the kernel tells packed steps from scattered
    ones itself), on a packed batch and on the same frames scattered; below
    256 B -> slot2; all exact."""
    rng = np.random.default_rng(91)
    buf, desc = packed_batch(rng, 5000, MIXES["imix"])
    sbuf, sdesc = random_batch(rng, 5000, 700)
    engine.set_desc_len_hint(354)
    try:
        for layout in (cgck.LAYOUT_PACKED, cgck.LAYOUT_ANY):
            engine.set_desc_layout(layout)
            _, k = run(engine, port, buf, desc, cgck.GEN_BOTH)
            assert k.startswith(LPW), (layout, k)
            _, k = run(engine, port, sbuf, sdesc, cgck.VERIFY_BSD)
            assert k.startswith(LPW), (layout, k)
        engine.set_desc_len_hint(200)
        _, k = run(engine, port, sbuf, sdesc, cgck.GEN_BOTH)
        assert k.startswith("slot2_kernel<"), k
    finally:
        engine.set_desc_layout(cgck.LAYOUT_ANY)
        engine.set_desc_len_hint(1500)
    with pytest.raises(cgck.CgckError, match="unknown layout"):
        engine.set_desc_layout(2)


@pytest.mark.slow
def test_full_size_imix(lpw, port):
    """BASELINE configs[3] (16M IMIX packets, packed by cgck_synth_imix)
    through lpw: every 64th packet against the referee, and the whole batch
    against the slot2 kernel's results."""
    n = 16 << 20
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    ref = cgck.DeviceBuffer(4 * n)
    lpw.synth_imix(buf.ptr, desc.ptr, n, 0xC0C1)
    e = cgck.Engine(0, kernel="slot2")   # the register-gather path as the second opinion
    e.set_desc_len_hint(nbytes // n)
    e.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, ref.ptr)
    assert e.last_kernel.startswith("slot2_kernel<")
    e.sync()
    e.close()
    lpw.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
    assert lpw.last_kernel.startswith(LPW)
    o = np.zeros(n, np.uint32)
    r = np.zeros(n, np.uint32)
    out.download(o, stream=lpw.stream)
    ref.download(r, stream=lpw.stream)
    lpw.sync()
    for b in (buf, desc, out, ref):
        b.free()
    bad, chk = port.check_synth_imix(n, 0xC0C1, cgck.GEN_BOTH, o, 64)
    assert bad == 0 and chk == n // 64
    assert np.array_equal(o, r)


@pytest.mark.parametrize("stride,ln,want", [(576, 576, LPW), (300, 300, LPW),
                                            (1024, 576, LPW), (2048, 300, LPW),
                                            (160, 160, "slot2_kernel<"), (1500, 1500, "cksum_kernel<")])
def test_dispatcher_strided(engine, port, stride, ln, want):
    """Strided batches from 256 B to 1 KiB stream through lpw, back to back
    (stride <= length: the span) or gapped (ring slots: the frames' chunk runs
    gathered); smaller ones gather in registers (slot2), 1 KiB and up stream
    through LDS four frames a step (dstr), or take the group kernel when they
    verify; all exact."""
    n = 3001
    rng = np.random.default_rng(stride + ln)
    buf = rng.integers(0, 256, n * stride + ln + 64, dtype=np.uint8)
    for k in range(n):
        buf[k * stride] = 0x45 if k % 5 else 0x46
        buf[k * stride + 9] = (6, 17, 1)[k % 3]
    for flags in (cgck.GEN_BOTH, cgck.VERIFY_BSD, cgck.RAW):
        exp, ever = port.batch_strided(buf.copy(), n, stride, 0, ln, flags)
        out, ver = engine.run_host_strided(buf.copy(), n, stride, 0, ln, flags)
        assert np.array_equal(out, exp) and np.array_equal(ver, ever), (stride, ln, flags)
        k = engine.last_kernel
        if want == "cksum_kernel<" and not flags & cgck.VERIFY:   # dense 1500 B: dstr
            assert k.startswith("dstr_kernel<"), k
        else:
            assert k.startswith(want), k


@pytest.mark.slow
def test_full_size_imix_ring(port):
    """The 16M IMIX frames in 2048 B ring slots at +14 (the netmap layout)
    through the default dispatch (lpw, gathered steps): every 64th frame
    against the referee, the whole batch against slot2."""
    n = 16 << 20
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(2048 * n)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    ref = cgck.DeviceBuffer(4 * n)
    e = cgck.Engine(0)
    s2 = cgck.Engine(0, kernel="slot2")
    try:
        e.synth_imix_ring(buf.ptr, desc.ptr, n, 2048, 14, 0xC0C2)
        for x in (e, s2):
            x.set_desc_len_hint(nbytes // n)
        e.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)
        assert e.last_kernel.startswith(LPW), e.last_kernel
        e.sync()
        s2.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, ref.ptr)
        assert s2.last_kernel.startswith("slot2_kernel<")
        o = np.zeros(n, np.uint32)
        r = np.zeros(n, np.uint32)
        out.download(o, stream=s2.stream)
        ref.download(r, stream=s2.stream)
        s2.sync()
    finally:
        for b in (buf, desc, out, ref):
            b.free()
        e.close()
        s2.close()
    bad, chk = port.check_synth_ring(n, 2048, 14, 0xC0C2, cgck.GEN_BOTH, o, 64)
    assert bad == 0 and chk == n // 64
    assert np.array_equal(o, r)
