"""The output paths added late in round 2, at sizes where every wave of the
grid walks more than one chunk (so staged outputs of one chunk are flushed
while the next chunk is in flight), against the oracle referee
(oracle/cksum_oracle.c, pinned to the reference's subr.c:119-223):

- dstr_kernel (cgck_dense.hip, the 1500 B default): a writer wave finishes
  and stores each chunk's frames from sums the DMA wave staged; frames of any
  length 20..1520 at 4-byte alignment, BAD_LEN verdicts, partial last chunks,
  RAW / IP / L4 / L4_NOPSEUDO; an unaligned output array takes the group
  kernel instead (exact as well).
- lpw_kernel (packed IMIX): a full chunk's outputs leave as one 16-byte
  store per lane issued after the next DMA round; batches without verdicts
  take that path, with verdicts (or an unaligned output array) the
  end-of-chunk flush."""

import numpy as np
import pytest

import cgck

pytestmark = pytest.mark.gpu


def strided_frames(rng, n, stride, l3, ln, bad_len=False):
    """n records of `stride` bytes, an IPv4 header at +l3 with ip_hl 5 mostly
    (6..15 in some, more than ip_len allows when bad_len)."""
    buf = rng.integers(0, 256, n * stride + l3 + ln + 64, dtype=np.uint8)
    at = np.arange(n, dtype=np.int64) * stride + l3
    hl = np.where(rng.random(n) < 0.8, 5, rng.integers(5, 16, n))
    if bad_len:
        hl[::7] = 15   # 60-byte header in a shorter datagram: BAD_LEN
    buf[at] = (0x40 | hl).astype(np.uint8)
    buf[at + 9] = rng.choice(np.array([6, 17, 1, 6], np.uint8), n)
    return buf


def run_device_strided(engine, buf, n, stride, l3, ln, flags, verdict=False, out_shift=0):
    d = cgck.DeviceBuffer(buf.nbytes)
    o = cgck.DeviceBuffer(4 * n + 16)
    v = cgck.DeviceBuffer(n) if verdict else None
    d.upload(buf, stream=engine.stream)
    engine.strided(d.ptr, n, stride, l3, ln, flags, o.ptr + out_shift, v.ptr if v else None)
    kern = engine.last_kernel
    out = np.zeros(n, np.uint32)
    o.download(out, off=out_shift, stream=engine.stream)
    ver = None
    if v:
        ver = np.zeros(n, np.uint8)
        v.download(ver, stream=engine.stream)
    engine.sync()
    for b in (d, o, v):
        if b:
            b.free()
    return out, ver, kern


@pytest.fixture(scope="module")
def dstr_engine():
    """An engine pinned to the dstr family (cgck_ctx_set_kernel)."""
    e = cgck.Engine(0, kernel="dstr")
    yield e
    e.close()


# (stride, l3_off, ip_len, frames): > 64 x 2048 frames, so each wave of the
# grid takes two or three chunks; counts leave a partial last chunk
DENSE_SHAPES = [(100, 0, 100, 200003), (64, 4, 21, 300001), (1024, 12, 1000, 140003), (32, 8, 24, 262147)]


@pytest.mark.parametrize("stride,l3,ln,n", DENSE_SHAPES)
@pytest.mark.parametrize("flags", [cgck.GEN_BOTH, cgck.RAW, cgck.L4 | cgck.L4_NOPSEUDO])
def test_dstr_multichunk(dstr_engine, port, stride, l3, ln, n, flags):
    rng = np.random.default_rng(stride + l3 + ln + n + flags)
    buf = strided_frames(rng, n, stride, l3, ln, bad_len=ln < 60)
    exp, ever = port.batch_strided(buf.copy(), n, stride, l3, ln, flags)
    out, ver, kern = run_device_strided(dstr_engine, buf, n, stride, l3, ln, flags, verdict=True)
    assert kern.startswith("dstr_kernel<"), kern
    bad = np.nonzero((out != exp) | (ver != ever))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}"
    if ln < 60 and not flags & cgck.RAW:
        assert np.count_nonzero(ever & cgck.BAD_LEN) > 0   # the BAD_LEN frames were there


def test_dstr_default_1500_multichunk(engine, port):
    """The dispatcher's own choice for dense >= 1 KiB frames, multi-chunk,
    with and without verdicts, and with an output array that is not 16-byte
    aligned (the group kernel then; exact either way)."""
    n, stride, ln = 140001, 1500, 1500
    rng = np.random.default_rng(1500)
    buf = strided_frames(rng, n, stride, 0, ln)
    exp, ever = port.batch_strided(buf.copy(), n, stride, 0, ln, cgck.GEN_BOTH)
    for verdict, shift, want in ((False, 0, "dstr_kernel<"), (True, 0, "dstr_kernel<"),
                                 (False, 4, "cksum_kernel<")):
        out, ver, kern = run_device_strided(engine, buf, n, stride, 0, ln, cgck.GEN_BOTH, verdict, shift)
        assert kern.startswith(want), (verdict, shift, kern)
        assert np.array_equal(out, exp), (verdict, shift, int(np.count_nonzero(out != exp)))
        if verdict:
            assert np.array_equal(ver, ever)


def packed_imix(rng, n):
    """IMIX frames (64/576/1500 at 7:4:1) back to back, vectorised."""
    L = rng.choice(np.array([64] * 7 + [576] * 4 + [1500]), n)
    offs = np.concatenate(([0], np.cumsum(L[:-1]))).astype(np.int64)
    buf = rng.integers(0, 256, int(offs[-1] + L[-1]) + 256, dtype=np.uint8)
    hl = np.where(rng.random(n) < 0.9, 5, rng.integers(5, 16, n))
    buf[offs] = (0x40 | hl).astype(np.uint8)
    buf[offs + 9] = rng.choice(np.array([6, 17, 1, 6], np.uint8), n)
    buf[offs + 2] = (L >> 8).astype(np.uint8)
    buf[offs + 3] = (L & 0xFF).astype(np.uint8)
    desc = np.zeros(n, cgck.DESC_DTYPE)
    desc["frame_off"] = offs
    desc["ip_len"] = L
    return buf, desc


@pytest.mark.parametrize("verdict,shift", [(False, 0), (True, 0), (False, 4)])
def test_lpw_deferred_flush_multichunk(engine, port, verdict, shift):
    """Packed IMIX through the dispatcher under the layout hint, > 256 x 2048
    frames (two chunks per wave for many waves, a partial last chunk)."""
    n = 600011
    rng = np.random.default_rng(7 + verdict + shift)
    buf, desc = packed_imix(rng, n)
    exp, ever = port.batch_desc(buf.copy(), desc.view(np.uint8), n, cgck.GEN_BOTH)
    d = cgck.DeviceBuffer(buf.nbytes)
    dd = cgck.DeviceBuffer(desc.nbytes)
    o = cgck.DeviceBuffer(4 * n + 16)
    v = cgck.DeviceBuffer(n) if verdict else None
    d.upload(buf, stream=engine.stream)
    dd.upload(desc, stream=engine.stream)
    engine.set_desc_len_hint(int(buf.nbytes // n))
    engine.set_desc_layout(cgck.LAYOUT_PACKED)
    try:
        engine.desc(d.ptr, dd.ptr, n, cgck.GEN_BOTH, o.ptr + shift, v.ptr if v else None)
        kern = engine.last_kernel
    finally:
        engine.set_desc_layout(cgck.LAYOUT_ANY)
        engine.set_desc_len_hint(1500)
    out = np.zeros(n, np.uint32)
    o.download(out, off=shift, stream=engine.stream)
    ver = np.zeros(n, np.uint8)
    if v:
        v.download(ver, stream=engine.stream)
    engine.sync()
    for b in (d, dd, o, v):
        if b:
            b.free()
    assert kern.startswith("lpw_kernel<"), kern
    bad = np.nonzero(out != exp)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}"
    if verdict:
        assert np.array_equal(ver, ever)
