"""GPU parity of the Toeplitz RSS row: the gfx950
kernels (cgck_rss.hip, through the C-ABI) against the fixtures made from the
reference's own toeplitz_hash / rss_hash4 (tests/golden/rss.json) and against
the oracle restatement on the same bytes.  Integer work: bit-exact."""
import hashlib
import json
import os

import numpy as np
import pytest

import cgck

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def g():
    with open(os.path.join(GOLDEN, "rss.json")) as f:
        return json.load(f)


def hexa(s):
    return np.frombuffer(bytes.fromhex(s), np.uint8).copy()


def test_dropin_ms_vectors(engine, g):
    key = hexa(g["freebsd_rss_key"])
    for v in g["ms_vectors"]:
        d = hexa(v["data_hex"])
        assert cgck.toeplitz_hash(d, key) == v["ipv4_tcp"]
        assert cgck.toeplitz_hash(d, key, 8) == v["ipv4"]
        assert cgck.rss_hash4(v["laddr"], v["faddr"], v["lport"], v["fport"], key) == v["rss_hash4"]


def test_dropin_grid(engine, g):
    t = g["toeplitz_grid"]
    buf, key = hexa(t["data_hex"]), hexa(t["key_hex"])
    for ks, row in zip(t["key_sizes"], t["hash"]):
        got = [cgck.toeplitz_hash(buf, key, c, ks) for c in t["cnts"]]
        assert got == row, f"key_size {ks}"


def test_dropin_negative_cnt(engine, g):
    key = hexa(g["freebsd_rss_key"])
    assert cgck.toeplitz_hash(np.zeros(4, np.uint8), key, -3) == 0


def run_batch(engine, host, n, stride, cnt, key, mask=0xFFFFFFFF, off=0, key_size=None):
    d = cgck.DeviceBuffer(max(host.nbytes + off, 16))
    o = cgck.DeviceBuffer(4 * max(n, 1))
    d.upload(host, off=off, stream=engine.stream)
    engine.toeplitz(d.ptr + off, n, stride, cnt, key, o.ptr, mask=mask, key_size=key_size)
    out = np.zeros(n, np.uint32)
    o.download(out, stream=engine.stream)
    engine.sync()
    return out


def test_batch_tuples12(engine, g):
    key = hexa(g["freebsd_rss_key"])
    d = hexa(g["tuples12"]["data_hex"])
    out = run_batch(engine, d, 4096, 12, 12, key)
    assert out.tolist() == g["tuples12"]["hash"]
    out7 = run_batch(engine, d, 4096, 12, 12, key, mask=0x7F)
    assert np.array_equal(out7, out & 0x7F)


@pytest.mark.parametrize("n,stride,cnt,off,ks", [
    (1000, 16, 12, 0, 40),      # padded records, dword path
    (777, 36, 36, 0, 52),       # IPv6 4-tuple, dword path
    (513, 13, 13, 0, 40),       # byte path, odd stride
    (300, 12, 12, 1, 40),       # misaligned base: byte path
    (200, 40, 40, 0, 64),       # table past the LDS limit: global-table path
    (50, 128, 100, 0, 16),      # long records, short key (zeros shifted in)
    (64, 12, 12, 0, 2),         # key_size < 4 still reads key[0..3]
    (33, 0, 12, 0, 40),         # stride 0: every record the same bytes
    (100, 8, 0, 0, 40),         # cnt 0: hash 0
])
def test_batch_shapes(engine, port, n, stride, cnt, off, ks):
    rng = np.random.default_rng(n * 7 + cnt)
    host = rng.integers(0, 256, max(n * stride, cnt, 1), dtype=np.uint8)
    key = rng.integers(0, 256, max(ks, 4), dtype=np.uint8)
    out = run_batch(engine, host, n, stride, cnt, key, off=off, key_size=ks)
    exp = port.toeplitz_batch(host, n, stride, cnt, key, key_size=ks)
    assert np.array_equal(out, exp)


@pytest.mark.parametrize("mask", [0xFFFFFFFF, 0x7F])
def test_batch_dense_ring_wrap(engine, port, mask):
    """The default dense-tuple kernel (toeplitz12x4_ab_kernel<12>, one block per
    CU) over more 256-group chunks than its register ring holds per block, a
    partial last chunk and an n % 4 tail handed to the per-record kernel:
    n = 4*256*CUs*13 + 4*37 + 3 with CUs = 256 (MI355X), compared in full."""
    n = 4 * 256 * 256 * 13 + 4 * 37 + 3
    rng = np.random.default_rng(1213)
    host = rng.integers(0, 256, 12 * n, dtype=np.uint8)
    key = rng.integers(0, 256, 40, dtype=np.uint8)
    out = run_batch(engine, host, n, 12, 12, key, mask=mask)
    exp = port.toeplitz_batch(host, n, 12, 12, key, mask=mask)
    assert np.array_equal(out, exp)


def test_batch_empty(engine, g):
    key = hexa(g["freebsd_rss_key"])
    engine.toeplitz(None, 0, 12, 12, key, None)
    engine.sync()


def test_key_switch(engine, g):
    """The context's cached tables follow the key of each call."""
    d = hexa(g["tuples12"]["data_hex"])
    k1 = hexa(g["freebsd_rss_key"])
    k2 = hexa(g["keys"]["random52"])
    a1 = run_batch(engine, d, 4096, 12, 12, k1)
    b = run_batch(engine, d, 4096, 12, 12, k2)
    a2 = run_batch(engine, d, 4096, 12, 12, k1)
    assert np.array_equal(a1, a2) and not np.array_equal(a1, b)
    assert a1.tolist() == g["tuples12"]["hash"]


def params(g, s):
    key = hexa(g["keys"][s["key"]])
    return cgck.Engine.dst_params(s["laddr"], s["faddr"], s["fport"], s["queue_num"],
                                  s["queue_id"], key)


@pytest.mark.parametrize("idx", range(15))
def test_dst_sets(engine, g, idx):
    s = g["dst_sets"][idx]
    e = engine.dst_cache_host(params(g, s), s["cap"])
    assert len(e) == s["count"], s["name"]
    assert hashlib.sha256(e.tobytes()).hexdigest() == s["sha256"], s["name"]
    if len(e):
        assert e[:32].tobytes().hex() == s["head"]
        assert e[-32:].tobytes().hex() == s["tail"]


def test_dst_device_variant_repeat(engine, g, port):
    """Device out/count, asynchronous, run twice on the same scratch (the
    control and look-back words are re-zeroed per launch)."""
    s = g["dst_sets"][5]
    p = params(g, s)
    out = cgck.DeviceBuffer(16 * s["cap"])
    cnt = cgck.DeviceBuffer(4)
    for _ in range(2):
        out_h = np.zeros(s["cap"], cgck.DST_DTYPE)
        c = np.zeros(1, np.uint32)
        engine.dst_cache(p, out.ptr, s["cap"], cnt.ptr)
        cnt.download(c, stream=engine.stream)
        out.download(out_h, stream=engine.stream)
        engine.sync()
        assert int(c[0]) == s["count"]
        assert hashlib.sha256(out_h[:c[0]].tobytes()).hexdigest() == s["sha256"]


def test_dst_random_configs(engine, port):
    """Random small ranges, queue counts and caps against the restated loop."""
    rng = np.random.default_rng(5)
    for _ in range(12):
        l0 = int(rng.integers(0, 1 << 31))
        f0 = int(rng.integers(0, 1 << 31))
        nl, nf = int(rng.integers(1, 3)), int(rng.integers(1, 90))
        qn, qi = int(rng.integers(0, 20)), int(rng.integers(0, 20))
        if rng.integers(0, 4) == 0:
            qi = 128 + int(rng.integers(0, 100))
        cap = int(rng.integers(1, 400000))
        fport = int(rng.integers(0, 1 << 16))
        key = rng.integers(0, 256, 40, dtype=np.uint8)
        exp = port.dst_cache(l0, l0 + nl - 1, f0, f0 + nf - 1, fport, qn, qi, key, cap)
        got = engine.dst_cache_host(cgck.Engine.dst_params((l0, l0 + nl - 1), (f0, f0 + nf - 1),
                                                           fport, qn, qi, key), cap)
        assert np.array_equal(got, exp), (l0, nl, f0, nf, qn, qi, cap)


def test_dst_errors(engine, g):
    s = g["dst_sets"][0]
    with pytest.raises(cgck.CgckError, match="cap"):
        engine.dst_cache_host(params(g, s), 0)
    bad = dict(s, laddr=[s["laddr"][1] + 1, s["laddr"][1]])
    with pytest.raises(cgck.CgckError, match="min > max"):
        engine.dst_cache_host(params(g, bad), 10)


@pytest.mark.slow
def test_batch_full_size_sample(engine, g, port):
    """16M dense 12-byte tuples (the bench shape): device output checked on a
    strided 1/256 sample plus the first 4096 against the restatement."""
    n = 16 << 20
    key = hexa(g["freebsd_rss_key"])
    d = cgck.DeviceBuffer(n * 12)
    o = cgck.DeviceBuffer(4 * n)
    engine.synth_strided(d.ptr, n * 12 // 1500, 1500, 1500, 77)   # random bytes (tail too)
    engine.toeplitz(d.ptr, n, 12, 12, key, o.ptr)
    host = np.zeros(n * 12, np.uint8)
    out = np.zeros(n, np.uint32)
    d.download(host, stream=engine.stream)
    o.download(out, stream=engine.stream)
    engine.sync()
    idx = np.concatenate([np.arange(4096), np.arange(4096, n, 256)])
    sub = np.ascontiguousarray(host.reshape(n, 12)[idx]).reshape(-1)
    exp = port.toeplitz_batch(sub, len(idx), 12, 12, key)
    assert np.array_equal(out[idx], exp)
