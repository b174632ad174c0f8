"""Shards of the multi-GPU batch split (BASELINE configs[4]) on
one device: two contexts, as two ranks would hold them, generate shards 0 and
1 (seeds 0xC0C0 and 0xC0C1, bench.shard_plan) and checksum them; bench.py's
own checker leg verifies each shard against the oracle, as every rank does in
a scaling run."""
import numpy as np
import pytest

import bench
import cgck

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size", [1500, 64])
def test_two_shards_two_contexts(size):
    n = 1 << 16
    engines = [cgck.Engine(0), cgck.Engine(0)]
    try:
        res = []
        for r, eng in enumerate(engines):
            plan = bench.shard_plan(r, 2, n)
            buf = cgck.DeviceBuffer(n * size)
            out = cgck.DeviceBuffer(4 * n)
            eng.synth_strided(buf.ptr, n, size, size, plan["seed"])
            eng.strided(buf.ptr, n, size, 0, size, cgck.GEN_BOTH, out.ptr)
            o = np.zeros(n, np.uint32)
            out.download(o, stream=eng.stream)
            eng.sync()
            buf.free()
            out.free()
            par = bench.checker_leg({str(size): {"out": o}}, plan, cgck)
            res.append((plan, o, par[str(size)]))
        every = bench.CHECK_EVERY[str(size)]
        for plan, o, (checked, bad) in res:
            assert checked == -(-n // every) and bad == 0, plan
        assert not np.array_equal(res[0][1], res[1][1])    # different shards, different sums
        # a result of shard 1 checked against shard 0's generator must fail
        wrong = bench.checker_leg({str(size): {"out": res[1][1]}}, res[0][0], cgck)
        assert wrong[str(size)][1] > 0
    finally:
        for e in engines:
            e.close()


@pytest.mark.slow
def test_configs4_eight_shards_full_size(golden_synth, port):
    """BASELINE configs[4] at full size, serially on one MI355X: the eight
    16M x 1500 B shards of the 128M-packet batch (bench.shard_plan(r, 8, 16M),
    seeds 0xC0C0..0xC0C7), each generated on the device and checksummed by
    the dispatcher's own kernel (dstr), each checked by the oracle on every
    64th packet of the whole shard (SURVEY §8(d) parity gate), shard 0 also
    against the reference-made fixture (tests/golden/synth.json).  Only the
    cross-device concurrency of an 8-GPU node stays unmeasured here; the
    shards' checked / mismatch counts are printed for the log."""
    n, size = 16 << 20, 1500
    every = bench.CHECK_EVERY["1500"]
    eng = cgck.Engine(0)
    buf = cgck.DeviceBuffer(n * size)
    out = cgck.DeviceBuffer(4 * n)
    o = np.zeros(n, np.uint32)
    fx = golden_synth["sets"]["1500"]
    exp0 = np.array(fx["expect"], np.uint32)
    assert golden_synth["seed"] == bench.SEED
    sums = []
    try:
        for r in range(8):
            plan = bench.shard_plan(r, 8, n)
            assert plan["seed"] == 0xC0C0 + r and plan["first"] == r * n
            eng.synth_strided(buf.ptr, n, size, size, plan["seed"])
            eng.strided(buf.ptr, n, size, 0, size, cgck.GEN_BOTH, out.ptr)
            kernel = eng.last_kernel
            out.download(o, stream=eng.stream)
            eng.sync()
            bad, chk = port.check_synth_strided(n, size, size, plan["seed"], cgck.GEN_BOTH, o, every)
            fixture = ""
            if r == 0:
                m = len(exp0)
                fbad = int(np.count_nonzero((o[:m] & 0xFFFF) != exp0[:, 0]) +
                           np.count_nonzero((o[:m] >> 16) != exp0[:, 1]))
                fixture = f" fixture {m} checked, {fbad} mismatches"
                assert fbad == 0
            print(f"configs[4] shard {r}/8 seed {plan['seed']:#x} packets [{plan['first']}, "
                  f"{plan['first'] + n}) kernel {kernel}: oracle {chk} checked, {bad} mismatches;{fixture}",
                  flush=True)
            assert kernel.startswith("dstr_kernel<"), kernel
            assert bad == 0 and chk == -(-n // every), (r, bad, chk)
            sums.append(int(o[:4096].astype(np.uint64).sum()))
        assert len(set(sums)) == 8                      # eight different shards
    finally:
        buf.free()
        out.free()
        eng.close()
