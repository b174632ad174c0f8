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
