"""The seq-wrap test (tests/test_gpu_burst_seq.py, which the product gate
runs against libcgck.so) against libcgck_lab.so, so tools/gpu_r6.sh can run
it with CGCK_SERVER_OPTS=512 (every workgroup but the leader starts its slice
20 us late): its control — the same run with the done-word refresh switched
off (opts 528) — then fails deterministically instead of by timing."""
import os

import pytest

import cgck
from test_gpu_burst_seq import wrap_body

pytestmark = [pytest.mark.gpu, pytest.mark.lab]


@pytest.fixture(scope="module")
def lab():
    if not os.path.exists(cgck.LAB_PATH):
        pytest.skip("libcgck_lab.so not built (make -C tools lab)")
    saved = cgck.load()
    cgck._lib = cgck.bind(cgck.LAB_PATH)
    try:
        if cgck.device_count() < 1:
            pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
        e = cgck.Engine(0)
        yield e
        e.close()
    finally:
        cgck._lib = saved


@pytest.mark.parametrize("start", [0xFFFFFFF0, 0x7FFFFFF8, 1000])
def test_seq_wrap_and_stale_done_words(lab, port, start):
    wrap_body(lab, port, start)
