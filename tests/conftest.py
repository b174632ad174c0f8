import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "con-gen_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) parity runs")
    config.addinivalue_line("markers", "lab: needs libcgck_lab.so (make -C tools lab); runs only when "
                                       "the -m expression names it")


def pytest_collection_modifyitems(config, items):
    """Lab-build tests (A/B-only kernel families) stay out of the product
    runs (`-m gpu`, `-m "not gpu"`) unless the marker expression asks."""
    if "lab" in (config.getoption("markexpr") or ""):
        return
    skip = pytest.mark.skip(reason="lab build only: run with -m \"gpu and lab\"")
    for it in items:
        if "lab" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_basic():
    return load_golden("basic.json")


@pytest.fixture(scope="session")
def golden_synth():
    return load_golden("synth.json")


@pytest.fixture(scope="session")
def golden_verify():
    return load_golden("verify.json")


@pytest.fixture(scope="session")
def port():
    import oracle
    return oracle.port()


@pytest.fixture(scope="session")
def engine():
    import cgck
    if cgck.device_count() < 1:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    e = cgck.Engine(0)
    yield e
    e.close()
