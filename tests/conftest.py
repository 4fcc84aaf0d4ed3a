import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs through libbsm_hip.so)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def golden():
    from golden import golden_io

    return golden_io.load()


@pytest.fixture(scope="session")
def golden_c5():
    """The band oracle's C5 solve (scripts/make_c5_fixture.py)."""
    import json

    with open(os.path.join(HERE, "golden", "c5_poisson_1000.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    from oracle import pyoracle

    pyoracle.lib()
    return pyoracle
