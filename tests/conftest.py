import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "crypto3-fil-proofs_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import oracle_py

    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def ctx():
    import fil_groth16

    c = fil_groth16.Context(0)
    yield c
    c.close()


class _Tune:
    """Library A/B switches for one test (fil_groth16.tuning; csrc/tune.h): set(name, value) / clear(name)."""

    def set(self, name, value):
        import fil_groth16

        fil_groth16.tune_set(name, value)

    def clear(self, name):
        import fil_groth16

        fil_groth16.tune_clear(name)


@pytest.fixture
def tune():
    """Switches set through this fixture are all cleared after the test (the library's defaults come back)."""
    import fil_groth16

    yield _Tune()
    fil_groth16.tune_clear()
