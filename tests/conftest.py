import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


import pytest  # noqa: E402


@pytest.fixture(scope="session")
def cpusim_engine():
    """The engine's host build (libkp_cpusim.so): engine.cpp + the kernel bodies on the CPU."""
    from karmada_amd.engine import PKG, Engine
    e = Engine(0, lib_path=os.path.join(PKG, "libkp_cpusim.so"))
    yield e
    e.close()


@pytest.fixture(scope="session")
def gpu_engine():
    """libkp.so on HIP device 0 (tests marked gpu only)."""
    from karmada_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()
