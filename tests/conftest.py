import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library on the device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    """The CPU oracle (test infrastructure): built from oracle/ on first use."""
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def cube():
    from eray_amd.objfile import load_obj_file
    return load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))


@pytest.fixture(scope="session")
def gpu():
    """One eray context on GPU 0 for the whole GPU session (fails loudly without a GPU)."""
    from eray_amd import capi
    ctx = capi.Context(0)
    yield ctx
    ctx.close()
