import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from oracle import jdoracle
    jdoracle.build()
    return jdoracle


@pytest.fixture(scope="session")
def built_lib():
    """Build the engine library (cross-compiles for gfx950, no GPU needed)."""
    lib = os.path.join(ROOT, "jdeflate_amd", "lib", "libjdeflate_amd.so")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "jdeflate_amd", "csrc")],
                   check=True)
    return lib


@pytest.fixture(scope="session")
def engine(built_lib):
    import jdeflate_amd as J
    if not J.available():
        pytest.fail("gpu test without a usable gfx950 engine (no silent fallback)")
    return J
