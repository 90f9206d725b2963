import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracing-with-zig_amd")
for p in (PKG, ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


def _ensure_built():
    """Build the oracle and the product library if their .so files are missing (CPU-only step)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(PKG, "librtzig.so")):
        subprocess.run(["make", "-j8", "-C", os.path.join(PKG, "csrc")], check=True,
                       stdout=subprocess.DEVNULL)


_ensure_built()


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib.Oracle()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
