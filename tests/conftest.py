import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); parity tests through the C-ABI")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (test infrastructure) and the product library if needed."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "memcached_amd", "libmcrc32c.so")):
        from memcached_amd import build
        build.build_lib()
