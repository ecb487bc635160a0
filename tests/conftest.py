import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build libpm.so and the oracle in-tree if they are missing."""
    lib = os.path.join(REPO, "patternmatching_amd", "libpm.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "patternmatching_amd", "csrc")], check=True)
    if not os.path.exists(os.path.join(REPO, "oracle", "_build", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
