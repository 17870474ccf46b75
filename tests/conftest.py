import os
import subprocess
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = os.path.join(REPO, "loona_amd", "libhpk.so")
    orc = os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "loona_amd", "csrc")])


_ensure_built()
