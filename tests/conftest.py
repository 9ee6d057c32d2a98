import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "raft-simulation_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libraftsim.so)")
    config.addinivalue_line("markers", "slow: long CPU-side cases")


@pytest.fixture(scope="session", autouse=True)
def _oracle_built():
    lib = ROOT / "oracle" / "build" / "libraftref.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    return lib
