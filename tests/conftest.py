import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "reed-solomon-16_amd"
for p in (str(PKG_DIR), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU case (large reference vectors)")


def expand(ranges):
    """[[a, b], ...] index ranges (half-open) -> list of ints."""
    out = []
    for a, b in ranges:
        out.extend(range(a, b))
    return out
