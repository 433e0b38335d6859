"""Shared pytest setup: the `gpu` marker, import paths, and lazy fixtures."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "smith-waterman-fpga-module_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    return O


@pytest.fixture(scope="session")
def swbank():
    import swbank as S
    return S


@pytest.fixture
def poisoned_buffers(monkeypatch):
    """SWBANK_POISON=1: every device buffer a bank allocates starts as 0x3C bytes (f16 1.0)
    instead of whatever the allocator hands back (often zeros in a fresh process, stale data
    late in a long session), so a kernel that reads a word nobody wrote fails every time."""
    monkeypatch.setenv("SWBANK_POISON", "1")
