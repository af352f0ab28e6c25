"""pytest configuration.

Markers: ``gpu`` — needs an MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on the CPU-only build container.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mojo-bm25_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built_libs():
    """Build the in-tree libraries once (no-op when up to date)."""
    from bm25mi.build import build
    build()
    from oracle import oracle
    oracle.build()
    yield


def gpu_available() -> bool:
    try:
        from bm25mi import _capi
        return _capi.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("no HIP device visible: -m gpu tests must run on the GPU box")
    return 0
