"""Shared test setup.

Markers:
  gpu  -- needs an MI355X (run with `-m gpu` on the GPU box).  Everything else
          runs on the CPU-only build container.
"""
import os
import sys

import pytest

# torch bundles its own libamdhip64.so; the engine library links the system
# one under the same soname.  Whichever loads first serves both, and torch
# only initializes with its own: load torch before anything loads the engine
# (bench.py imports torch first for the same reason).
try:
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-rate-limiter_amd")
for p in (ROOT, os.path.join(PKG, "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (gfx950)")


@pytest.fixture(scope="session")
def rl():
    """The HIP engine binding (raises if the library is not built)."""
    import rl_amd
    return rl_amd


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle
