"""Shared test setup.

Markers: `gpu` — needs an MI355X (run with `-m gpu` on the GPU box); everything else runs on CPU.
The oracle (oracle/, test infrastructure only) and the synthetic workload generator are compiled
on first use; the HIP library is built by __graft_entry__.build() (cross-compiles without a GPU).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pfilter-noetic_amd")
for p in (ROOT, PKG, os.path.join(PKG, "synth"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP device 0)")
    config.addinivalue_line("markers", "slow: long CPU case")


@pytest.fixture(scope="session")
def pfref():
    import pfref as m
    m.lib()
    return m


@pytest.fixture(scope="session")
def pfsynth():
    import pfsynth as m
    m.lib()
    return m


@pytest.fixture(scope="session")
def pa():
    """The HIP library through its C ABI. GPU tests only: fails loudly when it is not built."""
    import pfilter_amd as m
    m.lib()
    if m.device_count() < 1:
        pytest.fail("no HIP device visible to libpfilter_hip.so")
    return m

