import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pivot-scheduling_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and the HIP library")


@pytest.fixture(scope="session")
def engine():
    """The GPU engine; every gpu test fails loudly (never skips) when it cannot load."""
    from pivot_place.engine import PlacementEngine
    return PlacementEngine(0)
