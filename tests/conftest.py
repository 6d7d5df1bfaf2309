import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path")
    config.addinivalue_line("markers", "slow: full-size (BASELINE-resolution) GPU runs")


@pytest.fixture(scope="session")
def built():
    """Build the in-tree libraries once (no-op when up to date)."""
    from grayshift_amd import build
    build.build_product()
    build.build_oracle()
    build.build_kat()
    return True
