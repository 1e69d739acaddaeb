import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from black_hole_ray_marching_amd.build import build_all
    build_all()


@pytest.fixture(scope="session")
def sky_small():
    """1024x512 synthetic sky (same generator as the 4096x2048 bench sky, smaller for speed)."""
    import black_hole_ray_marching_amd as bh
    return bh.synthetic_sky(1024, 512, seed=0x5EED_B1AC_401E)
