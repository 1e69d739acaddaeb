"""The shard tile math the kernels use (bh_common.hpp), compiled for the host and checked
exhaustively over shard counts 1..17 and a range of frame sizes (tests/native/shard_check.cpp)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_shard_tile_coords_and_index_are_inverse_bijections(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("hipcc not available")
    exe = tmp_path / "shard_check"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-I", str(ROOT / "black_hole_ray_marching_amd" / "csrc"),
                    str(ROOT / "tests" / "native" / "shard_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 bad" in r.stdout
