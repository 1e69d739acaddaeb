"""The shard tile math the kernels use (bh_common.hpp), compiled for the host and checked
exhaustively over shard counts 1..17 and a range of frame sizes (tests/native/shard_check.cpp)."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
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


@pytest.mark.parametrize("W,H,weights", [(200, 100, [1, 2]), (4096, 2048, [16] + [20] * 7), (96, 72, [0, 3, 3, 3]),
                                         (104, 40, [5, 1, 7]), (64, 64, [1])])
def test_partition_map_matches_mirror(W, H, weights):
    """bh_partition_map (the C host map behind bh_partition_create) equals the Python mirror
    (multigpu.partition_owners / shard_tiles): every tile owned once, each shard's packed order
    row-major over its tiles, shares proportional to the weights."""
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    owner, index = bh.partition_map(W, H, weights)
    tx_n = (W + 7) // 8
    S = len(weights)
    for k in range(S):
        tiles = multigpu.shard_tiles(W, H, k, S, weights)
        t = tiles[:, 1] * tx_n + tiles[:, 0]
        assert np.all(owner[t] == k)
        assert np.array_equal(index[t], np.arange(len(t)))
    assert sum(len(multigpu.shard_tiles(W, H, k, S, weights)) for k in range(S)) == owner.size
    M = sum(weights)
    for k in range(S):
        assert abs((owner == k).mean() - weights[k] / M) < 0.02


def test_partition_owner_spread():
    """Smooth weighted round robin: each shard's residues are spread, never a run longer than needed."""
    from black_hole_ray_marching_amd import multigpu
    own = multigpu.partition_owners([16] + [20] * 7)
    assert len(own) == 156 and own.count(0) == 16
    runs = max(len(r) for r in "".join("x" if o == 0 else "." for o in own).split("."))
    assert runs == 1
