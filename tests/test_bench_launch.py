"""bench.py's N-rank launcher and N>1 data path on CPU (gloo), without torchrun and without a GPU.

`python bench.py --gpus N` started without WORLD_SIZE must start its own N ranks before anything
touches a GPU, and must exit non-zero unless all N finish (VERDICT r01 "Next round" 1); the ranks of
the --plumbing mode run the same GatherPipeline and RGBM transport as the GPU path, with synthetic
shards packed by the host mirror of the march kernel's store and unpacked by the mirror of
bh_tiles_unpack_rgbm."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _bench(*args, env=None, timeout=240):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=str(ROOT))
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    return r.returncode, lines, r.stderr


@pytest.mark.parametrize("transport", ["rgbm14", "rgbm"])
@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_runs_n_ranks_and_verifies_the_gather(n, transport):
    rc, lines, err = _bench("--gpus", str(n), "--plumbing", "--steps", "3", "--transport", transport)
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines            # rank 0 alone prints the line
    d = lines[0]
    assert d["n_gpus"] == n and d["world_size"] == n and d["backend"] == "gloo" and d["transport"] == transport
    assert d["frames_checked"] == 3 and d["gather_verified_bit_exact"] is True


def test_self_launch_fails_loudly_when_a_rank_fails():
    # rank 1 dies after joining the group (test hook); the launcher must stop rank 0, which would
    # otherwise wait in the gather, and return non-zero: never a line claiming n_gpus 2
    rc, lines, _ = _bench("--gpus", "2", "--plumbing", "--steps", "3", env={"BH_PLUMBING_FAIL_RANK": "1"})
    assert rc != 0
    assert all(d.get("gather_verified_bit_exact") is not True for d in lines)


def test_self_launch_deadline_stops_a_hung_rank():
    """A rank that hangs (not one that exits) must not hold the run for the driver's whole limit: the
    launcher's deadline stops every rank and prints one {"error": ...} line."""
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e["BH_PLUMBING_HANG_RANK"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing", "--steps", "3",
                        "--deadline-s", "25", "--pg-timeout-s", "600"],
                       capture_output=True, text=True, timeout=120, env=e, cwd=str(ROOT))
    assert r.returncode != 0
    errs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"error"')]
    assert len(errs) == 1 and "deadline" in errs[0]["error"], r.stdout[-2000:]
    assert not any(x.startswith('{"metric"') for x in r.stdout.splitlines())


def test_process_group_timeout_ends_a_wedged_collective():
    """With the deadline out of the way, the process group's own timeout ends the wait of the rank
    blocked in the gather on the hung peer: it raises, exits non-zero, and the launcher stops the rest."""
    rc, lines, _ = _bench("--gpus", "2", "--plumbing", "--steps", "3", "--deadline-s", "600", "--pg-timeout-s", "8",
                          env={"BH_PLUMBING_HANG_RANK": "1"}, timeout=180)
    assert rc != 0
    assert all(d.get("gather_verified_bit_exact") is not True for d in lines)


def test_watchdog_ends_a_stalled_rank_well_inside_the_driver_limit():
    """A rank that stops making progress (here: the hang hook; on the node, a kernel or a collective that
    never returns) exits through its watchdog after --stall-s, and the launcher stops the rest and prints
    one {"error": ...} line -- long before the deadline and the driver's 600 s."""
    import time
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e["BH_PLUMBING_HANG_RANK"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing", "--steps", "3",
                        "--stall-s", "4", "--deadline-s", "300", "--pg-timeout-s", "300"],
                       capture_output=True, text=True, timeout=200, env=e, cwd=str(ROOT))
    took = time.monotonic() - t0
    assert r.returncode != 0
    assert took < 100, took
    errs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"error"')]
    assert len(errs) == 1 and "watchdog" in errs[0]["error"], r.stdout[-2000:] + r.stderr[-2000:]
    assert "no progress" in r.stderr
    assert not any(x.startswith('{"metric"') for x in r.stdout.splitlines())


def test_default_deadline_is_below_the_driver_limit():
    sys.path.insert(0, str(ROOT))
    import bench
    a = bench.parse([])
    assert 0 < a.deadline_s <= 450 and 0 < a.stall_s < a.deadline_s


def test_frames_per_launch_is_capped_by_rank0_bytes():
    """N > 1: 64 frames per batch, fewer when rank 0's targets and receive slots of a batch would pass the
    byte budget (16384 x 8192 frames at 64 would not fit)."""
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.auto_frames_per_launch(8, 8192, 4096, 512) == 64
    D = bench.auto_frames_per_launch(8, 16384, 8192, 512)
    assert 1 <= D < 64
    per_frame = 2 * 16384 * 8192 * 8 + 2 * (16384 // 8) * (8192 // 8) * 344
    assert D * per_frame <= bench.RANK0_FRAME_BYTES


def test_world_size_mismatch_is_refused():
    rc, lines, err = _bench("--gpus", "2", "--plumbing", env={"WORLD_SIZE": "3", "RANK": "0"})
    assert rc != 0 and not lines
    assert "refusing" in err


@pytest.mark.parametrize("cfg,want", [(1, (256, 256, 64, "A", "off", "strong")), (2, (1920, 1080, 256, "B", "on", "strong")),
                                      (3, (0, 0, 512, "A", "on", "strong")), (4, (0, 0, 512, "A", "on", "config4")),
                                      (5, (0, 0, 1000, "C", "on", "strong"))])
def test_config_flag_maps_the_baseline_configs(cfg, want):
    """bench.py --config N selects BASELINE.json configs[N-1] (frame, cap, camera, scene, workload)."""
    sys.path.insert(0, str(ROOT))
    import bench
    a = bench.apply_config(bench.parse(["--config", str(cfg)]))
    assert (a.width, a.height, a.max_iters, a.camera, a.surfaces, a.workload) == want


def test_rccl_dry_run_needs_one_rank():
    rc, lines, err = _bench("--gpus", "2", "--rccl-dry-run", env={"WORLD_SIZE": "2"})
    assert rc != 0 and not lines and "one rank" in err


@pytest.mark.gpu
def test_rccl_dry_run_gathers_bit_exact():
    """The N>1 code path at one rank over a real RCCL group (nccl backend): RGBM shard render,
    pipelined dist.gather on the GPU, rank-0 unpack of both targets, barrier and the max-over-ranks
    all_gather -- the collectives the driver's 8-GPU run makes, checked on a 1-GPU box."""
    pytest.importorskip("torch")
    rc, lines, err = _bench("--gpus", "1", "--rccl-dry-run", "--verify-gather", "--steps", "16", "--warmup", "8",
                            "--width", "1024", "--height", "512", timeout=300)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    d = lines[0]
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["n_gpus"] == 1
    assert d["gather_verified_bit_exact"] is True
    assert "RCCL DRY RUN" in d["config"]["parallelism"]


def test_steps_are_batches_and_the_settle_is_optional():
    """A step is one batch (one bh_render_frames launch of D frames, VERDICT/ADVICE r02): the driver's
    --steps / --warmup count batches and are never changed; the power-state settle of round 2 is off
    by default (the warm-up batches cover the clock ramp) and can still be asked for."""
    sys.path.insert(0, str(ROOT))
    import bench
    a = bench.parse(["--warmup", "5", "--steps", "20"])
    assert a.settle_ms == 0.0 and a.warmup == 5 and a.steps == 20
    assert bench.parse(["--settle-ms", "100"]).settle_ms == 100.0
    assert bench.auto_frames_per_launch(1, 4096, 2048, 512) == 32
    assert bench.auto_frames_per_launch(8, 4096, 2048, 512) == 64


def test_clock_accumulators_to_mhz():
    """bh_set_clock_probe's per-XCD accumulators (shader ticks, 100 MHz ticks, waves) -> MHz."""
    import numpy as np
    import black_hole_ray_marching_amd as bh
    acc = np.zeros(128, np.int64)
    acc[0:3] = (2_100_000, 100_000, 10)       # XCD 0: 2100 MHz
    acc[16:19] = (2_300_000, 100_000, 10)     # XCD 1: 2300 MHz
    c = bh.clock_mhz(acc)
    assert c["mhz"] == 2200.0 and c["per_xcd_mhz"][:2] == [2100.0, 2300.0] and c["per_xcd_mhz"][2] is None
    assert c["waves"] == 20 and c["wave_ms"] == 0.1  # 1 ms of 100 MHz ticks per 10 waves
