"""In-tree build of the native libraries (no cmake, no JIT cache — the .so files travel with the repo).

  black_hole_ray_marching_amd/libbh_render.so   product: HIP kernels for gfx950 + C ABI (hipcc)
  oracle/libbh_oracle.so                        test infrastructure: CPU oracle (gcc, OpenMP)

Run `python -m black_hole_ray_marching_amd.build` or call build_all().
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "_build"
LIB = PKG / "libbh_render.so"
ORACLE_SRCS = [ROOT / "oracle" / "bh_oracle.c", ROOT / "oracle" / "bh_bloom_oracle.c"]
EXAMPLE_SRC = ROOT / "examples" / "render_frame.c"
EXAMPLE_BIN = ROOT / "examples" / "render_frame"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ORACLE_LIB = ROOT / "oracle" / "libbh_oracle.so"

ARCH = os.environ.get("BH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

COMMON = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
# per-translation-unit floating-point contracts (DESIGN.md "Math modes")
TU_FLAGS = {
    # packed FP32 has no throughput advantage on gfx950 (tools/ubench/valu_rates.hip): no SLP packing.
    # No machine scheduling (pre- or post-RA): the step's source order issues faster than the
    # scheduler's interleavings (0.687 -> 0.644 ms headline, A/B r01).  No
    # machine LICM: it hoists loop-invariant materialisations (e.g. the shading's f64 constants) out of
    # the frame-independent loops and lengthens live ranges; off, 0.6226 -> 0.6168 ms per frame
    # headline, 1920x1080 0.162 -> 0.159 ms (A/B r02, profiles/r02b/ab_nolicm.log; the scheduled
    # build below got slower with it, 0.736 -> 0.768 ms at cap 1000, so it keeps LICM).
    "bh_march_exact.hip": ["-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
                           "-mllvm", "-enable-misched=0", "-mllvm", "-enable-post-misched=0",
                           "-mllvm", "-disable-machine-licm"],
    # the same kernels WITH machine scheduling: shorter per-step latency for tail-bound frames
    "bh_march_exact_lat.hip": ["-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize"],
    # the fast (tolerance) kernels: no machine scheduling either (0.468 -> 0.440 ms headline, A/B r01)
    "bh_march_fast.hip": ["-ffp-contract=fast", "-fno-hip-fp32-correctly-rounded-divide-sqrt",
                          "-mllvm", "-enable-misched=0", "-mllvm", "-enable-post-misched=0"],
    "bh_tiles.hip": [],
    # post-RA scheduling off: fused bloom chain 0.556 -> 0.548 ms (A/B r01; pre-RA off too: 0.561)
    # no SLP vectorisation: packed-FP32 forms of the filter's adjacent channel ops cost more than the
    # scalar ops on gfx950 (a v_pk op issues slower than two scalar ones, plus the shuffles and hazard
    # nops around it) and hold more VGPRs
    "bh_bloom.hip": ["-ffp-contract=off", "-fno-slp-vectorize", "-mllvm", "-enable-post-misched=0",
                     "-mllvm", "-pragma-unroll-threshold=200000"],  # the quad pass's 8 taps x 9 read forms
    "bh_selftest.hip": ["-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt"],
    "bh_host.cpp": ["-ffp-contract=off", "-x", "hip"],
    "bh_present.cpp": ["-x", "hip"],
}


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_product(force: bool = False) -> Path:
    OBJ.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.hpp")) + [ROOT / "include" / "bh_render.h"]
    objs, jobs = [], []
    for src, flags in TU_FLAGS.items():
        s = CSRC / src
        o = OBJ / (s.stem + ".o")
        deps = [s, *headers, Path(__file__)] + ([CSRC / "bh_march_exact.hip"] if src == "bh_march_exact_lat.hip" else [])
        if force or _stale(o, deps):
            jobs.append([HIPCC, *COMMON, *flags, "-c", str(s), "-o", str(o)])
        objs.append(o)
    # the translation units compile independently: in parallel (BH_BUILD_JOBS, default min(cpus, 8))
    n = int(os.environ.get("BH_BUILD_JOBS", "0")) or min(os.cpu_count() or 1, 8)
    with ThreadPoolExecutor(max_workers=max(1, n)) as ex:
        list(ex.map(_run, jobs))
    if force or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs)])
        os.replace(tmp, LIB)
    return LIB


def build_oracle(force: bool = False) -> Path:
    if force or _stale(ORACLE_LIB, [*ORACLE_SRCS, ROOT / "include" / "bh_render.h", Path(__file__)]):
        tmp = ORACLE_LIB.with_suffix(".so.tmp")
        # -O3 -ffp-contract=off (no fast-math: the golden tests prove the bits unchanged)
        _run(["gcc", "-O3", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC",
              "-shared", "-o", str(tmp), *map(str, ORACLE_SRCS), "-lm"])
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_example(force: bool = False) -> Path:
    """examples/render_frame: a plain C11 host of the C ABI (gcc + the HIP runtime's C API, no torch)."""
    if force or _stale(EXAMPLE_BIN, [EXAMPLE_SRC, ROOT / "include" / "bh_render.h", LIB, Path(__file__)]):
        tmp = EXAMPLE_BIN.with_suffix(".tmp")
        _run(["gcc", "-std=c11", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT / 'include'}",
              f"-I{ROCM / 'include'}", str(EXAMPLE_SRC), "-o", str(tmp), f"-L{PKG}", "-lbh_render",
              f"-L{ROCM / 'lib'}", "-lamdhip64", "-Wl,-rpath,$ORIGIN/../black_hole_ray_marching_amd",
              f"-Wl,-rpath,{ROCM / 'lib'}", "-lm"])
        os.replace(tmp, EXAMPLE_BIN)
    return EXAMPLE_BIN


def build_all(force: bool = False) -> None:
    build_product(force)
    build_oracle(force)
    build_example(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(LIB)
    print(ORACLE_LIB)
