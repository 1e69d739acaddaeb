#!/bin/bash
# Short f64 atan2 core: device selftest against ocml's atan2 (2^28 pairs + fallback rate), GPU parity,
# A/B against the previous build.
set -u
O=gpurun_out/r02aj; mkdir -p $O
timeout -k 10 300 python -u - > $O/selftest_atan2.log 2>&1 <<'PY' || exit 10
import ctypes as C, json, sys
sys.path.insert(0, ".")
import torch
import black_hole_ray_marching_amd as bh
lib = bh.load()
out = {}
for op, n in ((8, 1 << 28), (9, 1 << 28)):
    for seed in (1, 2):
        mm = C.c_uint64(0); ex = (C.c_uint32 * 8)()
        st = lib.bh_selftest_crmath(op, seed, n, C.byref(mm), ex, 0)
        out[f"op{op}_seed{seed}"] = {"status": st, "count": mm.value, "pairs": n, "examples": [hex(v) for v in ex]}
print(json.dumps(out))
PY
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_crmath.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
run() { name=$1; lib=$2; shift 2; BH_LIB=tools/variants/$lib.so timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2 3; do
for v in prevatan newatan; do
  run c3D8_${v}_$r $v
  run c3D1_${v}_$r $v --frames-per-launch 1
  run c1_${v}_$r $v --config 1
done
done
echo done
