"""How much of the bloom runs under the march, from a rocprofv3 kernel trace (--kernel-trace --output-format csv) of
tools/bench_frame.py or any run that interleaves march and bloom launches:
    python tools/prof_overlap.py run_kernel_trace.csv [--from-dispatch N]
For every bloom kernel (bh::bloom::*) the share of its duration during which some march kernel (march_*_kernel)
was also executing, time-weighted over all bloom kernels; the same per queue pair; and the busy time of the union
of all kernels against the sum of the march and bloom kernel times (the overlap the trace shows)."""
import argparse
import csv
import json
from collections import defaultdict


def intervals_union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, merged):
    """length of [a, b) covered by the merged (sorted, disjoint) intervals"""
    tot = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        tot += min(b, y) - max(a, x)
    return tot


p = argparse.ArgumentParser()
p.add_argument("trace")
p.add_argument("--from-dispatch", type=int, default=0, help="ignore dispatches before this id (warm-up)")
args = p.parse_args()
march, bloom = [], []
queues = defaultdict(int)
with open(args.trace) as f:
    for r in csv.DictReader(f):
        if int(r["Dispatch_Id"]) < args.from_dispatch:
            continue
        name, a, b = r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "march_" in name and "_kernel" in name:
            march.append((a, b))
            queues[("march", r["Queue_Id"])] += 1
        elif "bh::bloom::" in name:
            bloom.append((a, b, name))
            queues[("bloom", r["Queue_Id"])] += 1
mm = intervals_union([(a, b) for a, b in march])
bl_t = sum(b - a for a, b, _ in bloom)
bl_under = sum(covered(a, b, mm) for a, b, _ in bloom)
per = defaultdict(lambda: [0, 0])
for a, b, n in bloom:
    k = n.split("(")[0].split("<")[0]
    per[k][0] += b - a
    per[k][1] += covered(a, b, mm)
allu = intervals_union([(a, b) for a, b in march] + [(a, b) for a, b, _ in bloom])
busy = sum(y - x for x, y in allu)
out = {"march_kernels": len(march), "bloom_kernels": len(bloom),
       "march_ms": round(sum(y - x for x, y in mm) / 1e6, 4), "bloom_kernel_ms": round(bl_t / 1e6, 4),
       "bloom_share_under_march": round(bl_under / bl_t, 4) if bl_t else None,
       "busy_union_ms": round(busy / 1e6, 4),
       "saved_vs_serial_ms": round((sum(y - x for x, y in mm) + bl_t - busy) / 1e6, 4),
       "per_bloom_kernel": {k: {"ms": round(v[0] / 1e6, 4), "under_march": round(v[1] / v[0], 3)} for k, v in per.items()},
       "queues": {f"{k[0]}:{k[1]}": v for k, v in queues.items()}}
print(json.dumps(out))
