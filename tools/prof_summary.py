"""Summarise a tools/profile.sh output directory: per-kernel avg duration and PMC counters per dispatch.

  python tools/prof_summary.py gpurun_out/prof_TAG [--json out.json]
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def summarise(d: Path) -> dict:
    res = {"dir": str(d)}
    stats = _rows(str(d / "trace" / "**" / "*kernel_stats.csv"))
    res["kernel_stats"] = [{k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                                                         "MinNs", "MaxNs")} for r in stats]
    # counters per dispatch of the march kernel instantiation with the most dispatches (the timed one)
    by_kernel = defaultdict(lambda: defaultdict(list))
    for p in ("pmc1", "pmc2", "pmc3", "pmc4"):
        for r in _rows(str(d / p / "**" / "*counter_collection.csv")):
            if "march" not in r.get("Kernel_Name", ""):
                continue
            by_kernel[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not by_kernel:
        res["counters_per_dispatch"] = {}
        return res
    name = max(by_kernel, key=lambda k: max(len(v) for v in by_kernel[k].values()))
    counters = by_kernel[name]
    res["counters_kernel"] = name
    res["counters_dispatches"] = max(len(v) for v in counters.values())
    res["counters_per_dispatch"] = {k: sum(v) / len(v) for k, v in counters.items()}
    c = res["counters_per_dispatch"]
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        res["valu_lane_utilization"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                res[f"{k}/SQ_WAVE_CYCLES"] = c[k] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
        # VALU busy estimate: issue cycles of the executed VALU instructions (wave64 on a SIMD-32:
        # 2 cycles, transcendental f32 8 cycles, MI355X_MICROARCH.md cycle constants) over the SIMD
        # cycles of the dispatch (GRBM_GUI_ACTIVE sums the 8 XCDs; 256 CUs x 4 SIMDs)
        trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        busy = (c["SQ_INSTS_VALU"] - trans) * 2.0 + trans * 8.0
        res["valu_busy_est"] = busy / (c["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
    return res


if __name__ == "__main__":
    r = summarise(Path(sys.argv[1]))
    s = json.dumps(r, indent=1)
    if "--json" in sys.argv:
        Path(sys.argv[sys.argv.index("--json") + 1]).write_text(s)
    print(s)
