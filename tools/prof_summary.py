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
    counters = defaultdict(list)
    for p in ("pmc1", "pmc2", "pmc3", "pmc4"):
        for r in _rows(str(d / p / "**" / "*counter_collection.csv")):
            if "march" not in r.get("Kernel_Name", ""):
                continue
            counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res["counters_per_dispatch"] = {k: sum(v) / len(v) for k, v in counters.items()}
    c = res["counters_per_dispatch"]
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        res["valu_lane_utilization"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in c:
                res[f"{k}/SQ_WAVE_CYCLES"] = c[k] / c["SQ_WAVE_CYCLES"]
    return res


if __name__ == "__main__":
    r = summarise(Path(sys.argv[1]))
    s = json.dumps(r, indent=1)
    if "--json" in sys.argv:
        Path(sys.argv[sys.argv.index("--json") + 1]).write_text(s)
    print(s)
