"""Summarise tools/gpu/pmc_configs.sh output into profiles/pmc_traffic.json (read by bench.py).

For each configuration directory: the march kernel's average duration from the kernel trace
(rocprofv3 --stats), the bench's own HIP-event average from its JSON line (they must agree), and
per-launch PMC averages over the dispatches of the full launches (the most common grid size: the
bench's single-frame debug launch and partial launches are excluded).  Corrections per
MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE is reported as x2 of the raw value for wide
coalesced reads (the sky gathers here are 4-byte: the true fetch lies between raw and x2, both are
kept); WRITE_SIZE is exact for 16-B streaming stores (8-B RGBA16F stores: uncalibrated, kept as is).
traffic = FETCH_SIZE x2 + WRITE_SIZE (bytes per launch).

    python tools/pmc_summary.py gpurun_out/pmc_TAG [--write profiles/pmc_traffic.json] [--source TEXT]"""
import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import Counter, defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def kernel_rows(d, pattern="march_tile"):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if pattern in r["Kernel_Name"]]
    return rows


def per_dispatch(rows):
    """{dispatch id: {counter: value}} and each dispatch's grid size."""
    by = defaultdict(dict)
    grid = {}
    for r in rows:
        k = r["Dispatch_Id"]
        by[k][r["Counter_Name"]] = by[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        grid[k] = int(r.get("Grid_Size") or 0)
    return by, grid


def summarise(cdir):
    out = {}
    bench = None
    for f in [f"{cdir}/trace.log"] + sorted(glob.glob(f"{cdir}/p*.log")):
        for line in open(f, errors="replace"):
            if line.startswith('{"metric"') and f.endswith("trace.log"):
                bench = json.loads(line)
    stats = glob.glob(f"{cdir}/trace/**/*kernel_stats.csv", recursive=True)
    if stats:
        rows = [r for r in csv.DictReader(open(stats[0])) if "march_tile" in r["Name"]]
        if rows:  # the build that ran the frames (the bench's one-frame debug launch may pick the other)
            r = max(rows, key=lambda r: int(r["Calls"]))
            out["rocprof_kernel"] = r["Name"]
            out["rocprof_stats_avg_ms_all_dispatches"] = round(float(r["AverageNs"]) / 1e6, 5)
            out["rocprof_calls"] = int(r["Calls"])
    trace = glob.glob(f"{cdir}/trace/**/*kernel_trace.csv", recursive=True)
    if trace:
        # full launches only (the most common grid size), as the bench's HIP-event average
        rows = sorted((r for r in csv.DictReader(open(trace[0])) if "march_tile" in r["Kernel_Name"]),
                      key=lambda r: int(r["Start_Timestamp"]))
        d = [(int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r.get("Grid_Size", 0)),
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]
        if d:
            g = Counter(x for x, _ in d).most_common(1)[0][0]
            full = [t for x, t in d if x == g]
            out["rocprof_avg_ms_all_full_launches"] = round(sum(full) / len(full), 5)
            # the bench's timed launches: the last K full launches (a step is one launch; older bench
            # lines timed `steps` frames in steps // frames_per_launch launches).  The warm-up launches
            # before them run on a still ramping clock
            if bench:
                nt = bench["kernel"].get("launches") or bench["steps"] // bench["kernel"]["frames_per_launch"]
            else:
                nt = len(full)
            timed = full[-nt:] if 0 < nt <= len(full) else full
            out["rocprof_avg_ms"] = round(sum(timed) / len(timed), 5)
            out["rocprof_full_launches"] = len(timed)
    counters = defaultdict(list)
    for p in sorted(glob.glob(f"{cdir}/p[0-9]")):
        by, grid = per_dispatch(kernel_rows(p))
        if not by:
            continue
        g = Counter(grid.values()).most_common(1)[0][0]
        for k, cs in by.items():
            if grid[k] == g:
                for n, v in cs.items():
                    counters[n].append(v)
    c = {n: sum(v) / len(v) for n, v in counters.items()}
    out["counters_per_launch"] = {n: round(v, 1) for n, v in sorted(c.items())}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB
        fetch, write = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        out["fetch_size_bytes_raw"] = int(fetch)
        out["fetch_size_bytes_x2"] = int(2 * fetch)
        out["write_size_bytes"] = int(write)
        out["hbm_bytes_per_launch"] = int(2 * fetch + write)
    if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
        tr = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        out["valu_busy_est"] = round(((c["SQ_INSTS_VALU"] - tr) * 2 + tr * 8) / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
        out["valu_lane_utilization"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
    if c.get("SQ_WAVES"):
        out["valu_per_wave"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"], 1)
        out["trans_per_wave"] = round(c.get("SQ_INSTS_VALU_TRANS_F32", 0) / c["SQ_WAVES"], 2)
        out["salu_per_wave"] = round(c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"], 1)
    if bench:
        k = bench["kernel"]
        out["bench_hip_event_avg_ms"] = k["avg_ms"]
        out["bench_value"] = bench["value"]
        out["algorithmic_bytes_per_launch"] = bench["roofline_hbm"]["algorithmic_bytes_per_launch"]
        cfg = bench["config"]
        out["_key"] = (cfg["width"], cfg["height"], cfg["max_iters"], cfg["camera"], cfg["math"], cfg["schedule"],
                       cfg["format"], bench["n_gpus"], cfg["frames_per_launch"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--write", default="")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    from bench import pmc_key
    table = json.loads(Path(a.write).read_text()) if a.write and os.path.exists(a.write) else {}
    for cdir in sorted(glob.glob(f"{a.dir}/*/")):
        s = summarise(cdir.rstrip("/"))
        key = s.pop("_key", None)
        print(os.path.basename(cdir.rstrip("/")), json.dumps(s))
        if key and a.write:
            cmd = re.sub(r"\S*/bench\.py", "bench.py", open(cdir + "cmd.txt").read().strip())
            s["source"] = a.source or f"rocprofv3 of `{cmd}` ({cdir})"
            s["correction"] = ("FETCH_SIZE x2 per MI355X_MICROARCH.md (gfx950 reports half of wide coalesced reads; "
                               "the sky's 4-B gathers are uncalibrated: true fetch between raw and x2); WRITE_SIZE as read")
            table[pmc_key(*key)] = s
    if a.write:
        Path(a.write).write_text(json.dumps(table, indent=1) + "\n")


if __name__ == "__main__":
    main()
