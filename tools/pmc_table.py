"""Per-kernel average PMC counters of a tools/prof_pmc.sh output: python tools/pmc_table.py gpurun_out/pmc_TAG"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    line = {n: f"{v:.4g}" for n, v in sorted(c.items())}
    if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
        tr = c.get("SQ_INSTS_VALU_TRANS_F32", 0)
        line["valu_busy_est"] = f'{((c["SQ_INSTS_VALU"] - tr) * 2 + tr * 8) / (c["GRBM_GUI_ACTIVE"] / 8 * 1024):.3f}'
    if c.get("SQ_WAVES"):
        line["valu_per_wave"] = f'{c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]:.0f}'
        line["lds_per_wave"] = f'{c.get("SQ_INSTS_LDS", 0) / c["SQ_WAVES"]:.0f}'
    print(k[:70], line)
