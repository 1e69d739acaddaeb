"""Summarise tools/gpu/bloom_pmc.sh output: per kernel, instructions per wave and the share of wave
cycles parked on waits / stalled at issue / active, LDS bank-conflict cycles over LDS-active cycles.
    python tools/bloom_pmc_summary.py gpurun_out/bloom_pmc_1920"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted({k for k, _ in agg}):
    d = {c: sum(v) / len(v) for (kk, c), v in agg.items() if kk == k}
    w = d.get("SQ_WAVES", 0) or 1
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(k, "waves", int(w), "valu/w %.0f lds/w %.0f salu/w %.0f vmem/w %.0f" % (
        d.get("SQ_INSTS_VALU", 0) / w, d.get("SQ_INSTS_LDS", 0) / w, d.get("SQ_INSTS_SALU", 0) / w,
        d.get("SQ_INSTS_VMEM", 0) / w),
        "wait %.2f issue-stall %.2f (lds %.2f) active %.2f valu-active %.2f" % (
            d.get("SQ_WAIT_ANY", 0) / wc, d.get("SQ_WAIT_INST_ANY", 0) / wc, d.get("SQ_WAIT_INST_LDS", 0) / wc,
            d.get("SQ_ACTIVE_INST_ANY", 0) / wc, d.get("SQ_ACTIVE_INST_VALU", 0) / wc),
        "bankconf/ldsactive %.2f" % (d.get("SQ_LDS_BANK_CONFLICT", 0) / (d.get("SQ_LDS_IDX_ACTIVE", 0) or 1)),
        "wavecyc/wave %.0f" % (wc / w))
