"""Per-wave counters of the march kernel from rocprofv3 --pmc runs of tools/probe_rank0.py (tools/gpu/r04o.sh):
    python tools/shard_pmc.py gpurun_out/r04o
For each n: VALU / SALU / VMEM instructions per wave, wave cycles per wave, the share of wave cycles waiting,
and L2->HBM fetch bytes per tile (FETCH_SIZE in KiB, x2 per MI355X_MICROARCH.md)."""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    tot = defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "march_tile" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


for n in (1, 8):
    a, b = load(f"{sys.argv[1]}/n{n}_p1"), load(f"{sys.argv[1]}/n{n}_p2")
    w = a.get("SQ_WAVES", 0) or 1
    wb = b.get("SQ_WAVES", 0) or 1
    print(f"n={n}: waves {w:.0f}  valu/wave {a['SQ_INSTS_VALU'] / w:.1f}  salu/wave {a['SQ_INSTS_SALU'] / w:.1f}  "
          f"vmem_rd/wave {a['SQ_INSTS_VMEM_RD'] / w:.2f}  wave-cycles/wave {a['SQ_WAVE_CYCLES'] / w:.0f}  "
          f"wait-inst share {a['SQ_WAIT_INST_ANY'] / max(a['SQ_WAVE_CYCLES'], 1):.3f}  "
          f"valu-active/wave-cycles {a['SQ_ACTIVE_INST_VALU'] / max(a['SQ_WAVE_CYCLES'], 1):.3f}  "
          f"fetch KiB/wave (x2) {2 * b['FETCH_SIZE'] / wb:.2f}")
