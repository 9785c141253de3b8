"""Print per-kernel PMC averages of a rocprofv3 output tree (dev tool): python scripts/sum_pmc.py DIR"""
import collections
import csv
import glob
import sys

src = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "fa2::" not in n:
            continue
        agg[n.split("<")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    e = {c: sum(v) / len(v) for c, v in d.items()}
    print(k, " ".join(f"{c}={v / 1e6:.1f}M" for c, v in sorted(e.items())))
    if "SQ_WAVE_CYCLES" in e:
        w = e["SQ_WAVE_CYCLES"]
        print("   wait_any %.0f%% wait_inst_any %.0f%% active %.0f%%" % (
            100 * e["SQ_WAIT_ANY"] / w, 100 * e["SQ_WAIT_INST_ANY"] / w, 100 * e["SQ_ACTIVE_INST_ANY"] / w))
        print("   mfma busy %.1f%%" % (100 * e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * e["GRBM_GUI_ACTIVE"] / 8)))
