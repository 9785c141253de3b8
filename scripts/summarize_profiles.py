"""Condense rocprofv3 outputs of scripts/profile_round.sh into profiles/<tag>_*.{csv,json}."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = f"gpurun_out/prof_{tag}"
dst = "profiles"
os.makedirs(dst, exist_ok=True)
stats = glob.glob(f"{src}/bench/**/*kernel_stats.csv", recursive=True)[0]
shutil.copy(stats, f"{dst}/{tag}_bench_kernel_stats.csv")
for f in glob.glob(f"{src}/bench_dropout/**/*kernel_stats.csv", recursive=True)[:1]:
    shutil.copy(f, f"{dst}/{tag}_bench_dropout_kernel_stats.csv")


def counters(sub):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{src}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "fa2::" not in name:
                continue
            short = name.split("<")[0].replace("void ", "")
            agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
                # the effective clock of this very dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs
                ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                agg[short]["pass_ms"].append(ns * 1e-6)
                agg[short]["clock_ghz"].append(float(r["Counter_Value"]) / 8.0 / ns)
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


fetch, write = counters("fetch"), counters("write")
sq = collections.defaultdict(dict)
for sub in ("sq", "sq1", "sq2"):
    for k, d in counters(sub).items():
        sq[k].update(d)
out = {}
for k in sorted(set(fetch) | set(write) | set(sq)):
    e = {}
    if k in fetch:
        # gfx950: FETCH_SIZE (KB) counts half the bytes of wide coalesced reads -> x2 (MI355X_MICROARCH.md, HBM)
        e["fetch_bytes_raw"] = fetch[k]["FETCH_SIZE"] * 1024
        e["fetch_bytes_corrected"] = 2 * e["fetch_bytes_raw"]
    if k in write:
        e["write_bytes"] = write[k]["WRITE_SIZE"] * 1024
    if "fetch_bytes_corrected" in e and "write_bytes" in e:
        e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
    e.update({c: v for c, v in sq.get(k, {}).items()})
    if "SQ_VALU_MFMA_BUSY_CYCLES" in e and e.get("GRBM_GUI_ACTIVE"):
        # MFMA-busy share of every SIMD's cycles: busy cycles (summed over the 1024 SIMDs) over
        # 1024 x the kernel's GPU-active cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
        e["mfma_busy_pct"] = 100.0 * e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * e["GRBM_GUI_ACTIVE"] / 8)
    out[k] = e
json.dump(out, open(f"{dst}/{tag}_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
