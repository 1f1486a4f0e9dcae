"""Per-kernel effective clock and issue mix from a rocprofv3 --kernel-trace --pmc run.
Usage: python tools/clock_summary.py DIR   (DIR holds run_counter_collection.csv, run_kernel_trace.csv)
clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md 'DVFS give-back')."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import kname  # noqa: E402

d = sys.argv[1]
dur = {}
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
per = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    k = r["Dispatch_Id"]
    names[k] = kname(r["Kernel_Name"])
    per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for k, c in per.items():
    if "k_eval" not in names[k] and "k_multi" not in names[k] and "k_tiled" not in names[k]:
        continue
    ns = dur.get(k)
    if not ns or ns < 1e6:
        continue
    a = agg[names[k]]
    a["ms"].append(ns / 1e6)
    a["clock_ghz"].append(c["GRBM_GUI_ACTIVE"] / 8 / ns)
    for key, v in c.items():
        if key.startswith("SQ_"):
            a[key].append(v)
for name, a in agg.items():
    m = {k: sum(v) / len(v) for k, v in a.items()}
    extra = ""
    if "SQ_INSTS_MFMA" in m:
        extra = f"valu/mfma={m['SQ_INSTS_VALU'] / max(m['SQ_INSTS_MFMA'], 1):.2f} "
    print(f"{name}: launches={len(a['ms'])} ms={m['ms']:.2f} clock={m['clock_ghz']:.3f} GHz " + extra
          + " ".join(f"{k}={m[k]:.4g}" for k in sorted(m) if k.startswith("SQ_")))
