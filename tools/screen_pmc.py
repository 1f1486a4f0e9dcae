"""Summary of tools/gpu_screen_pmc.sh: per kernel (screen launches only), the mean of every counter
of the three PMC passes, the clock (GRBM_GUI_ACTIVE over 8 XCDs) and the per-SIMD cycle split.
Usage: python tools/screen_pmc.py DIR (holding p1/ p2/ p3/)"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import kname  # noqa: E402


def main():
    d = sys.argv[1]
    cnt = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for p in ("p1", "p2", "p3"):
        for f in glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, p, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in cnt.items():
        c = {n: sum(x) / len(x) for n, x in v.items()}
        ms = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        cyc = c.get("GRBM_GUI_ACTIVE", float("nan")) / 8
        print(f"{k}: {len(dur[k])} launches, {ms:.3f} ms, {cyc / (ms * 1e-3) / 1e9:.2f} GHz, {cyc:.4g} cycles")
        simd = 1024.0
        for n in sorted(c):
            per = c[n] / simd
            print(f"   {n:30s} {c[n]:12.4g}   per SIMD {per:12.4g}   per SIMD / cycles {per / cyc:8.3f}")


if __name__ == "__main__":
    main()
