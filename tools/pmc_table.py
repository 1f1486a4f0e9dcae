"""Per-kernel table from a rocprofv3 clock pass (--kernel-trace --pmc, tools/prof_r03c.sh) and
optional FETCH_SIZE / WRITE_SIZE passes: launches, mean duration, clock (GRBM_GUI_ACTIVE over
the 8 XCDs), matrix-core busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs), VALU / MFMA
/ LDS instructions, HBM bytes per launch (FETCH_SIZE·2·1024 + WRITE_SIZE·1024, the gfx950
correction of MI355X_MICROARCH.md).
Usage: python tools/pmc_table.py DIR (holding c*_clock/, c*_fetch/, c*_write/) PREFIX"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import kname  # noqa: E402


def load(path):
    agg = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[kname(r["Kernel_Name"])][r["Counter_Name"]].append(
            float(r["Counter_Value"]))
    return agg


def main():
    d, pre = sys.argv[1], sys.argv[2]
    clk = load(os.path.join(d, pre + "_clock", "run_counter_collection.csv"))
    fet = load(os.path.join(d, pre + "_fetch", "run_counter_collection.csv"))
    wri = load(os.path.join(d, pre + "_write", "run_counter_collection.csv"))
    dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, pre + "_clock", "run_kernel_trace.csv"))):
        dur[kname(r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print("%-58s %5s %9s %5s %6s %9s %9s %9s %10s" % ("kernel", "n", "ms", "GHz", "mfma", "VALU", "MFMA", "LDS",
                                                    "HBM GB"))
    rows = []
    for k, v in clk.items():
        c = {n: sum(x) / len(x) for n, x in v.items()}
        ms = sum(dur[k]) / len(dur[k]) if dur[k] else 0.0
        if ms < 0.02:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        f = fet.get(k, {}).get("FETCH_SIZE")
        w = wri.get(k, {}).get("WRITE_SIZE")
        hbm = (sum(f) / len(f) * 2048 + (sum(w) / len(w) * 1024 if w else 0.0)) / 1e9 if f else float("nan")
        rows.append((ms * len(dur[k]), "%-58s %5d %9.3f %5.2f %6.2f %9.3g %9.3g %9.3g %10.3f" % (
            k[:58], len(dur[k]), ms, cyc / (ms * 1e-3) / 1e9, c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc,
            c["SQ_INSTS_VALU"], c["SQ_INSTS_MFMA"], c["SQ_INSTS_LDS"], hbm)))
    for _, line in sorted(rows, reverse=True):
        print(line)


if __name__ == "__main__":
    main()
