"""Summarise a rocprofv3 --pmc FETCH_SIZE[/WRITE_SIZE] CSV for the fused pass.

HBM bytes per launch = FETCH_SIZE(KB)·1024·2 (+ WRITE_SIZE·1024): on gfx950
FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact for 16-B stores.
Usage: python tools/pmc_summary.py <counter_collection.csv> <n> <t_local> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, n, t_local = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else None
    vals = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            if "k_eval_fused" not in row["Kernel_Name"]:
                continue
            vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    best = max(vals, key=lambda k: len(vals[k]["FETCH_SIZE"]))
    fetch = sum(vals[best]["FETCH_SIZE"]) / len(vals[best]["FETCH_SIZE"])
    write = (sum(vals[best]["WRITE_SIZE"]) / len(vals[best]["WRITE_SIZE"])) if vals[best]["WRITE_SIZE"] else 0.0
    hbm = fetch * 1024 * 2 + write * 1024
    res = {"kernel": best, "n": n, "t_local": t_local, "launches": len(vals[best]["FETCH_SIZE"]),
           "fetch_size_kb_raw": fetch, "write_size_kb_raw": write, "hbm_bytes_per_launch": hbm,
           "algorithmic_bytes_per_launch": 8.0 * n * t_local, "ratio": hbm / (8.0 * n * t_local),
           "source": path}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
