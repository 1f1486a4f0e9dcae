"""Per-kernel HBM traffic, clock and issue mix from separate rocprofv3 passes.

Usage: python tools/pmc_kernels.py OUT.json ALG.json DIR [DIR ...]
  each DIR holds run_counter_collection.csv (and run_kernel_trace.csv when the
  pass ran with --kernel-trace). Counters are averaged per kernel name (template
  arguments kept, parameter list dropped) over launches longer than 0.2 ms.
  ALG.json maps a substring of the kernel name to its algorithmic bytes per
  launch ({"k_eval_loss2<0, false": 1.024e11, ...}); the first match wins.

HBM bytes = FETCH_SIZE·1024·2 + WRITE_SIZE·1024 (gfx950: FETCH_SIZE reports
half the bytes of a wide coalesced streaming read; WRITE_SIZE is exact for
16-B stores — MI355X_MICROARCH.md §HBM). clock = GRBM_GUI_ACTIVE / 8 XCDs /
duration. MFMA issue share = SQ_INSTS_MFMA·64 cycles / (SQ_BUSY_CYCLES-based
SIMD cycles), VALU share = (SQ_INSTS_VALU − SQ_INSTS_MFMA)·4 / same.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import kname  # noqa: E402


def load(d):
    dur = {}
    tp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per = collections.defaultdict(dict)
    names = {}
    cp = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(cp)):
        k = r["Dispatch_Id"]
        names[k] = kname(r["Kernel_Name"])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return dur, per, names


def main():
    out_path, alg_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    alg = json.load(open(alg_path)) if os.path.exists(alg_path) else {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        dur, per, names = load(d)
        for k, c in per.items():
            ns = dur.get(k)
            if ns is not None and ns < 2e5:
                continue
            a = agg[names[k]]
            if ns is not None:
                a["ms"].append(ns / 1e6)
                if "GRBM_GUI_ACTIVE" in c:
                    a["clock_ghz"].append(c["GRBM_GUI_ACTIVE"] / 8 / ns)
            for key, v in c.items():
                a[key].append(v)
    res = {"sources": dirs, "kernels": {}}
    for name, a in sorted(agg.items()):
        m = {k: sum(v) / len(v) for k, v in a.items()}
        e = {"launches": max(len(v) for v in a.values())}
        if "ms" in m:
            e["avg_ms"] = m["ms"]
        if "clock_ghz" in m:
            e["clock_ghz"] = m["clock_ghz"]
        if "FETCH_SIZE" in m:
            e["fetch_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            e["write_bytes"] = m["WRITE_SIZE"] * 1024
        if "fetch_bytes" in e or "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e.get("fetch_bytes", 0.0) + e.get("write_bytes", 0.0)
        for sub, b in alg.items():
            if sub in name:
                e["algorithmic_bytes_per_launch"] = b
                if "hbm_bytes_per_launch" in e and "fetch_bytes" in e and "write_bytes" in e:
                    e["traffic_ratio"] = e["hbm_bytes_per_launch"] / b
                break
        if "SQ_INSTS_MFMA" in m and "SQ_INSTS_VALU" in m:
            e["valu_per_mfma"] = m["SQ_INSTS_VALU"] / max(m["SQ_INSTS_MFMA"], 1.0)
            if "ms" in m and "clock_ghz" in m:
                simd_cycles = m["ms"] * 1e-3 * m["clock_ghz"] * 1e9 * 1024  # 256 CUs × 4 SIMDs
                e["mfma_issue_share"] = m["SQ_INSTS_MFMA"] * 64 / simd_cycles
                e["valu_issue_share"] = (m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]) * 4 / simd_cycles
        for key in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES",
                    "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU"):
            if key in m:
                e[key] = m[key]
        res["kernels"][name] = e
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for name, e in res["kernels"].items():
        cols = [f"{name[:60]:60s}", f"n={e['launches']:4d}"]
        if "avg_ms" in e:
            cols.append(f"{e['avg_ms']:9.3f} ms")
        if "clock_ghz" in e:
            cols.append(f"{e['clock_ghz']:.3f} GHz")
        if "hbm_bytes_per_launch" in e:
            cols.append(f"hbm {e['hbm_bytes_per_launch'] / 1e9:8.3f} GB")
        if "traffic_ratio" in e:
            cols.append(f"x{e['traffic_ratio']:.3f} alg")
        if "mfma_issue_share" in e:
            cols.append(f"mfma {e['mfma_issue_share']:.2f} valu {e['valu_issue_share']:.2f}")
        print("  ".join(cols))


if __name__ == "__main__":
    main()
