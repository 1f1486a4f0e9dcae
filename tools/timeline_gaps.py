"""Where a short-kernel run spends its wall time, from one rocprofv3 --kernel-trace --hip-trace
--memory-copy-trace directory: GPU busy time (kernels, copies) against the span from the first to
the last kernel of the solver's passes, the idle gaps between consecutive GPU operations (summed,
by size), and the HIP API calls by total host time.
Usage: python tools/timeline_gaps.py DIR [kernel-substring that marks the fit, default k_eval_fused]"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import kname  # noqa: E402


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_eval_fused"
    ops = []
    for r in rows(d, "*kernel_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + kname(r["Kernel_Name"])))
    for r in rows(d, "*memory_copy_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "copy")))
    ops.sort()
    fit = [o for o in ops if mark in o[2]]
    if not fit:
        print("no kernel matching", mark)
        return
    t0, t1 = fit[0][0], max(o[1] for o in fit)
    win = [o for o in ops if o[0] >= t0 and o[1] <= t1]
    busy = defaultdict(float)
    for s, e, n in win:
        busy[n] += (e - s) / 1e6
    gaps, prev = [], t0
    for s, e, n in win:
        if s > prev:
            gaps.append((s - prev) / 1e6)
        prev = max(prev, e)
    span = (t1 - t0) / 1e6
    print(f"window {span:.3f} ms from the first to the last '{mark}' kernel; GPU busy {sum(busy.values()):.3f} ms, "
          f"idle {sum(gaps):.3f} ms in {len(gaps)} gaps")
    for n, ms in sorted(busy.items(), key=lambda x: -x[1])[:12]:
        cnt = sum(1 for o in win if o[2] == n)
        print(f"  {ms:9.3f} ms  {cnt:5d}x  {n[:90]}")
    gaps.sort()
    if gaps:
        q = lambda p: gaps[min(len(gaps) - 1, int(p * len(gaps)))]  # noqa: E731
        print(f"gaps: median {q(0.5) * 1e3:.1f} us, p90 {q(0.9) * 1e3:.1f} us, max {gaps[-1] * 1e3:.1f} us; "
              f"gaps > 50 us: {sum(g for g in gaps if g > 0.05):.3f} ms in {sum(1 for g in gaps if g > 0.05)}")
    api = defaultdict(lambda: [0.0, 0])
    for r in rows(d, "*hip_api_trace.csv"):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and e <= t1:
            a = api[r["Function"]]
            a[0] += (e - s) / 1e6
            a[1] += 1
    print("HIP API inside the window (host ms, calls):")
    for n, (ms, c) in sorted(api.items(), key=lambda x: -x[1][0])[:12]:
        print(f"  {ms:9.3f} ms  {c:6d}  {n}")


if __name__ == "__main__":
    main()
