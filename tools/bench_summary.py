"""Print the key numbers of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4g  ms/step %.1f  passes/iter %.2f (+%.2f screens)  iters %s" % (
    d["value"], d["ms_per_step"], d["passes_per_iter"], d.get("screen_passes_per_iter", 0.0), d["iters_to_tol"]))
if d.get("whole_fit"):
    w = d["whole_fit"]
    print("whole fit %.4g samples/s/iter  %.2f s  %.2f passes/iter" % (w["samples_per_s_per_iter"], w["iterations_s"],
                                                                     w["passes_per_iter"]))
for r in d.get("roofline_kernels", []):
    print("  %-44s %8.2f ms  frac %.3f (%s %.4g of %.4g)  traffic %s" % (
        r["kernel"], r["avg_kernel_ms"], r["frac"], r["unit"], r["achieved"], r["peak"], r["traffic"]))
for k, c in (d.get("other_configs") or {}).items():
    print("  %s %-48s iters %4d  setup %.2fs  iter %.2fs  %.3g samples/s/iter  passes %d  amari %.2e" % (
        k, c["workload"], c["iters_to_tol"], c["setup_s"], c["iterations_s"], c["samples_per_s_per_iter"],
        c["passes"], c["amari_vs_true_mixing"]))
    print("      kernel ms", c["kernel_ms"], "launches", c["kernel_launches"])
    for key in ("cpu_baseline", "cpu_baseline_jade"):
        if c.get(key):
            print("      %s %.4g %s (%s cores)" % (key, c[key]["value"], c[key]["unit"], c[key]["cores"]))
if d.get("cpu_baseline"):
    print("  C3 cpu_baseline %.4g %s (%s cores)" % (d["cpu_baseline"]["value"], d["cpu_baseline"]["unit"], d["cpu_baseline"]["cores"]))
if d.get("transform"):
    t = d["transform"]
    print("  transform %s %.2f ms  frac %.3f of its executed roof (%.2f ms)  %.0f GB/s" % (
        t["kernel"], t["avg_kernel_ms"], t["frac"], t["executed_bound_ms"], t["hbm_gbs_algorithmic"]))
