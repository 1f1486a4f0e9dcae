"""Fixed host-side cost of one evaluator call (upload of W and its digits, launch, the
stats download and synchronisation) at a tiny T where the kernels take microseconds: wall
time per call minus HIP-event kernel time. W alternates between two values so that the
digit split is redone as in a line search. Usage: python tools/bench_overhead.py [reps] [N] [T]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n = int(sys.argv[2]) if len(sys.argv) > 2 else 128
t = int(float(sys.argv[3])) if len(sys.argv) > 3 else 65536
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
rng = np.random.default_rng(0)
ws = [np.ascontiguousarray(np.linalg.qr(rng.normal(size=(n, n)))[0]) for _ in range(2)]
d = pa.DensityType.tanh()
calls = {
    "screen": lambda w: ctx.eval_loss_screen(w, mu, d),
    "loss (split)": lambda w: ctx.eval_split(w, mu, d, False),
    "fused": lambda w: ctx.eval(w, mu, d, False, need_y2=False),
}
for name, f in calls.items():
    for i in range(5):
        f(ws[i & 1])
    ctx.kernel_stats(reset=True)
    ctx.kernel_breakdown(reset=True)
    ctx.screen_stats(reset=True)
    t0 = time.perf_counter()
    for i in range(reps):
        f(ws[i & 1])
    wall = (time.perf_counter() - t0) / reps * 1e3
    _, call_ms, _ = ctx.kernel_stats(reset=False)
    kern = sum(v[0] for v in ctx.kernel_breakdown().values()) + ctx.screen_stats()[0]
    print(f"{name:14s} wall {wall:.3f} ms per call, in-library {call_ms / reps:.3f} ms, "
          f"kernels {kern / reps:.3f} ms", flush=True)
