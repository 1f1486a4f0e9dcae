"""Time the tiled-path passes (full with/without H, loss-only, multi-try) at one shape.
Usage: python tools/bench_tiled.py N T [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

n = int(sys.argv[1]); t = int(float(sys.argv[2])); reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
rng = np.random.default_rng(0)
w = np.linalg.qr(rng.normal(size=(n, n)))[0] * 0.05
z = rng.normal(size=(n, n)) * 0.001
d = pa.DensityType.tanh()
gemm = 2.0 * n * n * t


def timeit(label, fn, units, kind):
    fn()
    ctx.kernel_breakdown(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    wall = (time.perf_counter() - t0) / reps * 1e3
    b = ctx.kernel_breakdown()
    ms = b[kind][0] / max(b[kind][1], 1)
    print(f"N={n} T={t} {label:14s}: kernel {ms:8.2f} ms  wall {wall:8.2f} ms  "
          f"{units * gemm / ms / 1e9:6.2f} TF/s (GEMM-units {units})", flush=True)


timeit("full+H", lambda: ctx.eval(w, mu, d, True), 3, "fused")
timeit("full", lambda: ctx.eval(w, mu, d, False), 2, "fused")
timeit("loss-only", lambda: ctx.eval_split(w, mu, d, True), 1, "loss")
for na in (1, 3, 11):
    timeit(f"multi na={na}", lambda: ctx.eval_loss_multi(w, z, 0.5 ** np.arange(na), mu, d), 2, "multi")
