"""Time the row-major Y = W·(X − μ) store pass (the transform / sources kernel) alone: the
fp64 MFMA store (k_ystore) first, then — after one loss-only pass has built the int8 digit
image — the int8-digit store (k_ystore_oz). Usage: python tools/bench_transform.py N T [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

n = int(sys.argv[1]); t = int(float(sys.argv[2]))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
w = np.ascontiguousarray(np.linalg.qr(np.random.default_rng(0).normal(size=(n, n)))[0])
fl = 2.0 * n * n * t
for label in ("k_ystore", "k_ystore_oz"):
    if label == "k_ystore_oz":
        ctx.eval_split(w, mu, pa.DensityType.tanh(), False)  # builds the digit image
    n8 = ctx.int8_passes
    ctx.sources_device(w, mu)
    ms = [ctx.sources_device(w, mu)[2] for _ in range(reps)]
    assert (ctx.int8_passes > n8) == (label == "k_ystore_oz"), label
    avg = sum(ms) / len(ms)
    print(f"N={n} T={t}: {label:12s} {avg:.3f} ms  {fl / avg / 1e9:.2f} TF/s-equiv ({fl / avg / 1e9 / 78.6 * 100:.1f}% of "
          f"fp64 78.6)  {16.0 * n * t / avg / 1e6:.0f} GB/s (8 B read + 8 B written per element)", flush=True)
