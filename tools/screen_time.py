"""Timing of the line-search screen at (N, T) = (128, 2e7): python screen_time.py reps [gap_ms]
(env picks the form; gap_ms > 0 sleeps that long on the host between launches)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import picard_ica_amd as pa
n, t = 128, 20_000_000
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
gap = float(sys.argv[2]) / 1e3 if len(sys.argv) > 2 else 0.0
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
w = np.ascontiguousarray(np.linalg.qr(np.random.default_rng(0).normal(size=(n, n)))[0] * 0.05)
d = pa.DensityType.tanh()
ll0, b0 = ctx.eval_loss_screen(w, mu, d)
ctx.screen_stats(reset=True)
for _ in range(reps):
    if gap > 0:
        time.sleep(gap)
    ctx.eval_loss_screen(w, mu, d)
ms, nl = ctx.screen_stats(reset=False)[:2]
print(f"PICARD_SCREEN32={os.environ.get('PICARD_SCREEN32', '0')} gap {gap * 1e3:g} ms: screen {ms / max(nl, 1):.3f} ms over {nl}  "
      f"ll[0] {ll0[0]:.10e} bound[0] {b0[0]:.3e}", flush=True)
