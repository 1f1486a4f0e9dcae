"""Time fused vs split (loss-only + completion) evaluation at one shape.
Usage: python tools/bench_split.py N T [reps] [density]"""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa

n = int(sys.argv[1]); t = int(float(sys.argv[2])); reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dens = sys.argv[4] if len(sys.argv) > 4 else "tanh"
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
scale = float(sys.argv[5]) if len(sys.argv) > 5 else 0.05
w = np.linalg.qr(np.random.default_rng(0).normal(size=(n, n)))[0] * scale
d = {"tanh": pa.DensityType.tanh(), "exp": pa.DensityType.exp(), "cube": pa.DensityType.cube()}[dens]
ctx.eval(w, mu, d, False, need_y2=False); ctx.eval_split(w, mu, d, False, need_y2=False)
ctx.kernel_breakdown(reset=True)
for _ in range(reps):
    ctx.eval(w, mu, d, False, need_y2=False)  # as the orthogonal solver calls them
    ctx.eval_split(w, mu, d, False, need_y2=False)
b = ctx.kernel_breakdown()
fl = 4.0 * n * n * t
for k, (ms, nl) in b.items():
    if nl:
        avg = ms / nl
        f = fl if k == "fused" else fl / 2
        print(f"N={n} T={t} {dens:4s} {k:6s}: {avg:8.3f} ms  {f/avg/1e9:6.2f} TF/s ({f/avg/1e9/78.6*100:5.1f}%)  "
              f"store={'off' if os.environ.get('PICARD_NO_YSTORE') else 'on'}", flush=True)
