"""Time the fused evaluation pass alone (HIP events around the kernel).
Usage: python tools/bench_pass.py N T [density] [reps] [need_h] [need_y2] [gap_ms]  (need_y2=0: the
orthogonal solver's pass, no Σy²; gap_ms: host idle time between passes, as the solver's host work)"""
import sys
import os
import time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa

n = int(sys.argv[1]); t = int(float(sys.argv[2]))
dens = sys.argv[3] if len(sys.argv) > 3 else "tanh"
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
need_h = bool(int(sys.argv[5])) if len(sys.argv) > 5 else False
need_y2 = bool(int(sys.argv[6])) if len(sys.argv) > 6 else True
gap_ms = float(sys.argv[7]) if len(sys.argv) > 7 else 0.0
d = {"tanh": pa.DensityType.tanh(), "exp": pa.DensityType.exp(), "cube": pa.DensityType.cube()}[dens]
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
w = np.linalg.qr(np.random.default_rng(0).normal(size=(n, n)))[0] * 0.05
ctx.eval(w, mu, d, need_h, need_y2)
ctx.kernel_stats(reset=True)
t0 = time.perf_counter()
for _ in range(reps):
    if gap_ms > 0:
        t_end = time.perf_counter() + gap_ms / 1e3
        while time.perf_counter() < t_end:  # busy host, idle GPU
            pass
    ctx.eval(w, mu, d, need_h, need_y2)
wall = (time.perf_counter() - t0) / reps
k, c, nl = ctx.kernel_stats()
avg = k / nl if nl else c / max(reps, 1)  # tiled / generic paths: whole eval call
fl = (6.0 if need_h else 4.0) * n * n * t
print(f"N={n} T={t} {dens} H={need_h}: kernel {avg:.3f} ms  call {c/max(nl,1):.3f} ms  wall {wall*1e3:.3f} ms  "
      f"{fl/avg/1e9:.2f} TF/s ({fl/avg/1e9/78.6*100:.1f}% of 78.6)  HBM {8*n*t/avg/1e6:.1f} GB/s", flush=True)
