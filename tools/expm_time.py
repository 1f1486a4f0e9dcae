"""Try 1's map: device (pc_ctx_matrix_exp, k_expm_ps) against host (pc_matrix_exp) time per call
for skew directions of the sizes the fits use. Usage: python tools/expm_time.py [reps]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = pa.DeviceContext(0)
ctx.load(np.random.default_rng(0).normal(size=(8, 64)))
P = C.POINTER(C.c_double)
for n in (64, 128):
    for scale in (1e-17, 0.05, 0.3, 1.0):
        b = np.random.default_rng(n).normal(size=(n, n)) * scale / np.sqrt(n)
        a = np.ascontiguousarray(b - b.T)
        out = np.empty_like(a)
        try:
            ctx.matrix_exp(a)
        except pa.Unsupported as e:
            print(f"n {n} scale {scale}: {e}", flush=True)
            continue
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.matrix_exp(a)
        td = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        for _ in range(reps):
            pa.lib.pc_matrix_exp(a.ctypes.data_as(P), n, out.ctypes.data_as(P))
        th = (time.perf_counter() - t0) / reps * 1e3
        print(f"n {n} scale {scale}: device {td:.3f} ms  host {th:.3f} ms  same bits {np.array_equal(ctx.matrix_exp(a), out)}",
              flush=True)
