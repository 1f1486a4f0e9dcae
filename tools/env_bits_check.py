"""Bit-identity of the fused pass under two environment settings read at context creation
(schedule knobs such as PICARD_G8X_SKEW): one context per setting on the same generated X,
the same W, and the pass statistics compared exactly. Also checks the digit-G path ran.
Usage: python tools/env_bits_check.py VAR VALUE_A VALUE_B [N] [T]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 128
t = int(float(sys.argv[5])) if len(sys.argv) > 5 else 2_000_000
out = {}
for v in (va, vb):
    os.environ[var] = v
    ctx = pa.DeviceContext(0)
    ctx.generate(n, t, 42)
    mu = ctx.rowsum() / t
    res = []
    for seed in range(3):
        w = np.linalg.qr(np.random.default_rng(seed).normal(size=(n, n)))[0] * (0.05 + 0.3 * seed)
        st = ctx.eval(w, mu, pa.DensityType.tanh(), False, need_y2=False)
        res.append(np.concatenate([np.ravel(np.asarray(st[k])) for k in sorted(st) if st[k] is not None]))
    out[v] = (res, ctx.g8_passes)
    ctx.close()
same = all(np.array_equal(a, b) for a, b in zip(out[va][0], out[vb][0]))
print(f"{var}={va} vs {vb}: bit-identical {same}; digit-G passes {out[va][1]} / {out[vb][1]}")
sys.exit(0 if same and out[va][1] > 0 and out[vb][1] > 0 else 1)
