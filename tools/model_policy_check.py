"""Count the schedule policies' passes on the bit-identity fits of tests/test_gpu_int8.py
(test_screened_fit_bit_identical): per (n, seed), the "[picard-model]" full passes (later tries
the quadratic model predicts accepted), screens, and whether the fit equals the int8-exact one.
Usage (GPU): PICARD_TRACE=1 python tools/model_policy_check.py 2> trace.err"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

for n, seed, t in [(128, 42, 200003), (96, 7, 200003), (64, 42, 200003), (48, 3, 200003), (128, 42, 2000003),
                   (128, 7, 2000003)]:
    res = {}
    for mode in ("auto", "int8-exact"):
        ctx = pa.DeviceContext(0)
        ctx.generate(n, t, seed)
        ctx.set_y_stage(mode)
        sv = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60))
        sys.stderr.write(f"=== fit n={n} seed={seed} t={t} mode={mode}\n")
        sys.stderr.flush()
        while not sv.step():
            pass
        res[mode] = (sv.finish(), ctx.screen_stats())
        sv.close()
    (r, st), (r0, _) = res["auto"], res["int8-exact"]
    same = r.n_iterations == r0.n_iterations and np.array_equal(r.unmixing, r0.unmixing)
    print(f"n={n} seed={seed} t={t}: iterations {r.n_iterations}, screen stats {st}, bit-identical {same}", flush=True)
