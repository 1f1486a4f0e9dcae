"""Time the loss-only line-search pass alone (HIP events around the kernel), int8-slice
and fp64 Y stages. Usage: python tools/bench_loss.py N T [reps] [mode ...]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import picard_ica_amd as pa  # noqa: E402

n = int(sys.argv[1]); t = int(float(sys.argv[2]))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
modes = sys.argv[4:] or ["auto", "f64"]
ctx = pa.DeviceContext(0)
ctx.generate(n, t, 42)
mu = ctx.rowsum() / t
w = np.ascontiguousarray(np.linalg.qr(np.random.default_rng(0).normal(size=(n, n)))[0] * 0.05)
d = pa.DensityType.tanh()
st = np.empty(n * n + 3 * n)
kept = C.c_int32()
err = C.create_string_buffer(1024)
for mode in modes:
    ctx.set_y_stage(mode)
    call = lambda: lib_call()  # noqa: E731

    def lib_call():
        rc = pa.lib.pc_ctx_eval_loss(ctx.h, w.ctypes.data_as(C.POINTER(C.c_double)), n,
                                     mu.ctypes.data_as(C.POINTER(C.c_double)), d._c(), 2,
                                     st.ctypes.data_as(C.POINTER(C.c_double)), C.byref(kept), err, len(err))
        assert rc == 0, err.value
    lib_call()
    ctx.kernel_breakdown(reset=True)
    for _ in range(reps):
        lib_call()
    ms, nl = ctx.kernel_breakdown()["loss"]
    avg = ms / max(nl, 1)
    fl = 2.0 * n * n * t
    print(f"{mode:5s} N={n} T={t}: loss kernel {avg:.3f} ms  {fl / avg / 1e9:.2f} TF/s-equiv "
          f"({fl / avg / 1e9 / 78.6 * 100:.1f}% of fp64 78.6)  int8 passes {ctx.int8_passes}", flush=True)
    if mode == "auto":
        ctx.eval_loss_screen(w, mu, d)
        ctx.screen_stats(reset=True)
        for _ in range(reps):
            ctx.eval_loss_screen(w, mu, d)
        ms, nl = ctx.screen_stats()
        print(f"{mode:5s} N={n} T={t}: screen kernel {ms / max(nl, 1):.3f} ms", flush=True)
        w2 = np.ascontiguousarray(w[::-1])  # another try of the same shape
        try:
            ctx.eval_loss_screen2(w, w2, mu, d)
            ctx.screen_stats(reset=True)
            for _ in range(reps):
                ctx.eval_loss_screen2(w, w2, mu, d)
            ms, nl = ctx.screen_stats()
            print(f"{mode:5s} N={n} T={t}: screen pair kernel {ms / max(nl, 1):.3f} ms "
                  f"({ms / max(nl, 1) / 2:.3f} ms per try)", flush=True)
        except pa.Unsupported:
            pass
    ctx.eval(w, mu, d, False, need_y2=False)
    ctx.kernel_breakdown(reset=True)
    for _ in range(reps):
        ctx.eval(w, mu, d, False, need_y2=False)
    ms, nl = ctx.kernel_breakdown()["fused"]
    avg = ms / max(nl, 1)
    print(f"{mode:5s} N={n} T={t}: fused kernel {avg:.3f} ms  {2 * fl / avg / 1e9:.2f} TF/s-equiv "
          f"({2 * fl / avg / 1e9 / 78.6 * 100:.1f}% of fp64 78.6)", flush=True)
