"""Run BASELINE configs end-to-end on one GPU (device-generated bench mixture).
Usage: python tools/run_configs.py C2 [C4 C5 ...] [--oracle] [--max-iter=K] [--maps=PATH]  → one JSON line per config."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import picard_ica_amd as pa  # noqa: E402

CONFIGS = {
    "C1": dict(n=8, t=10_000, kw=dict()),
    "C2": dict(n=64, t=1_000_000, kw=dict()),
    "C3": dict(n=128, t=100_000_000, kw=dict()),
    "C4": dict(n=256, t=10_000_000, kw=dict(ortho=False, extended=False, m=7)),
    "C5": dict(n=64, t=10_000_000, kw=dict(jade_it=50)),
}


def run(name, oracle=False, max_iter=None):
    c = CONFIGS[name]
    n, t = c["n"], c["t"]
    kw = dict(c["kw"], **({"max_iter": max_iter} if max_iter else {}))
    ctx = pa.DeviceContext(0)
    a = ctx.generate(n, t, 42)
    t0 = time.perf_counter()
    s = pa.Solver(ctx, pa.PicardConfig(random_state=42, want_sources=False, **kw))
    t_setup = time.perf_counter() - t0
    ctx.kernel_breakdown(reset=True)
    t1 = time.perf_counter()
    done = False
    while not done:
        done = s.step()
    t_iter = time.perf_counter() - t1
    r = s.finish()
    out = {"config": name, "n": n, "t": t, **{k: v for k, v in c["kw"].items()},
           "setup_s": t_setup, "iterations_s": t_iter, "n_iterations": r.n_iterations, "converged": r.converged,
           "gradient_norm": r.gradient_norm, "passes": r.n_evaluations,
           "samples_per_s_per_iter": t * r.n_iterations / t_iter,
           "amari": pa.utils.amari_distance(r.full_unmixing(), a),
           "kernels": {k: v for k, v in ctx.kernel_breakdown().items()}}
    s.close()
    if oracle:
        from oracle import picard_oracle as po
        x = ctx.download()
        t2 = time.perf_counter()
        ro = po.fit_with_config(x, po.PicardConfig(random_state=42, **c["kw"]),
                                w_init_random=None)
        out["oracle_s"] = time.perf_counter() - t2
        out["oracle_amari"] = po.amari_distance(ro.full_unmixing(), a)
        out["oracle_n_iterations"] = ro.n_iterations
    ctx.close()
    print(json.dumps(out), flush=True)


def dump_maps_at_exit(path):
    """--maps=PATH: write /proc/self/maps when the interpreter finalises (to map the PCs of
    a crash in exit() to libraries and offsets afterwards)."""
    import atexit

    def dump():
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())
    atexit.register(dump)


if __name__ == "__main__":
    for a in sys.argv[1:]:
        if a.startswith("--maps="):
            dump_maps_at_exit(a.split("=", 1)[1])
    want_oracle = "--oracle" in sys.argv
    mi = [int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--max-iter=")]
    for name in [a for a in sys.argv[1:] if not a.startswith("--")]:
        run(name, want_oracle, mi[0] if mi else None)

