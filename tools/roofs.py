"""Empirical roofs on the box (SURVEY.md §8(d) "measure empirical roofs"): HBM streaming read
(torch.sum over 16 GiB of fp64), HBM copy (read + write), and the library fp64 GEMM
(torch.matmul → rocBLAS / hipBLASLt dgemm) square and in the pass's shapes at C3 per 1/8
shard (Y = W·X: 128×128 · 128×T; Gram ψ·Yᵀ: 128×T · T×128). HIP-event timing, best of reps.
Usage: python tools/roofs.py"""
import json

import torch


def timed(f, reps=10):
    f()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best  # ms


dev = torch.device("cuda:0")
out = {}
n = (16 << 30) // 8
x = torch.ones(n, dtype=torch.float64, device=dev)
ms = timed(lambda: x.sum())
out["hbm_read_gbs"] = n * 8 / ms / 1e6
y = torch.empty_like(x)
ms = timed(lambda: y.copy_(x))
out["hbm_copy_gbs"] = 2 * n * 8 / ms / 1e6
del x, y
for m in (4096, 8192):
    a = torch.randn(m, m, dtype=torch.float64, device=dev)
    b = torch.randn(m, m, dtype=torch.float64, device=dev)
    ms = timed(lambda: a @ b, reps=5)
    out[f"dgemm_{m}_tflops"] = 2.0 * m ** 3 / ms / 1e9
    del a, b
t = 12_500_000
w = torch.randn(128, 128, dtype=torch.float64, device=dev)
xs = torch.randn(128, t, dtype=torch.float64, device=dev)
ms = timed(lambda: w @ xs, reps=5)
out["dgemm_WX_128x128x1.25e7_tflops"] = 2.0 * 128 * 128 * t / ms / 1e9
out["dgemm_WX_ms"] = ms
ms = timed(lambda: xs @ xs.T, reps=5)
out["dgemm_gram_128xTx128_tflops"] = 2.0 * 128 * 128 * t / ms / 1e9
out["dgemm_gram_ms"] = ms
print(json.dumps(out, indent=1))
