"""Multi-process (world_size 2, gloo, CPU) coverage of the T-sharded path.

The device path shards T in contiguous blocks (DeviceCtx::shard_t0/shard_n)
and sums every per-pass statistic with ONE all-reduce (RCCL on the GPU).
Here each rank evaluates its shard's sums (the oracle stands in for the HIP
pass), the sums are all-reduced over gloo, and the C++ host driver runs
replicated on every rank — exactly the structure of bench.py --gpus N.
Checks: shard sums add up to the full-data statistics, the replicated host
drivers stay in lockstep (bit-identical W on both ranks), and the result
matches the single-process fit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def shard(n_total, world, rank):
    base, rem = divmod(n_total, world)
    t0 = rank * base + min(rank, rem)
    return t0, base + (1 if rank < rem else 0)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import picard_ica_amd as pa
        from oracle import datagen, picard_oracle as po
        nf, T = 8, 10001
        x_full, s, a = datagen.generate_data(nf, T, 42)
        t0, nl = shard(T, world, rank)
        x = np.ascontiguousarray(x_full[:, t0:t0 + nl])

        def allreduce(v):
            t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64).reshape(-1).copy())
            dist.all_reduce(t)
            return t.numpy().reshape(np.shape(v))

        def ev(w, mu, d, need_h):
            st = po.pass_stats(w, mu, x, po.Density(["tanh", "exp", "cube"][d.kind], d.alpha), need_h)
            return {k: allreduce(v) for k, v in st.items()}

        def gram(mu):
            xc = x - mu[:, None] if mu is not None else x
            return allreduce(xc @ xc.T)

        def sources(w, mu):
            return w @ (x - mu[:, None] if mu is not None else x)

        # 1) shard sums == full sums
        w = np.random.default_rng(0).normal(size=(nf, nf))
        mu = x_full.mean(axis=1)
        full = po.pass_stats(w, mu, x_full, po.Density(), True)
        got = ev(w, mu, pa.DensityType.tanh(), True)
        ok_sums = all(np.max(np.abs(got[k] - full[k])) <= 1e-12 * np.max(np.abs(full[k])) for k in full)

        # 2) replicated host driver over the sharded evaluator (sources: local shard only)
        cfg = pa.PicardConfig(w_init=np.eye(nf))

        # n_samples is the GLOBAL T; sources return this rank's shard (padded for the callback shape)
        r = pa.fit_with_host_evaluator(nf, T, cfg, rowsum=lambda: allreduce(x.sum(axis=1)), gram=gram, eval=ev,
                                       sources=lambda w, mu: np.pad(sources(w, mu), ((0, 0), (0, T - nl))))
        q.put((rank, ok_sums, r.unmixing, r.n_iterations, r.converged,
               pa.utils.amari_distance(r.full_unmixing(), a)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_sharded_fit():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, ok0, w0, it0, c0, am0), (_, ok1, w1, it1, c1, am1) = res
    assert ok0 and ok1
    assert np.array_equal(w0, w1) and it0 == it1 and c0 and c1  # lockstep across ranks
    # single-process oracle on the whole data
    import sys
    sys.path.insert(0, ROOT)
    from oracle import datagen, picard_oracle as po
    x, s, a = datagen.generate_data(8, 10001, 42)
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8)))
    assert abs(it0 - ro.n_iterations) <= 2
    assert abs(am0 - po.amari_distance(ro.full_unmixing(), a)) <= 1e-6


def test_shard_partition_covers_all():
    for T in [1, 7, 10001, 10 ** 8]:
        for world in [1, 2, 3, 8]:
            parts = [shard(T, world, r) for r in range(world)]
            assert parts[0][0] == 0
            assert sum(n for _, n in parts) == T
            for (t0, n), (t1, _) in zip(parts, parts[1:]):
                assert t0 + n == t1


def _rank_report_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        # synthetic per-step timings of a 5-step window: rank r has a host spike of 10·(r + 1) ms
        host = [1.0, 1.2, 10.0 * (rank + 1), 0.9, 1.1]
        step = [20.0 + h for h in host]
        ev = [19.0] * 5
        ranks = bench.gather_ranks(dist, bench.rank_entry(rank, 0.1 + rank, step, host, ev, 3.5 * (rank + 1), 11))
        q.put((rank, ranks))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_rank_report_gathers_every_rank():
    """bench.py's per-rank report: rank_entry summarises a rank's window
    and gather_ranks all-gathers the entries over the process group (gloo here, as bench.py
    does beside RCCL), so rank 0's JSON line holds every rank's window, host ms per step
    (mean / p90 / max), ms inside all-reduces and their count."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rank_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]  # every rank holds the same list
    ranks = res[0]
    assert [e["rank"] for e in ranks] == [0, 1]
    for r, e in enumerate(ranks):
        assert e["window_s"] == pytest.approx(0.1 + r) and e["steps"] == 5
        assert e["host_ms_max"] == pytest.approx(10.0 * (r + 1))
        assert e["host_ms_mean"] == pytest.approx((1.0 + 1.2 + 10.0 * (r + 1) + 0.9 + 1.1) / 5)
        assert e["host_ms_p90"] <= e["host_ms_max"]
        assert e["allreduce_ms"] == pytest.approx(3.5 * (r + 1)) and e["allreduces"] == 11
        assert e["allreduce_ms_per_step"] == pytest.approx(3.5 * (r + 1) / 5)
        assert e["eval_ms_per_step"] == pytest.approx(19.0)


def test_bench_single_process_report():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    e = bench.rank_entry(0, 1.0, [], [], [], 0.0, 0)
    assert bench.gather_ranks(None, e) == [e] and e["steps"] == 0
