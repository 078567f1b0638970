"""Restart sharding: sample ids, RNG stream, the reference driver's
convergence rule, and the world_size-2 gather over gloo — all on CPU with the oracle
standing in for the GPU engine."""
import contextlib
import io
import math
import os
import random

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.mmsbm_oracle import OracleModel
from oracle_engine import OracleEngine
from trigenicinteractionpredictor_amd.launch import free_port
from trigenicinteractionpredictor_amd.model import Model
from trigenicinteractionpredictor_amd.restarts import (fixed_run, gather_rows, init_samples,
                                                       replay_check, result_rows, rows_digest,
                                                       run_restarts, run_samples, shard_samples)

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny")
TRAIN, TEST = os.path.join(GOLD, "train.dat"), os.path.join(GOLD, "test.dat")


def _host():
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(TRAIN, TEST)
    return m


@pytest.mark.parametrize("n,world", [(1, 1), (5, 2), (64, 8), (3, 4), (10, 3)])
def test_shards_cover_each_sample_once(n, world):
    ids = [s for r in range(world) for s in shard_samples(n, world, r)]
    assert ids == list(range(n))


def test_init_stream_matches_sequential_reference_loop():
    m = _host()
    th, pr = init_samples(m, 3, [2, 3], seed=11)
    ref = OracleModel()
    ref.get_traintest(TRAIN, TEST)
    random.seed(11)
    for s in range(4):
        ref.initialize_parameters(3)
        if s >= 2:
            np.testing.assert_array_equal(th[s - 2], np.array(ref.theta))
            np.testing.assert_array_equal(pr[s - 2], np.array(ref.pr))


def _reference_driver(K, seed, n_samples, iterations, f, b):
    """The reference __main__ loop (:1253-1279) on the oracle, one sample after another."""
    m = OracleModel()
    m.get_traintest(TRAIN, TEST)
    random.seed(seed)
    out = []
    for s in range(n_samples):
        m.initialize_parameters(K)
        like0 = m.compute_likelihood()
        done = None
        for it in range(iterations):
            m.make_iteration()
            if it % f == 0 and it > b:
                like = m.compute_likelihood()
                if math.fabs((like - like0) / like0) < 0.01:
                    done = (s, it + 1, True, like)
                    break
                like0 = like
        if done is None:
            done = (s, iterations, False, m.compute_likelihood())
        out.append(done)
    return out


def test_batched_driver_matches_reference_loop():
    K, seed, n, iters, f, b = 2, 5, 3, 40, 3, 4
    ref = _reference_driver(K, seed, n, iters, f, b)
    m = _host()
    th, pr = init_samples(m, K, list(range(n)), seed)
    res = run_samples(OracleEngine(m.links, m.test_links, B=n), list(range(n)), th, pr, iters, f, b)
    for r, (s, it, conv, like) in zip(res, ref):
        assert (r.sample, r.iterations, r.converged) == (s, it, conv)
        assert r.loglik == like


def _worker(rank, world, port, queue):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _host()
    res = run_restarts(m, 2, 5, seed=5, iterations=30, fcheck=3, bcheck=4,
                       engine_factory=lambda B: OracleEngine(m.links, m.test_links, B=B))
    queue.put((rank, [(r.sample, r.iterations, r.converged, r.loglik, r.heldout) for r in res]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    m = _host()
    single = run_restarts(m, 2, 5, seed=5, iterations=30, fcheck=3, bcheck=4,
                          engine_factory=lambda B: OracleEngine(m.links, m.test_links, B=B))
    want = [(r.sample, r.iterations, r.converged, r.loglik, r.heldout) for r in single]
    assert got[0] == want and got[1] == want


def _fixed_worker(rank, world, port, queue):
    """bench.py's N>1 path on the oracle: this rank's block of samples for a fixed number of
    iterations, one all-gather of (sample, L), and rank 0's one-batch replay of all of them."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _host()
    ids = shard_samples(4, world, rank)
    th, pr = init_samples(m, 2, ids, seed=9)
    L = fixed_run(OracleEngine(m.links, m.test_links), th, pr, 6, chunks=(1, 2))
    rows = gather_rows(result_rows(ids, L), 4)
    check = None
    if rank == 0:
        check = replay_check(rows, m, 2, 9, 6, lambda B: OracleEngine(m.links, m.test_links))
    queue.put((rank, rows_digest(rows), check))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_fixed_run_digest_equals_one_rank_and_replay():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_fixed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (d, c) for r, d, c in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    m = _host()
    th, pr = init_samples(m, 2, list(range(4)), seed=9)
    one = rows_digest(result_rows(range(4), fixed_run(OracleEngine(m.links, m.test_links), th, pr, 6)))
    assert got[0][0] == got[1][0] == one
    check = got[0][1]
    assert check["bitwise_equal"] and check["samples"] == 4
    assert check["digest"] == check["replay_digest"] == one
