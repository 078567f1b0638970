"""Link sharding of one sample (secondary): the accumulate / M-step split, the
link blocks, the global degree and the world_size-2 all-reduce over gloo, on CPU with the
oracle standing in for the GPU engine (tests/oracle_engine.py)."""
import contextlib
import io
import os
import random

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import c_oracle
from oracle_engine import OracleShardEngine
from trigenicinteractionpredictor_amd.launch import free_port
from trigenicinteractionpredictor_amd.linkshard import LinkShardedEM, shard_links, train_degree
from trigenicinteractionpredictor_amd.model import Model
from trigenicinteractionpredictor_amd.restarts import run_samples

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TINY = os.path.join(GOLD, "tiny")


def _host(d=TINY, test="test.dat"):
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(os.path.join(d, "train.dat"), os.path.join(d, test))
    return m


def _init(m, K, seed):
    random.seed(seed)
    m.initialize_parameters(K)
    return np.array(m._theta), np.array(m._pr)


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 3), (400, 8), (5, 1)])
def test_link_blocks_partition_in_order(n, world):
    blocks = [shard_links(n, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
    assert max(h - l for l, h in blocks) - min(h - l for l, h in blocks) <= 1


def test_train_degree_is_reference_counter():
    ids = np.array([[0, 0, 1], [1, 2, 3]], np.int32)    # a repeated gene counts twice (:986-994)
    np.testing.assert_array_equal(train_degree(ids, 5), [2, 2, 1, 1, 0])


@pytest.mark.parametrize("parts", [1, 2, 3])
def test_partial_sums_over_any_partition_are_the_reference_step(parts):
    from oracle import shard_oracle
    m = _host()
    th, pr = _init(m, 3, 4)
    ids, counts = c_oracle.links_to_arrays(m.links)
    nth = np.zeros_like(th)
    S = np.zeros((2, 27))
    for r in range(parts):
        lo, hi = shard_links(ids.shape[0], parts, r)
        n, s = shard_oracle.accumulate(ids[lo:hi], counts[lo:hi], th, pr)
        nth += n
        S += s
    th1, pr1 = shard_oracle.mstep(th, pr, nth, S, train_degree(ids, m.P))
    th_o, pr_o = c_oracle.make_iteration(ids, counts, th, pr)
    np.testing.assert_allclose(th1, th_o, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(pr1, pr_o, rtol=1e-12, atol=1e-300)


def test_zero_degree_raises_like_reference():
    from oracle import shard_oracle
    with pytest.raises(ZeroDivisionError):
        shard_oracle.mstep(np.ones((2, 2)), np.ones((2, 2, 2, 2)), np.ones((2, 2)),
                           np.ones((2, 8)), np.array([1, 0]))


def _run(m, K, seed, iters, world=1):
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    th, pr = _init(m, K, seed)
    em = LinkShardedEM(OracleShardEngine(K, m.P), ids, counts, tids, tcounts)
    em.upload(th[None], pr[None])
    em.iterate(iters)
    t, p = em.download()
    return t[0], p[0], em.loglik(0)[0], em.loglik(1)[0], (ids, counts, tids, tcounts, th, pr)


def test_single_rank_is_the_reference_iteration():
    m = _host()
    t, p, L, LT, (ids, counts, tids, tcounts, th, pr) = _run(m, 3, 9, 4)
    for _ in range(4):
        th, pr = c_oracle.make_iteration(ids, counts, th, pr)
    np.testing.assert_allclose(t, th, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(p, pr, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(L, c_oracle.loglik(ids, counts, th, pr), rtol=1e-12)
    np.testing.assert_allclose(LT, c_oracle.loglik(tids, tcounts, th, pr), rtol=1e-12)


def _worker(rank, world, port, queue):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _host()
    t, p, L, LT, _ = _run(m, 3, 9, 4)
    # the restart driver's convergence loop runs the sharded sample unchanged
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    th, pr = _init(m, 2, 5)
    em = LinkShardedEM(OracleShardEngine(2, m.P), ids, counts, tids, tcounts)
    res = run_samples(em, [0], [th], [pr], iterations=30, fcheck=3, bcheck=4)[0]
    queue.put((rank, t, p, L, LT, (res.iterations, res.converged, res.loglik)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_allreduce_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {g[0]: g[1:] for g in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    m = _host()
    t, p, L, LT, _ = _run(m, 3, 9, 4)
    for r in (0, 1):
        gt, gp, gL, gLT, conv = got[r]
        np.testing.assert_allclose(gt, t, rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(gp, p, rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose([gL, gLT], [L, LT], rtol=1e-12)
    # both ranks hold bitwise identical parameters after every all-reduce
    np.testing.assert_array_equal(got[0][0], got[1][0])
    np.testing.assert_array_equal(got[0][1], got[1][1])
    th, pr = _init(m, 2, 5)
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    single = run_samples(LinkShardedEM(OracleShardEngine(2, m.P), ids, counts, tids, tcounts),
                         [0], [th], [pr], iterations=30, fcheck=3, bcheck=4)[0]
    assert got[0][4][:2] == (single.iterations, single.converged)
    np.testing.assert_allclose(got[0][4][2], single.loglik, rtol=1e-12)


def _active_worker(rank, world, port, queue):
    """Three samples; after 3 iterations the active prefix shrinks to 2 (the restart pool retiring
    slot 2): the collective then reduces the active slots only, so slot 2's stale local sums are
    never summed again (they grew by the world size each iteration)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _host()
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    ths, prs = zip(*[_init(m, 3, s) for s in (1, 2, 3)])
    em = LinkShardedEM(OracleShardEngine(3, m.P, B=3), ids, counts, tids, tcounts)
    em.upload(np.stack(ths), np.stack(prs))
    em.iterate(3)
    em.set_active(2)
    stale = em.nth[2].clone(), em.S[2].clone()
    em.iterate(40)
    t, p = em.download()
    queue.put((rank, t[:2], p[:2], bool((em.nth[2] == stale[0]).all() and (em.S[2] == stale[1]).all())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shrunken_active_prefix_reduces_active_slots_only():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_active_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {g[0]: g[1:] for g in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    m = _host()
    ids, counts = c_oracle.links_to_arrays(m.links)
    for r in (0, 1):
        t, p, untouched = got[r]
        assert untouched
        for b, s in enumerate((1, 2)):
            th, pr = _init(m, 3, s)
            for _ in range(43):
                th, pr = c_oracle.make_iteration(ids, counts, th, pr)
            np.testing.assert_allclose(t[b], th, rtol=1e-11, atol=1e-300)
            np.testing.assert_allclose(p[b], pr, rtol=1e-11, atol=1e-300)
