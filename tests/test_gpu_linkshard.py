"""Link-sharded iteration on the GPU (mmsbm_accumulate / mmsbm_mstep, SURVEY.md §8e secondary)
against the C oracle: one rank holding every link, and two contexts each holding one block of
the links with the global degree, their accumulators summed like the all-reduce does."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-9
ATOL = 1e-300


def _fold(tmp_path, P, E, seed, **kw):
    from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
    tr, te = str(tmp_path / "train.dat"), str(tmp_path / "test.dat")
    write_fold(FoldSpec(P=P, E=E, seed=seed, **kw), tr, te)
    return tr, te


def _setup(tmp_path, K, P, E, seed):
    import contextlib
    import io
    from trigenicinteractionpredictor_amd import Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, P, E, seed, multi_frac=0.05, both_frac=0.02)
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(tr, te)
    random.seed(seed)
    m.initialize_parameters(K)
    ids, counts = links_to_arrays(m.links)
    tids, tcounts = links_to_arrays(m.test_links)
    return m, ids, counts, tids, tcounts, np.array(m._theta), np.array(m._pr)


def _oracle(ids, counts, th, pr, iters):
    from oracle import c_oracle
    for _ in range(iters):
        th, pr = c_oracle.make_iteration(ids, counts, th, pr)
    return th, pr


@pytest.mark.parametrize("K,P,E,iters", [(10, 1500, 90000, 3), (11, 300, 4000, 2),
                                         (13, 200, 2000, 2), (3, 100, 800, 4)])
def test_single_rank_link_sharded_matches_oracle(tmp_path, K, P, E, iters):
    from trigenicinteractionpredictor_amd import EMEngine
    from trigenicinteractionpredictor_amd.linkshard import LinkShardedEM
    from oracle import c_oracle
    m, ids, counts, tids, tcounts, th, pr = _setup(tmp_path, K, P, E, K + 7)
    em = LinkShardedEM(EMEngine(K, m.P), ids, counts, tids, tcounts)
    em.upload(th[None], pr[None])
    em.iterate(iters)
    t, p = em.download()
    th_o, pr_o = _oracle(ids, counts, th, pr, iters)
    np.testing.assert_allclose(t[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(p[0], pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(em.loglik(0)[0], c_oracle.loglik(ids, counts, th_o, pr_o), rtol=RTOL)
    np.testing.assert_allclose(em.loglik(1)[0], c_oracle.loglik(tids, tcounts, th_o, pr_o), rtol=RTOL)


@pytest.mark.parametrize("K,parts", [(10, 2), (4, 3), (16, 2)])
def test_link_blocks_with_summed_accumulators_match_oracle(tmp_path, K, parts):
    """`parts` contexts on one GPU, each with one block of the train links and the global
    degree; the accumulators are summed (what the all-reduce does) and every context applies
    the M-step.  All contexts end bitwise identical and equal to the oracle."""
    import torch
    from trigenicinteractionpredictor_amd import EMEngine
    from trigenicinteractionpredictor_amd.linkshard import shard_links, train_degree
    m, ids, counts, tids, tcounts, th, pr = _setup(tmp_path, K, 400, 6000, K + 30)
    deg = train_degree(ids, m.P)
    engs = []
    for r in range(parts):
        lo, hi = shard_links(ids.shape[0], parts, r)
        e = EMEngine(K, m.P)
        e.set_links(0, ids[lo:hi], counts[lo:hi], deg=deg)
        e.upload(th[None], pr[None])
        engs.append(e)
    bufs = [(torch.zeros((1, m.P, K), dtype=torch.float64, device=e.device),
             torch.zeros((1, 2, K ** 3), dtype=torch.float64, device=e.device)) for e in engs]
    for _ in range(3):
        for e, (n, s) in zip(engs, bufs):
            e.accumulate(n, s)
        nsum = sum(b[0] for b in bufs)
        ssum = sum(b[1] for b in bufs)
        for e in engs:
            e.mstep(nsum, ssum)
    th_o, pr_o = _oracle(ids, counts, th, pr, 3)
    t0, p0 = engs[0].download()
    np.testing.assert_allclose(t0[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(p0[0], pr_o, rtol=RTOL, atol=ATOL)
    for e in engs[1:]:
        t, p = e.download()
        np.testing.assert_array_equal(t, t0)
        np.testing.assert_array_equal(p, p0)


def test_link_sharded_zero_degree_raises(tmp_path):
    from trigenicinteractionpredictor_amd import EMEngine
    from trigenicinteractionpredictor_amd.linkshard import LinkShardedEM
    m, ids, counts, tids, tcounts, th, pr = _setup(tmp_path, 3, 100, 800, 5)
    # a gene id beyond every train link: global degree 0 -> ZeroDivisionError like :1018
    eng = EMEngine(3, m.P + 1)
    em = LinkShardedEM(eng, ids, counts, tids, tcounts)
    em.upload(np.vstack([th, th[:1]])[None], pr[None])
    with pytest.raises(ZeroDivisionError):
        em.iterate(1)
