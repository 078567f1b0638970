"""BASELINE.json's five configurations at their real workload on the GPU.

The reference's EM step is `Model.make_iteration` (src/TrigenicInteractionPredictor.py:984-1043),
its likelihood `compute_likelihood` (:952-974) and its test-set prediction `do_prediction`
(:530-547).  Configs 1-4 are checked against the C oracle (oracle/mmsbm_oracle.c, pinned
bit-exact to the reference) on the same seeded inputs; config 5 (10M links, K=30) is beyond
any CPU check, so it is checked through size-independent properties plus one oracle-sized
block.  Tolerance: rtol 1e-9 on theta, p, L (north star: 1e-6 relative), 1e-12 where the two
sides sum the same terms on the GPU.
"""
import contextlib
import io
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-9
ATOL = 1e-300


def _model(tmp_path, spec):
    from trigenicinteractionpredictor_amd import Model
    from trigenicinteractionpredictor_amd.data import write_fold
    tr, te = str(tmp_path / "train.dat"), str(tmp_path / "test.dat")
    write_fold(spec, tr, te)
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(tr, te)
    return m


def _samples(m, K, B, seed):
    random.seed(seed)
    th, pr = [], []
    for _ in range(B):
        m.initialize_parameters(K)
        th.append(np.array(m._theta))
        pr.append(np.array(m._pr))
    return th, pr


def _engine(m, K, B, th, pr):
    from trigenicinteractionpredictor_amd import EMEngine
    eng = EMEngine(K, m.P, B=B)
    eng.set_links(0, *m._link_arrays(0))
    eng.set_links(1, *m._link_arrays(1))
    eng.upload(np.stack(th), np.stack(pr))
    return eng


def _oracle(ids, counts, th, pr, iters):
    from oracle import c_oracle
    for _ in range(iters):
        th, pr = c_oracle.make_iteration(ids, counts, th, pr)
    return th, pr


def test_config1_fold0_K2_50_iterations(tmp_path):
    """Config 1: fold0 stand-in, K=2, 1 sample, 50 iterations."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd.data import FOLD0
    m = _model(tmp_path, FOLD0)
    th, pr = _samples(m, 2, 1, 1)
    eng = _engine(m, 2, 1, th, pr)
    eng.iterate(50)
    t, p = eng.download()
    ids, counts = m._link_arrays(0)
    tids, tcounts = m._link_arrays(1)
    th_o, pr_o = _oracle(ids, counts, th[0], pr[0], 50)
    np.testing.assert_allclose(t[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(p[0], pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(eng.loglik(0)[0], c_oracle.loglik(ids, counts, th_o, pr_o), rtol=RTOL)
    np.testing.assert_allclose(eng.loglik(1)[0], c_oracle.loglik(tids, tcounts, th_o, pr_o), rtol=RTOL)


def _oracle_snapshots(ids, counts, th, pr, at):
    """The C oracle's (theta, p) after each iteration count in `at` (ascending)."""
    from oracle import c_oracle
    out, done = [], 0
    for n in at:
        for _ in range(n - done):
            th, pr = c_oracle.make_iteration(ids, counts, th, pr)
        done = n
        out.append((th, pr))
    return out


def _parallel(fn, items):
    """fn over items on host threads (the C oracle releases the GIL inside its ctypes calls)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, len(items))) as ex:
        return list(ex.map(fn, items))


def test_config2_fold0_K10_at_1_5_25_iterations(tmp_path):
    """Config 2 (the headline): fold0 stand-in, K=10, 1 sample, against the C oracle after 1, 5
    and 25 iterations: theta, p and the train / held-out likelihoods."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd.data import FOLD0
    m = _model(tmp_path, FOLD0)
    th, pr = _samples(m, 10, 1, 11)
    eng = _engine(m, 10, 1, th, pr)
    ids, counts = m._link_arrays(0)
    tids, tcounts = m._link_arrays(1)
    want = _oracle_snapshots(ids, counts, th[0], pr[0], (1, 5, 25))
    done = 0
    for n, (th_o, pr_o) in zip((1, 5, 25), want):
        eng.iterate(n - done)
        done = n
        t, p = eng.download()
        np.testing.assert_allclose(t[0], th_o, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(p[0], pr_o, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(eng.loglik(0)[0], c_oracle.loglik(ids, counts, th_o, pr_o), rtol=RTOL)
        np.testing.assert_allclose(eng.loglik(1)[0], c_oracle.loglik(tids, tcounts, th_o, pr_o), rtol=RTOL)


def test_config3_fold0_K20_batch8(tmp_path):
    """Config 3's per-GPU share: fold0 stand-in, K=20, 8 samples in one batched engine; EVERY
    sample against the C oracle after 2 and after 5 iterations (theta, p, train L)."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd.data import FOLD0
    m = _model(tmp_path, FOLD0)
    th, pr = _samples(m, 20, 8, 3)
    eng = _engine(m, 20, 8, th, pr)
    ids, counts = m._link_arrays(0)
    want = _parallel(lambda s: _oracle_snapshots(ids, counts, th[s], pr[s], (2, 5)), list(range(8)))
    done = 0
    for k, n in enumerate((2, 5)):
        eng.iterate(n - done)
        done = n
        t, p = eng.download()
        L = eng.loglik(0)
        assert np.isfinite(t).all() and np.isfinite(p).all()
        Lo = _parallel(lambda s: c_oracle.loglik(ids, counts, *want[s][k]), list(range(8)))
        for s in range(8):
            th_o, pr_o = want[s][k]
            np.testing.assert_allclose(t[s], th_o, rtol=RTOL, atol=ATOL)
            np.testing.assert_allclose(p[s], pr_o, rtol=RTOL, atol=ATOL)
            np.testing.assert_allclose(L[s], Lo[s], rtol=RTOL)


def test_config4_all_train_multicount_K10_batch8(tmp_path):
    """Config 4 stand-in ("full ORIGINAL_DATASET"): E=90k links, all train, 10 % of the links
    with repeated lines (n_r in 2..4, the `get_input` count path :301-309) and 2 % with both
    ratings, K=10, 8 samples batched, 2 iterations, every sample against the oracle."""
    from trigenicinteractionpredictor_amd.data import FoldSpec
    m = _model(tmp_path, FoldSpec(P=1500, E=90000, seed=17, test_frac=0.0, multi_frac=0.10,
                                  both_frac=0.02))
    ids, counts = m._link_arrays(0)
    assert (counts.max(axis=1) > 1).mean() > 0.05 and ((counts > 0).sum(axis=1) == 2).mean() > 0.01
    th, pr = _samples(m, 10, 8, 4)
    eng = _engine(m, 10, 8, th, pr)
    eng.iterate(2)
    t, p = eng.download()
    for s in range(8):
        th_o, pr_o = _oracle(ids, counts, th[s], pr[s], 2)
        np.testing.assert_allclose(t[s], th_o, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(p[s], pr_o, rtol=RTOL, atol=ATOL)
    assert eng.loglik(1).tolist() == [0.0] * 8        # empty test set


@pytest.mark.parametrize("K", [13, 20, 30, 32])
def test_prediction_large_K(tmp_path, K):
    """`do_prediction` (:530-547) through the batched prediction kernel at K > 10."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd.data import FoldSpec
    m = _model(tmp_path, FoldSpec(P=120, E=900, seed=K))
    th, pr = _samples(m, K, 2, K)
    eng = _engine(m, K, 2, th, pr)
    eng.iterate(1)
    t, p = eng.download()
    tids, _ = m._link_arrays(1)
    got = eng.predict(tids)
    for s in range(2):
        np.testing.assert_allclose(got[s], c_oracle.predict(tids, t[s], p[s]), rtol=RTOL, atol=ATOL)


# ------------------------------------------------------------------ config 5 (10M links, K=30)
C5_K = 30


@pytest.fixture(scope="module")
def c5():
    from trigenicinteractionpredictor_amd.data import FoldSpec, synthetic_links
    spec = FoldSpec(P=50000, E=10_000_000, seed=7, test_frac=0.0)
    ids, counts = synthetic_links(spec)
    rng = np.random.default_rng(5)
    th = rng.random((spec.P, C5_K))
    th /= th.sum(axis=1, keepdims=True)
    pr = rng.random((C5_K, C5_K, C5_K, 2))
    pr /= pr.sum(axis=-1, keepdims=True)
    return spec.P, ids, counts, th, pr


def _c5_engine(c5, lo=0, hi=None, deg=None):
    from trigenicinteractionpredictor_amd import EMEngine
    P, ids, counts, th, pr = c5
    hi = ids.shape[0] if hi is None else hi
    eng = EMEngine(C5_K, P, B=1)
    eng.set_links(0, ids[lo:hi], counts[lo:hi], deg=deg)
    eng.upload(th[None], pr[None])
    return eng


def test_config5_full_size_properties(c5):
    """Config 5 at full size on one GPU, 3 iterations: the train likelihood never decreases (EM),
    every theta / p value is finite, and p sums over r to 1 - eps / (eps + sum_r npr) with
    npr = p S from the same iterate's accumulators (:1021-1028)."""
    import torch
    P, ids, counts, th, pr = c5
    eng = _c5_engine(c5)
    nth = torch.zeros((1, P, C5_K), dtype=torch.float64, device=eng.device)
    S = torch.zeros((1, 2, C5_K ** 3), dtype=torch.float64, device=eng.device)
    eng.accumulate(nth, S)
    p_before = eng.pr.clone()
    L = [float(eng.loglik(0)[0])]
    eng.iterate(1)
    npr = p_before * S                                # [1][R][K^3]
    want = 1.0 - 1e-10 / (1e-10 + npr.sum(dim=1))
    np.testing.assert_allclose(eng.pr.sum(dim=1).cpu().numpy(), want.cpu().numpy(), rtol=1e-12)
    for _ in range(2):
        L.append(float(eng.loglik(0)[0]))
        eng.iterate(1)
    L.append(float(eng.loglik(0)[0]))
    assert all(b >= a - 1e-9 * abs(a) for a, b in zip(L, L[1:])), L
    t, p = eng.download()
    assert np.isfinite(t).all() and np.isfinite(p).all()
    eng.close()


def test_config5_link_blocks_sum_to_the_full_iteration(c5):
    """The accumulators of 8 link blocks (the link-sharded split, each block with the global
    degree) summed and applied by the M-step equal one full iteration over all 10M links."""
    import torch
    from trigenicinteractionpredictor_amd.linkshard import shard_links, train_degree
    P, ids, counts, th, pr = c5
    deg = train_degree(ids, P)
    nsum = torch.zeros((1, P, C5_K), dtype=torch.float64, device="cuda")
    ssum = torch.zeros((1, 2, C5_K ** 3), dtype=torch.float64, device="cuda")
    for r in range(8):
        lo, hi = shard_links(ids.shape[0], 8, r)
        e = _c5_engine(c5, lo, hi, deg=deg)
        n = torch.zeros_like(nsum)
        s = torch.zeros_like(ssum)
        e.accumulate(n, s)
        nsum += n
        ssum += s
        e.close()
        del e
    full = _c5_engine(c5)
    full.iterate(1)
    t_full, p_full = full.download()
    full.upload(th[None], pr[None])
    full.mstep(nsum, ssum)
    t_sh, p_sh = full.download()
    np.testing.assert_allclose(t_sh, t_full, rtol=1e-12, atol=ATOL)
    np.testing.assert_allclose(p_sh, p_full, rtol=1e-12, atol=ATOL)
    full.close()


def test_config5_block_against_oracle(c5):
    """One 5,000-link block of the 10M set at K=30 (realistic gene ids up to 50k, p staged in
    a-chunks): its accumulators against the numpy restatement of :986-1012."""
    import torch
    from oracle import shard_oracle
    from trigenicinteractionpredictor_amd.linkshard import train_degree
    P, ids, counts, th, pr = c5
    lo, hi = 4_000_000, 4_005_000
    deg = train_degree(ids, P)
    e = _c5_engine(c5, lo, hi, deg=deg)
    n = torch.zeros((1, P, C5_K), dtype=torch.float64, device=e.device)
    s = torch.zeros((1, 2, C5_K ** 3), dtype=torch.float64, device=e.device)
    e.accumulate(n, s)
    n_o, s_o = shard_oracle.accumulate(ids[lo:hi], counts[lo:hi], th, pr)
    np.testing.assert_allclose(n[0].cpu().numpy(), n_o, rtol=RTOL, atol=1e-300)
    np.testing.assert_allclose(s[0].cpu().numpy(), s_o, rtol=RTOL, atol=1e-300)
    e.close()


def test_config5_subfold_full_iteration_against_oracle(c5):
    """A 60,000-link sub-fold of the 10M set (links 3,000,000-3,060,000) as a fold of its own:
    its genes renumbered densely (ascending ids), its own degree, one full EM iteration at
    K=30 (theta, p, train L before and after) against the C oracle."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd import EMEngine
    P, ids, counts, th, pr = c5
    sub = ids[3_000_000:3_060_000]
    genes, inv = np.unique(sub.ravel(), return_inverse=True)
    sids = np.ascontiguousarray(inv.reshape(-1, 3).astype(np.int32))
    scounts = np.ascontiguousarray(counts[3_000_000:3_060_000])
    sth = np.ascontiguousarray(th[genes])
    eng = EMEngine(C5_K, genes.size, B=1)
    eng.set_links(0, sids, scounts)
    eng.upload(sth[None], pr[None])
    L0 = eng.loglik(0)[0]
    eng.iterate(1)
    t, p = eng.download()
    th_o, pr_o = c_oracle.make_iteration(sids, scounts, sth, pr)
    np.testing.assert_allclose(L0, c_oracle.loglik(sids, scounts, sth, pr), rtol=RTOL)
    np.testing.assert_allclose(t[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(p[0], pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(eng.loglik(0)[0], c_oracle.loglik(sids, scounts, th_o, pr_o), rtol=RTOL)
    eng.close()


def test_config5_full_iteration_theta_rows_against_oracle(c5):
    """Config 5 at full size (10M links, 50k genes, K=30): after ONE full GPU iteration, theta'
    of 200 genes against the C oracle.  The genes: the 20 of highest degree
    (the longest pivot runs, split over units, waves and workgroups, their partial rows merged)
    and 180 drawn at random.  The oracle accumulates :986-1012 over every link holding one of them
    (16 link blocks on threads, summed in block order) and divides by the degree over ALL links
    (:1016-1018), which is exactly theta' for those genes."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import c_oracle
    from trigenicinteractionpredictor_amd.linkshard import train_degree
    P, ids, counts, th, pr = c5
    deg = train_degree(ids, P)
    top = np.argsort(-deg, kind="stable")[:20]
    rest = np.setdiff1d(np.arange(P), top)
    pick = np.concatenate([top, np.random.default_rng(11).choice(rest, 180, replace=False)])
    sel = np.zeros(P, dtype=bool)
    sel[pick] = True
    mask = sel[ids].any(axis=1)
    sub_ids, sub_counts = ids[mask], counts[mask]
    eng = _c5_engine(c5)
    eng.iterate(1)
    t_gpu = eng.theta[0].cpu().numpy()[pick]
    eng.close()
    blocks = np.array_split(np.arange(sub_ids.shape[0]), 16)
    with ThreadPoolExecutor(16) as ex:
        parts = list(ex.map(lambda b: c_oracle.accumulate(sub_ids[b], sub_counts[b], th, pr)[0], blocks))
    nth = parts[0]
    for part in parts[1:]:
        nth = nth + part
    want = nth[pick] / deg[pick, None]
    assert sub_ids.shape[0] > 100_000 and deg[top].min() > deg.mean()
    np.testing.assert_allclose(t_gpu, want, rtol=RTOL, atol=ATOL)


def test_restart_driver_on_gpu_matches_oracle_driver(tmp_path):
    """restarts.run_samples on the batched GPU engine: the same per-sample iterations, convergence
    and likelihoods as the driver on the oracle engine (:1253-1279 per sample)."""
    from oracle_engine import OracleEngine
    from trigenicinteractionpredictor_amd.data import FoldSpec
    from trigenicinteractionpredictor_amd.restarts import init_samples, run_samples
    m = _model(tmp_path, FoldSpec(P=200, E=3000, seed=12))
    ids = list(range(4))
    th, pr = init_samples(m, 4, ids, seed=8)
    eng = _engine(m, 4, 4, th, pr)
    got = run_samples(eng, ids, th, pr, iterations=60, fcheck=5, bcheck=10)
    want = run_samples(OracleEngine(m.links, m.test_links, B=len(ids)), ids, th, pr, iterations=60, fcheck=5,
                       bcheck=10)
    for g, w in zip(got, want):
        assert (g.sample, g.iterations, g.converged) == (w.sample, w.iterations, w.converged)
        np.testing.assert_allclose(g.loglik, w.loglik, rtol=RTOL)
        np.testing.assert_allclose(g.heldout, w.heldout, rtol=RTOL)
