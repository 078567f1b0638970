"""GPU parity: the HIP path through the C ABI against the reference fixtures and the oracle.

Tolerance: north star "theta, p and log-likelihood within 1e-6 relative" — we
assert rtol=1e-9 on theta/p/L (FP64 with a re-associated sum order) and never
looser than 1e-6.  Predictions: rtol 1e-9.
"""
import json
import os
import random

import numpy as np
import pytest

from golden_util import GOLDEN, cases, load

pytestmark = pytest.mark.gpu

RTOL = 1e-9
ATOL = 1e-300
CASES = cases()


def _gpu_model(train, test):
    from trigenicinteractionpredictor_amd import Model
    m = Model()
    m.get_traintest(train, test)
    return m


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_model_matches_reference_fixture(case, name):
    meta, vec, train, test = load(case, name)
    m = _gpu_model(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"])
    np.testing.assert_array_equal(np.array(m.theta), vec["theta_0"])   # host RNG: bit-exact
    np.testing.assert_array_equal(np.array(m.pr), vec["pr_0"])
    done = 0
    for it in meta["iters"]:
        if it > done:
            m.make_iterations(it - done)
            done = it
        np.testing.assert_allclose(np.array(m.theta), vec["theta_%d" % it], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(np.array(m.pr), vec["pr_%d" % it], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(m.compute_likelihood("train"), float(vec["L_%d" % it]), rtol=RTOL)
        np.testing.assert_allclose(m.compute_likelihood("test"), float(vec["LT_%d" % it]), rtol=RTOL)
    m.calculate_test_set_results()
    got = np.array([r[0] for r in m.results])
    np.testing.assert_allclose(got, vec["pred"], rtol=RTOL, atol=1e-300)
    # Metrics depend on the ORDER of the predictions.  Where two predictions sit closer than
    # the FP64 re-association noise (degenerate K=1 fits are full of near-ties) the order is
    # not determined by the algorithm, so exact metric parity is asserted only when every
    # adjacent gap is well above it (the metric code itself: tests/test_host.py).
    srt = np.sort(vec["pred"])
    gaps = np.diff(srt) / np.maximum(np.abs(srt[1:]), 1e-300)
    if not np.isnan(vec["metrics"]).any() and (gaps.size == 0 or gaps.min() > 1e-7):
        np.testing.assert_allclose(np.array(m.calculate_metrics()), vec["metrics"], rtol=1e-12)


def test_single_make_iteration_calls_match_fixture():
    meta, vec, train, test = load("tiny", "K3_s1")
    m = _gpu_model(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(3)
    for _ in range(5):
        m.make_iteration()
        _ = m.theta  # host round trip between iterations (reference-style driver)
    np.testing.assert_allclose(np.array(m.theta), vec["theta_5"], rtol=RTOL)
    np.testing.assert_allclose(np.array(m.pr), vec["pr_5"], rtol=RTOL)


def test_zero_degree_raises_like_reference():
    d = os.path.join(GOLDEN, "edge")
    with open(os.path.join(d, "zerodeg.json")) as f:
        meta = json.load(f)
    m = _gpu_model(os.path.join(d, "train.dat"), os.path.join(d, "test_zerodeg.dat"))
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"])
    np.testing.assert_allclose(m.compute_likelihood("train"), meta["L_0"], rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), meta["LT_0"], rtol=RTOL)
    with pytest.raises(ZeroDivisionError):
        m.make_iteration()


def _fold(tmp_path, P, E, seed, **kw):
    from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
    tr, te = str(tmp_path / "train.dat"), str(tmp_path / "test.dat")
    write_fold(FoldSpec(P=P, E=E, seed=seed, **kw), tr, te)
    return tr, te


def _oracle_run(m, theta, pr, iters):
    from oracle import c_oracle
    ids, counts = c_oracle.links_to_arrays(m.links)
    for _ in range(iters):
        theta, pr = c_oracle.make_iteration(ids, counts, theta, pr)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    return theta, pr, c_oracle.loglik(ids, counts, theta, pr), c_oracle.loglik(tids, tcounts, theta, pr)


@pytest.mark.parametrize("K,P,E,iters", [(10, 1500, 90000, 3), (16, 300, 3000, 3),
                                         (20, 200, 1500, 2), (30, 120, 600, 2), (7, 400, 4000, 5),
                                         (1, 50, 300, 5)])
def test_against_c_oracle(tmp_path, K, P, E, iters):
    """fold0-sized K=10 (the headline config) and the large-K kernels vs the C oracle."""
    tr, te = _fold(tmp_path, P, E, seed=K + 100, multi_frac=0.05, both_frac=0.02)
    m = _gpu_model(tr, te)
    random.seed(K)
    m.initialize_parameters(K)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(iters)
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, iters)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


@pytest.mark.parametrize("hub", [(0.02, 0.3), (0.01, 0.6)])
def test_hub_fold0_against_c_oracle(tmp_path, hub):
    """A fold0-sized (P=1500, 90k triples) hub-heavy fold, shaped like get_input's trigenic screens
    (:218-318: a few query genes in many triples; data.FoldSpec.hub_*): hub genes' pivot runs span
    many units and blocks.  K=10 (the headline kernels) vs the C oracle, 2 iterations."""
    tr, te = _fold(tmp_path, 1500, 90000, seed=77, multi_frac=0.05, both_frac=0.02,
                   hub_frac=hub[0], hub_share=hub[1])
    m = _gpu_model(tr, te)
    random.seed(5)
    m.initialize_parameters(10)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(2)
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


@pytest.mark.parametrize("units", ["1,1", "3,5", None])
@pytest.mark.parametrize("K", [3, 10, 16])
def test_work_plan_splits_match_oracle(tmp_path, monkeypatch, K, units):
    """Unit / workgroup splits of the observation streams (csrc/plan.h): two units in all (every
    pivot run of a stream in one wave, up to lmax chunks), a few, and the default; K=16 has no
    zero V rows (16 = 4 b-tiles), K=3 / K=10 pad."""
    if units is None:
        monkeypatch.delenv("MMSBM_UNITS", raising=False)
    else:
        monkeypatch.setenv("MMSBM_UNITS", units)
    tr, te = _fold(tmp_path, 300, 6000, seed=K, multi_frac=0.05, both_frac=0.02)
    m = _gpu_model(tr, te)
    random.seed(K + 1)
    m.initialize_parameters(K)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(2)
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


@pytest.mark.parametrize("K,P,E,env", [
    (28, 40, 3000, {}),                        # balanced units + merged rows: runs span waves
    (28, 40, 3000, {"MMSBM_UNITS": "1,1"}),    # 64-chunk units: runs span 3+ waves of a workgroup
    (30, 60, 4000, {"MMSBM_MERGE": "0"}),      # one row per unit stretch (measurement path)
    (30, 60, 4000, {"MMSBM_BALANCE": "0"}),    # whole runs per unit (round-3 packing)
    (26, 50, 3000, {"MMSBM_SP_ROWS": "8"}),    # many short S-partial parts (gm_kernel row tiles)
    (20, 60, 4000, {"MMSBM_GCAP": "4"}),       # fewer V-table genes per pass-A workgroup
    (20, 60, 4000, {"MMSBM_UNITS": "1,1"}),    # balanced without merging (K < 25)
    (30, 60, 4000, {"MMSBM_GM_Q4": "0"}),      # a small plan at K >= 25 on gm_kernel's two halves
    (26, 50, 3000, {"MMSBM_SP_ROWS": "128"}),  # 128-row parts forced on a small plan (no 64-row rule)
])
def test_large_k_plan_variants_match_oracle(tmp_path, monkeypatch, K, P, E, env):
    """The large-K work plans (csrc/plan.h pack_balanced, Plan::merge; mmsbm.hip's merged partial
    rows, gm_kernel's S-partial parts, the pass-A gene cap) with few genes and long pivot runs, so a run's chunks
    spread over several waves of a workgroup, vs the C oracle after 2 iterations."""
    for k in ("MMSBM_UNITS", "MMSBM_MERGE", "MMSBM_BALANCE", "MMSBM_SP_ROWS", "MMSBM_GCAP", "MMSBM_GM_Q4"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tr, te = _fold(tmp_path, P, E, seed=K + 7, multi_frac=0.05, both_frac=0.02)
    m = _gpu_model(tr, te)
    random.seed(K + 3)
    m.initialize_parameters(K)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(2)
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


@pytest.mark.parametrize("K,P,E", [(30, 3000, 4000), (12, 4000, 3000), (4, 30, 1500), (32, 40, 900)])
def test_short_and_long_pivot_runs_match_oracle(tmp_path, K, P, E):
    """Many genes with one or two observations each (every chunk a new pivot gene: stream-0
    workgroups capped by their V table, one partial row per chunk) and few genes with very long
    runs (runs split over units and workgroups, partial rows summed per gene)."""
    tr, te = _fold(tmp_path, P, E, seed=K + P, multi_frac=0.05, both_frac=0.05)
    m = _gpu_model(tr, te)
    random.seed(K)
    m.initialize_parameters(K)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(2)
    info = m._engine.plan_info()
    assert info["genes_per_wg_max"] >= 1 and info["partial_rows"] >= 1
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


@pytest.mark.parametrize("K,P,E,B", [(2, 200, 3000, 3), (13, 200, 3000, 1), (17, 150, 2500, 2),
                                     (24, 120, 2000, 1), (29, 100, 1500, 1), (32, 100, 1200, 2)])
def test_batched_engine_matches_oracle(tmp_path, K, P, E, B):
    """EMEngine with B batched samples against the oracle, per sample, at K up to 32."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd import EMEngine
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, P, E, seed=70 + K, multi_frac=0.05, both_frac=0.02)
    m = _gpu_model(tr, te)
    random.seed(K)
    thetas, prs = [], []
    for _ in range(B):
        m.initialize_parameters(K)
        thetas.append(np.array(m.theta))
        prs.append(np.array(m.pr))
    eng = EMEngine(K, m.P, B=B)
    ids, counts = links_to_arrays(m.links)
    eng.set_links(0, ids, counts)
    eng.upload(np.stack(thetas), np.stack(prs))
    eng.iterate(2)
    th, pr = eng.download()
    L = eng.loglik(0)
    for b in range(B):
        th_o, pr_o = thetas[b], prs[b]
        for _ in range(2):
            th_o, pr_o = c_oracle.make_iteration(ids, counts, th_o, pr_o)
        np.testing.assert_allclose(th[b], th_o, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(pr[b], pr_o, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(L[b], c_oracle.loglik(ids, counts, th_o, pr_o), rtol=RTOL)


@pytest.mark.parametrize("K", [4, 10, 13])
def test_batched_samples_match_single_runs_bitwise(tmp_path, K):
    """Within one kernel family a sample's bits do not depend on its batch-mates, the batch size
    or its slot (the work plan is the same for every B), so restart sharding over 1 or 8 GPUs and
    the restart pool give identical samples (include/mmsbm.h mmsbm_set_family).
    Both small-K families (SK_U, SK_Y; K > 12 has one) are run at B = 3 and B = 1 and compared
    bit for bit, and each agrees with the C oracle at the parity tolerance."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 200, 2000, seed=3)
    m = Model()
    m.get_traintest(tr, te)
    B = 3
    random.seed(77)
    thetas, prs = [], []
    for _ in range(B):
        m.initialize_parameters(K)
        thetas.append(np.array(m.theta))
        prs.append(np.array(m.pr))
    ids, counts = links_to_arrays(m.links)
    tids, tcounts = links_to_arrays(m.test_links)
    oracle = []
    for s in range(B):
        th_o, pr_o = thetas[s], prs[s]
        for _ in range(4):
            th_o, pr_o = c_oracle.make_iteration(ids, counts, th_o, pr_o)
        oracle.append((th_o, pr_o))
    for family in (("sku", "sky") if K <= 12 else ("auto",)):
        eng = EMEngine(K, m.P, B=B, family=family)
        eng.set_links(0, ids, counts)
        eng.set_links(1, tids, tcounts)
        assert eng.plan_info()["small_k"] == {"sku": 2, "sky": 3, "auto": 0}[family]
        eng.upload(np.stack(thetas), np.stack(prs))
        eng.iterate(4)
        th_b, pr_b = eng.download()
        L_b = eng.loglik(0)
        for s in range(B):
            one = EMEngine(K, m.P, B=1, family=family)
            one.set_links(0, ids, counts)
            one.upload(thetas[s][None], prs[s][None])
            one.iterate(4)
            th1, pr1 = one.download()
            np.testing.assert_array_equal(th1[0], th_b[s])
            np.testing.assert_array_equal(pr1[0], pr_b[s])
            assert one.loglik(0)[0] == L_b[s]
            np.testing.assert_allclose(th_b[s], oracle[s][0], rtol=RTOL, atol=ATOL)
            np.testing.assert_allclose(pr_b[s], oracle[s][1], rtol=RTOL, atol=ATOL)


def test_family_defaults_follow_batch_size(tmp_path):
    """MMSBM_FAMILY_AUTO: SK_U for one sample (the drop-in Model), SK_Y from two."""
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 100, 800, seed=4)
    m = Model()
    m.get_traintest(tr, te)
    random.seed(1)
    m.initialize_parameters(6)
    m.make_iteration()
    assert m._engine.plan_info()["small_k"] == 2
    for B, want in ((1, 2), (2, 3), (5, 3)):
        eng = EMEngine(6, m.P, B=B)
        eng.set_links(0, *links_to_arrays(m.links))
        assert eng.plan_info()["small_k"] == want


@pytest.mark.parametrize("K", [10, 20])
def test_active_prefix_and_slot_moves_keep_bits(tmp_path, K):
    """mmsbm_set_active / EMEngine.move_slot / upload_slot (the restart pool's operations): slots
    outside the active prefix are not touched, and a sample moved between slots mid-run ends
    bitwise equal to an uninterrupted single run of the same family."""
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 150, 1500, seed=5)
    m = Model()
    m.get_traintest(tr, te)
    random.seed(2)
    th, pr = [], []
    for _ in range(4):
        m.initialize_parameters(K)
        th.append(np.array(m.theta))
        pr.append(np.array(m.pr))
    ids, counts = links_to_arrays(m.links)
    eng = EMEngine(K, m.P, B=4, family="sky")
    eng.set_links(0, ids, counts)
    for b in range(4):
        eng.upload_slot(b, th[b], pr[b])
    eng.iterate(2)
    eng.set_active(2)                      # slots 2, 3 frozen
    frozen = eng.download()
    eng.iterate(3)
    L = eng.loglik(0)
    assert np.isnan(L[2:]).all() and np.isfinite(L[:2]).all()
    now = eng.download()
    np.testing.assert_array_equal(now[0][2:], frozen[0][2:])
    np.testing.assert_array_equal(now[1][2:], frozen[1][2:])
    eng.move_slot(0, 1)                    # sample 1 continues in slot 0
    eng.upload_slot(1, th[3], pr[3])       # slot 1: sample 3 from its initial state
    eng.iterate(1)
    th_b, pr_b = eng.download()

    def single(s, n):
        one = EMEngine(K, m.P, B=1, family="sky")
        one.set_links(0, ids, counts)
        one.upload(th[s][None], pr[s][None])
        one.iterate(n)
        return one.download()
    t1, p1 = single(1, 6)
    np.testing.assert_array_equal(th_b[0], t1[0])
    np.testing.assert_array_equal(pr_b[0], p1[0])
    t3, p3 = single(3, 1)
    np.testing.assert_array_equal(th_b[1], t3[0])
    np.testing.assert_array_equal(pr_b[1], p3[0])
    td, pd = eng.download_slot(1)
    np.testing.assert_array_equal(td, t3[0])
    np.testing.assert_array_equal(pd, p3[0])


def test_bitwise_reproducible(tmp_path):
    tr, te = _fold(tmp_path, 300, 5000, seed=9)
    out = []
    for _ in range(2):
        m = _gpu_model(tr, te)
        random.seed(5)
        m.initialize_parameters(10)
        m.make_iterations(5)
        out.append((np.array(m.theta), np.array(m.pr), m.compute_likelihood()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


def test_empty_test_set(tmp_path):
    tr, _ = _fold(tmp_path, 60, 300, seed=4)
    te = str(tmp_path / "empty.dat")
    open(te, "w").close()
    m = _gpu_model(tr, te)
    random.seed(1)
    m.initialize_parameters(2)
    m.make_iteration()
    assert m.compute_likelihood("test") == 0.0


@pytest.mark.parametrize("G", [1, 3, 8])
def test_graph_replay_matches_direct_launches_bitwise(tmp_path, monkeypatch, G):
    """MMSBM_GRAPH=G replays G iterations per hipGraph launch: the same kernels with the same
    arguments, so the bits equal direct launches; a new link set (context generation) or new
    theta / p buffers re-capture the graph."""
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 300, 5000, seed=11)
    m = Model()
    m.get_traintest(tr, te)
    K, B = 10, 2
    random.seed(3)
    thetas, prs = [], []
    for _ in range(B):
        m.initialize_parameters(K)
        thetas.append(np.array(m.theta))
        prs.append(np.array(m.pr))
    ids, counts = links_to_arrays(m.links)
    out = {}
    for mode in ("0", str(G)):
        monkeypatch.setenv("MMSBM_GRAPH", mode)
        eng = EMEngine(K, m.P, B=B)
        eng.set_links(0, ids, counts)
        eng.upload(np.stack(thetas), np.stack(prs))
        eng.iterate(2 * G + 2)            # warm-up iteration, two graph launches, remainder
        eng.iterate(G)
        first = eng.download()
        eng.set_links(0, ids[::-1].copy(), counts[::-1].copy())   # new plan: re-capture
        eng.iterate(G + 1)
        out[mode] = (first, eng.download())
    for a, b in zip(out["0"], out[str(G)]):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


def test_context_reshaped_to_another_K_matches_oracle(tmp_path):
    """mmsbm_set_shape on a used context (K=10 -> K=20): the >64 KB dynamic-LDS opt-ins belong to
    the kernels of the new K, so they are redone, and the iteration matches the C oracle."""
    import torch
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd import EMEngine, Model, _lib
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 300, 5000, seed=21)
    m = Model()
    m.get_traintest(tr, te)
    ids, counts = links_to_arrays(m.links)
    random.seed(4)
    m.initialize_parameters(10)
    eng = EMEngine(10, m.P)
    eng.set_links(0, ids, counts)
    eng.upload(np.array(m.theta)[None], np.array(m.pr)[None])
    eng.iterate(1)
    m.initialize_parameters(20)
    th0, pr0 = np.array(m.theta), np.array(m.pr)
    _lib.check(eng.lib.mmsbm_set_shape(eng.ctx, 20, 2, 1, m.P, 1e-10))
    eng.K, eng.K3 = 20, 20 ** 3
    eng.theta = torch.zeros((1, m.P, 20), dtype=torch.float64, device=eng.device)
    eng.pr = torch.zeros((1, 2, 20 ** 3), dtype=torch.float64, device=eng.device)
    eng.set_links(0, ids, counts)
    eng.upload(th0[None], pr0[None])
    eng.iterate(2)
    th, pr = eng.download()
    th_o, pr_o = th0, pr0
    for _ in range(2):
        th_o, pr_o = c_oracle.make_iteration(ids, counts, th_o, pr_o)
    np.testing.assert_allclose(th[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(pr[0], pr_o, rtol=RTOL, atol=ATOL)


def test_reshape_without_new_links_is_refused(tmp_path):
    """mmsbm_set_shape with another K drops the old plans, degree and workspace: iterating before
    mmsbm_set_links is an error (MMSBM_ERR_INVALID), not a run on the old shape's plan."""
    from trigenicinteractionpredictor_amd import EMEngine, Model, _lib
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 300, 5000, seed=22)
    m = Model()
    m.get_traintest(tr, te)
    ids, counts = links_to_arrays(m.links)
    random.seed(5)
    m.initialize_parameters(20)
    eng = EMEngine(20, m.P)
    eng.set_links(0, ids, counts)
    eng.upload(np.array(m.theta)[None], np.array(m.pr)[None])
    eng.iterate(1)
    for K, B, P in ((10, 1, m.P), (20, 2, m.P), (20, 1, m.P + 7)):
        _lib.check(eng.lib.mmsbm_set_shape(eng.ctx, 20, 2, 1, m.P, 1e-10))   # back to the start
        eng.set_links(0, ids, counts)
        _lib.check(eng.lib.mmsbm_set_shape(eng.ctx, K, 2, B, P, 1e-10))
        with pytest.raises(_lib.MMSBMError) as err:
            eng.iterate(1)
        assert err.value.code == _lib.MMSBM_ERR_INVALID
        with pytest.raises(_lib.MMSBMError):   # the likelihood call checks its workspace too
            eng.loglik_async(0)
    eng.synchronize()


def test_degree_override_applies_to_the_next_train_set_only(tmp_path):
    """mmsbm_set_degree pins the degree for the next train link set; a later set_links(TRAIN)
    without one counts its own links again (the reference's `counter`, :986-994)."""
    from oracle import c_oracle
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    tr, te = _fold(tmp_path, 200, 3000, seed=23)
    m = Model()
    m.get_traintest(tr, te)
    ids, counts = links_to_arrays(m.links)
    random.seed(6)
    m.initialize_parameters(4)
    th0, pr0 = np.array(m.theta), np.array(m.pr)
    eng = EMEngine(4, m.P)
    eng.set_links(0, ids, counts, deg=np.full(m.P, 1000, dtype=np.int32))   # a bogus pin
    eng.set_links(0, ids, counts)                                           # counted afresh
    eng.upload(th0[None], pr0[None])
    eng.iterate(1)
    th, pr = eng.download()
    th_o, pr_o = c_oracle.make_iteration(ids, counts, th0, pr0)
    np.testing.assert_allclose(th[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(pr[0], pr_o, rtol=RTOL, atol=ATOL)


def test_accumulate_without_train_links_keeps_the_theta_addend(tmp_path):
    """A context with no train observations: mmsbm_accumulate returns nth = the theta addend
    (include/mmsbm.h), as the fin path would, and S = 0."""
    import torch
    from trigenicinteractionpredictor_amd import EMEngine, _lib
    P, K = 50, 3
    eng = EMEngine(K, P)
    deg = np.ones(P, dtype=np.int32)
    eng.set_links(0, np.zeros((0, 3), np.int32), np.zeros((0, 2), np.int32), deg=deg)
    add = torch.rand((1, P, K), dtype=torch.float64, device=eng.device)
    _lib.check(eng.lib.mmsbm_set_theta_addend(eng.ctx, add.data_ptr()))
    nth = torch.full((1, P, K), 7.0, dtype=torch.float64, device=eng.device)
    S = torch.full((1, 2, K ** 3), 7.0, dtype=torch.float64, device=eng.device)
    eng.accumulate(nth, S)
    eng.synchronize()
    assert torch.equal(nth, add)
    assert torch.count_nonzero(S).item() == 0


def test_in_place_link_edit_between_iterations_matches_oracle():
    """The reference re-reads `links` on every make_iteration (:987): an in-place edit between two
    iterations (a new rating on one link, a removed link) must reach the device."""
    from oracle import c_oracle
    meta, vec, train, test = load("tiny", "K3_s1")
    m = _gpu_model(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(3)
    m.make_iteration()
    th, pr = np.array(m.theta), np.array(m.pr)
    keys = list(m.links)
    m.links[keys[0]][1] += 2            # both ratings observed now
    del m.links[keys[-1]]
    ids, counts = c_oracle.links_to_arrays(m.links)
    deg = np.bincount(ids.ravel(), minlength=m.P)
    assert deg.min() > 0
    m.make_iteration()
    th_o, pr_o = c_oracle.make_iteration(ids, counts, th, pr)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), c_oracle.loglik(ids, counts, th_o, pr_o),
                               rtol=RTOL)


@pytest.mark.parametrize("K,env", [(10, {}), (10, {"MMSBM_SK": "0"}), (12, {"MMSBM_UNITS": "1,1"}),
                                   (7, {"MMSBM_UNITS": "5,9"}), (13, {}),
                                   (10, {"MMSBM_SK_FUSED": "0"}), (11, {"MMSBM_SK_FUSED": "0"}),
                                   (9, {"MMSBM_SK_FUSED": "0", "MMSBM_UNITS": "7,3"}),
                                   (10, {"MMSBM_UNITS": "1,1"}), (5, {"MMSBM_UNITS": "40,40"}),
                                   (10, {"MMSBM_SK_Y": "1"}), (12, {"MMSBM_SK_Y": "1"}),
                                   (3, {"MMSBM_SK_Y": "1", "MMSBM_UNITS": "7,3"}),
                                   (1, {"MMSBM_SK_Y": "1"}), (2, {"MMSBM_SK_Y": "1"}),
                                   (4, {"MMSBM_SK_Y": "1", "MMSBM_UNITS": "3,3"}),
                                   (11, {"MMSBM_SK_Y": "1"}), (9, {"MMSBM_SK_Y": "1", "MMSBM_UNITS": "1,1"}),
                                   (10, {"MMSBM_SK_RHO": "50"}), (6, {"MMSBM_SK_RHO": "100"})])
def test_kernel_family_matches_oracle(tmp_path, monkeypatch, K, env):
    """K <= 12 runs the small-K kernels (csrc/sk.h; the three-stream fused E-step by default
    (SK_U), the stream-0 E-step with Y entries with MMSBM_SK_Y=1 (SK_Y), pass A + pass B with
    MMSBM_SK_FUSED=0; 8 stretches per unit at K <= 10, 4 above), K > 12 the large-K ones;
    MMSBM_SK=0 forces the large-K family at K=10, MMSBM_UNITS forces long (up to 128 chunks: eight
    16-chunk blocks per unit) or short units.  Every variant matches the C oracle (2 iterations,
    train and held-out likelihood)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tr, te = _fold(tmp_path, 400, 12000, seed=31 + K, multi_frac=0.1, both_frac=0.03)
    m = _gpu_model(tr, te)
    random.seed(K)
    m.initialize_parameters(K)
    theta0, pr0 = np.array(m.theta), np.array(m.pr)
    m.make_iterations(2)
    info = m._engine.plan_info()
    small = K <= 12 and env.get("MMSBM_SK") != "0"
    assert info["small_k"] == (0 if not small else 1 if env.get("MMSBM_SK_FUSED") == "0"
                               else 3 if env.get("MMSBM_SK_Y") == "1" else 2)
    if small:
        assert info["genes_per_wg_max"] == (8 if K <= 10 else 4)
    th_o, pr_o, L_o, LT_o = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(np.array(m.theta), th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood("train"), L_o, rtol=RTOL)
    np.testing.assert_allclose(m.compute_likelihood("test"), LT_o, rtol=RTOL)


def _gm_valid_cs(K):
    """GM<K>::cs_ok: workgroups per S part that divide the NQ fixed X groups of QC chunks (up to
    four above K = 16 -- at K >= 25 on plans with fewer parts than CUs, like these -- two at
    K <= 16) and keep one workgroup's S accumulators within 8 chunks (csrc/mmsbm.hip GM)."""
    nch = (K * K + 63) // 64
    qc = (nch + 1) // 2 if K <= 16 else (nch + 3) // 4  # (K >= 25: these small plans take GM::Q4)
    nq = (nch + qc - 1) // qc
    return [cs for cs in range(1, nq + 1) if nq % cs == 0 and (cs > 1 or nch <= 8) and (nq // cs) * qc <= 8]


@pytest.mark.parametrize("K", [13, 16, 20, 22, 30])
def test_gm_workgroups_per_part_keep_bits(tmp_path, monkeypatch, K):
    """gm_kernel forms its X rows in NQ fixed groups of the cell chunks (up to four above K = 16,
    at K >= 25 on small plans (GM::Q4), two at K <= 16), so every valid count of workgroups per S part (MMSBM_GM_CS = 1, 2, 3,
    4 as GM<K> allows) gives the same bits: the launch may follow the batch.
    All agree bit for bit and with the C oracle."""
    tr, te = _fold(tmp_path, 150, 2500, seed=K + 40, multi_frac=0.05, both_frac=0.02)
    valid = _gm_valid_cs(K)
    assert len(valid) >= 2, valid
    out = {}
    for cs in valid:
        monkeypatch.setenv("MMSBM_GM_CS", str(cs))
        m = _gpu_model(tr, te)
        random.seed(K)
        m.initialize_parameters(K)
        theta0, pr0 = np.array(m.theta), np.array(m.pr)
        m.make_iterations(2)
        assert m._engine.plan_info()["gm_groups"] == cs
        out[cs] = (np.array(m.theta), np.array(m.pr), m.compute_likelihood("train"))
    ref = out[valid[0]]
    for cs in valid[1:]:
        np.testing.assert_array_equal(out[cs][0], ref[0])
        np.testing.assert_array_equal(out[cs][1], ref[1])
        assert out[cs][2] == ref[2]
    th_o, pr_o, L_o, _ = _oracle_run(m, theta0, pr0, 2)
    np.testing.assert_allclose(ref[0], th_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(ref[1], pr_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(ref[2], L_o, rtol=RTOL)


def test_gm_workgroups_follow_the_batch_with_the_same_bits(tmp_path, monkeypatch):
    """Without the override gm_kernel takes the most workgroups per S part whose grid fits one
    round of resident workgroups (one sample: four) and one where none would (8 samples): a
    sample run alone and the same sample in slot 3 of an 8-sample engine end bit for bit equal
    (K=20, ~38 parts of 64 rows)."""
    from trigenicinteractionpredictor_amd import EMEngine
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    monkeypatch.delenv("MMSBM_GM_CS", raising=False)
    tr, te = _fold(tmp_path, 1200, 20000, seed=61)
    m = _gpu_model(tr, te)
    K, B = 20, 8
    random.seed(9)
    thetas, prs = [], []
    for _ in range(B):
        m.initialize_parameters(K)
        thetas.append(np.array(m.theta))
        prs.append(np.array(m.pr))
    ids, counts = links_to_arrays(m.links)
    big = EMEngine(K, m.P, B=B)
    big.set_links(0, ids, counts)
    big.upload(np.stack(thetas), np.stack(prs))
    one = EMEngine(K, m.P, B=1)
    one.set_links(0, ids, counts)
    one.upload(thetas[3][None], prs[3][None])
    g8, g1 = big.plan_info()["gm_groups"], one.plan_info()["gm_groups"]
    import torch
    if torch.cuda.get_device_properties(big.device).multi_processor_count == 256:  # (the rule counts CUs)
        assert (g8, g1) == (1, 4), (g8, g1)
    big.iterate(2)
    one.iterate(2)
    tb, pb = big.download()
    t1, p1 = one.download()
    np.testing.assert_array_equal(tb[3], t1[0])
    np.testing.assert_array_equal(pb[3], p1[0])
