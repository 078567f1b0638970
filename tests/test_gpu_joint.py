"""GPU parity of the joint digenic + trigenic model (trigenicinteractionpredictor_amd/joint.py,
include/mmsbm_pairs.h) against the reference `_23` fixtures and the C oracle.

Tolerance as tests/test_gpu_parity.py: rtol 1e-9 on theta / pr / qr / L (FP64, re-associated
sums), predictions rtol 1e-9; the north star asks 1e-6.
"""
import json
import os
import random

import numpy as np
import pytest

from golden_util import JOINT, joint_cases, joint_load

pytestmark = pytest.mark.gpu

RTOL = 1e-9
ATOL = 1e-300
CASES = joint_cases()


def _model(meta, train, test):
    from trigenicinteractionpredictor_amd.joint import DataType, Model
    m = Model()
    m.get_train_test(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"], getattr(DataType, meta["interaction"]))
    return m


def _isolated(pred, gap=1e-7):
    srt = np.sort(pred)
    gaps = np.diff(srt) / np.maximum(np.abs(srt[1:]), 1e-300)
    return gaps.size == 0 or gaps.min() > gap


def compare_short(got, want, pred, rtol=RTOL):
    """to_string_short (:1359-1456): labels, counts, keys, real ratings and the gene list exactly;
    likelihood, predicted probabilities and metrics within rtol (metrics and row order only where
    the reference probabilities are isolated: closer ones are ordered by FP64 noise)."""
    g, w = got.split("\n"), want.split("\n")
    assert len(g) == len(w), (len(g), len(w))
    head = w.index("Predicted Interaction\tID of genes\tReal Interaction")
    end = w.index("", head)
    for i in list(range(head + 1)) + list(range(end, len(w))):
        if w[i].startswith("Max Likelihood:\t"):
            assert g[i].split("\t")[0] == w[i].split("\t")[0]
            np.testing.assert_allclose(float(g[i].split("\t")[1]), float(w[i].split("\t")[1]), rtol=rtol)
        elif i > 0 and w[i - 1] == "Precision\tRecall\tFallout\tAUC":
            if _isolated(pred):
                np.testing.assert_allclose([float(x) for x in g[i].split("\t")],
                                           [float(x) for x in w[i].split("\t")], rtol=rtol)
        else:
            assert g[i] == w[i], (i, g[i], w[i])
    rg = [r.split("\t") for r in g[head + 1:end]]
    rw = [r.split("\t") for r in w[head + 1:end]]
    np.testing.assert_allclose([float(r[0]) for r in rg], [float(r[0]) for r in rw], rtol=rtol, atol=ATOL)
    if _isolated(pred):
        assert [r[1:] for r in rg] == [r[1:] for r in rw]
    assert sorted(tuple(r[1:]) for r in rg) == sorted(tuple(r[1:]) for r in rw)


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_joint_model_matches_reference_fixture(case, name):
    meta, vec, train, test = joint_load(case, name)
    m = _model(meta, train, test)
    np.testing.assert_array_equal(np.array(m.qr), vec["qr_0"])
    done = 0
    for it in meta["iters"]:
        if it > done:
            m.make_iterations(it - done)
            done = it
        np.testing.assert_allclose(np.array(m.theta), vec["theta_%d" % it], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(np.array(m.pr), vec["pr_%d" % it], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(np.array(m.qr), vec["qr_%d" % it], rtol=RTOL, atol=ATOL)
        L = m.compute_likelihood()
        np.testing.assert_allclose(L, float(vec["L_%d" % it]), rtol=RTOL)
        m.likelihoodVector.append([0, it, L])
    m.calculate_test_set_results()
    np.testing.assert_allclose([r[0] for r in m.results], vec["pred"], rtol=RTOL, atol=ATOL)
    assert sorted(r[1] for r in m.results) == sorted(vec["pred_key"].tolist())
    if meta["text"]["to_string_short"] is not None:
        compare_short(m.to_string_short(), meta["text"]["to_string_short"], vec["pred"])


def test_joint_single_iterations_match_fixture():
    meta, vec, train, test = joint_load("tiny", "K3_s2")
    m = _model(meta, train, test)
    for _ in range(5):
        m.make_iteration()
    np.testing.assert_allclose(np.array(m.theta), vec["theta_5"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.qr), vec["qr_5"], rtol=RTOL, atol=ATOL)


def test_joint_zero_degree_raises():
    from trigenicinteractionpredictor_amd.joint import Model
    with open(os.path.join(JOINT, "zerodeg.json")) as f:
        z = json.load(f)
    d = os.path.join(JOINT, "tiny")
    m = Model()
    m.get_train_test(os.path.join(d, "train.dat"), os.path.join(d, "test_zerodeg.dat"))
    random.seed(z["seed"])
    m.initialize_parameters(z["K"])
    np.testing.assert_allclose(m.compute_likelihood(), z["L_0"], rtol=RTOL)
    th0 = np.array(m.theta)
    with pytest.raises(ZeroDivisionError):
        m.make_iteration()
    np.testing.assert_array_equal(np.array(m.theta), th0)   # nothing applied


def _joint_fold(tmp_path, **kw):
    from trigenicinteractionpredictor_amd.data import JointFoldSpec, write_joint_fold
    from trigenicinteractionpredictor_amd.joint import Model
    spec = JointFoldSpec(**kw)
    tr, te = str(tmp_path / "train.dat"), str(tmp_path / "test.dat")
    write_joint_fold(spec, tr, te)
    m = Model()
    m.get_train_test(tr, te)
    return m


def _oracle_arrays(m):
    from oracle import c_oracle
    ids3, c3 = c_oracle.links_to_arrays(m.links)
    ids2, c2 = c_oracle.links_to_arrays(m.dlinks, arity=2)
    return ids3, c3, ids2, c2


@pytest.mark.parametrize("K,P,E3,E2", [(1, 60, 300, 150), (3, 120, 900, 500), (4, 100, 600, 700),
                                       (10, 1500, 90000, 30000), (13, 200, 1500, 800),
                                       (20, 150, 1200, 600), (32, 120, 700, 400),
                                       (5, 80, 0, 600), (6, 90, 700, 0)])
def test_joint_engine_matches_c_oracle(tmp_path, K, P, E3, E2):
    """Against oracle/mmsbm_oracle.c's joint iteration (bit-exact with the reference) at
    K = 1..32, fold0 size (P=1500, 72k train triplets, 24k train pairs), pair-only genes,
    and the degenerate sets: no triplets, no pairs."""
    from oracle import c_oracle
    m = _joint_fold(tmp_path, P=P, E3=E3, E2=E2, seed=K + P, pair_only=P // 20 if E3 and E2 else 0,
                    multi_frac=0.05, both_frac=0.02, ho_frac=0.1, pos_frac=0.1, pair_pos_frac=0.2)
    random.seed(K)
    m.initialize_parameters(K)
    ids3, c3, ids2, c2 = _oracle_arrays(m)
    th, pr, qr = np.array(m.theta), np.array(m.pr), np.array(m.qr)
    n_it = 2
    for _ in range(n_it):
        th, pr, qr = c_oracle.joint_make_iteration(ids3, c3, ids2, c2, th, pr, qr)
    m.make_iterations(n_it)
    np.testing.assert_allclose(np.array(m.theta), th, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.pr), pr, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(np.array(m.qr), qr, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(m.compute_likelihood(), c_oracle.joint_loglik(ids3, c3, ids2, c2, th, pr, qr),
                               rtol=RTOL)
    # prediction of both arities at this K
    keys = list(m.test_links) + list(m.dtest_links)
    m.calculate_test_set_results()
    want = []
    for key in keys:
        ids = np.array([[int(s) for s in key.split("_")]], dtype=np.int32)
        want.append(float((c_oracle.predict(ids, th, pr) if ids.shape[1] == 3
                           else c_oracle.pair_predict(ids, th, qr))[0]))
    np.testing.assert_allclose([r[0] for r in m.results], sorted(want, reverse=True), rtol=RTOL, atol=ATOL)


def test_joint_batched_samples_and_reproducibility(tmp_path):
    """B=3 samples in one JointEngine: each equals its own B=1 run bitwise (the plan does not
    depend on B) and a second run reproduces every bit."""
    from trigenicinteractionpredictor_amd import _lib
    from trigenicinteractionpredictor_amd.joint import JointEngine, _pair_arrays
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    m = _joint_fold(tmp_path, P=300, E3=3000, E2=1500, seed=5, pair_only=10)
    K, B = 7, 3
    inits = []
    for s in range(B):
        random.seed(100 + s)
        m.initialize_parameters(K)
        inits.append((np.array(m.theta), np.array(m.pr), np.array(m.qr)))
    tabs = (*links_to_arrays(m.links, 2), *_pair_arrays(m.dlinks, 2))

    def run(b_inits):
        eng = JointEngine(K, m.P, B=len(b_inits))
        eng.set_links(_lib.SET_TRAIN, *tabs)
        eng.upload(np.stack([x[0] for x in b_inits]), np.stack([x[1] for x in b_inits]),
                   np.stack([x[2] for x in b_inits]))
        eng.iterate(4)
        out = eng.download(), eng.loglik()
        eng.close()
        return out

    (thB, prB, qrB), LB = run(inits)
    for s in range(B):
        (th1, pr1, qr1), L1 = run([inits[s]])
        np.testing.assert_array_equal(thB[s], th1[0])
        np.testing.assert_array_equal(prB[s], pr1[0])
        np.testing.assert_array_equal(qrB[s], qr1[0])
        assert LB[s] == L1[0]
    (thR, prR, qrR), LR = run(inits)
    np.testing.assert_array_equal(thR, thB)
    np.testing.assert_array_equal(qrR, qrB)
    np.testing.assert_array_equal(LR, LB)


def _lines_close(got, want, rtol=RTOL):
    """stdout of the driver: every line exact except the likelihood values (rtol)."""
    g, w = got.split("\n"), want.split("\n")
    assert len(g) == len(w)
    for a, b in zip(g, w):
        if b.startswith("· Likelihood "):
            ha, va = a.rsplit(" ", 1)
            hb, vb = b.rsplit(" ", 1)
            assert ha == hb
            np.testing.assert_allclose(float(va), float(vb), rtol=rtol)
        else:
            assert a == b


@pytest.mark.parametrize("name", ["v0", "v1"])
def test_joint_driver_on_gpu_matches_reference_run(name, tmp_path, monkeypatch, capsys):
    """cli23 on the HIP engine against the reference's run of src/trigenic_fromtesttrain_2+3.py:
    same convergence points and files; likelihoods, probabilities and theta / pr / qr text
    within rtol (to_file) or the to_string_short comparison above."""
    from trigenicinteractionpredictor_amd import cli23
    with open(os.path.join(JOINT, "cli", "driver.json"), encoding="utf-8") as f:
        run = json.load(f)[name]
    d = os.path.join(JOINT, "tiny")
    argv = run["argv"][:5] + [os.path.join(d, "train.dat"), os.path.join(d, "test.dat"),
                              str(run["argv"][5]), str(run["argv"][6])]
    monkeypatch.chdir(tmp_path)
    cli23.main(argv)
    _lines_close(capsys.readouterr().out, run["stdout"])
    got = {f: open(f, encoding="utf-8").read() for f in sorted(os.listdir("."))}
    assert sorted(got) == sorted(run["files"])
    for f, text in got.items():
        want = run["files"][f]
        if run["argv"][5] == 0:
            head = want.split("\n").index("Predicted Interaction\tID of genes\tReal Interaction")
            end = want.split("\n").index("", head)
            pred = np.array([float(r.split("\t")[0]) for r in want.split("\n")[head + 1:end]])
            compare_short(text, want, pred)
        else:   # to_file: numbers printed with 6 / 12 decimals; compare as numbers
            for a, b in zip(text.split("\n"), want.split("\n")):
                fa, fb = a.split("\t"), b.split("\t")
                assert len(fa) == len(fb)
                for x, y in zip(fa, fb):
                    try:
                        np.testing.assert_allclose(float(x), float(y), rtol=1e-6, atol=2e-12)
                    except ValueError:
                        assert x == y


def test_joint_fused_and_unfused_paths_agree(tmp_path):
    """JointEngine.iterate (pair launch + triplet iteration with the theta addend and q cells) against the
    accumulate / mstep / qstep building blocks: same values within FP64 re-association."""
    from trigenicinteractionpredictor_amd import _lib
    from trigenicinteractionpredictor_amd.joint import JointEngine, _pair_arrays
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    m = _joint_fold(tmp_path, P=400, E3=4000, E2=2500, seed=9, pair_only=15)
    random.seed(3)
    m.initialize_parameters(12)
    init = (np.array(m.theta)[None], np.array(m.pr)[None], np.array(m.qr)[None])
    out = []
    for mode in ("iterate", "iterate_unfused"):
        eng = JointEngine(12, m.P, B=1)
        eng.set_links(_lib.SET_TRAIN, *links_to_arrays(m.links, 2), *_pair_arrays(m.dlinks, 2))
        eng.upload(*init)
        getattr(eng, mode)(3)
        out.append(eng.download())
        eng.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-300)


def test_joint_plan_splits_agree(tmp_path, monkeypatch):
    """Small pair workgroups (MMSBM_PAIR_PARTS=16: many workgroups, every gene block split
    differently) give the same iteration as the default plan, up to the S2 re-association."""
    from trigenicinteractionpredictor_amd import _lib
    from trigenicinteractionpredictor_amd.joint import JointEngine, _pair_arrays
    from trigenicinteractionpredictor_amd.layout import links_to_arrays
    m = _joint_fold(tmp_path, P=300, E3=2500, E2=3000, seed=11, pair_only=20)
    random.seed(4)
    m.initialize_parameters(9)
    init = (np.array(m.theta)[None], np.array(m.pr)[None], np.array(m.qr)[None])
    out = []
    for parts in (None, "16"):
        if parts:
            monkeypatch.setenv("MMSBM_PAIR_PARTS", parts)
        eng = JointEngine(9, m.P, B=1)
        eng.set_links(_lib.SET_TRAIN, *links_to_arrays(m.links, 2), *_pair_arrays(m.dlinks, 2))
        if parts:
            assert eng.plan_info(0)["pair_wg_parts_max"] <= 16 * 4
        eng.upload(*init)
        eng.iterate(3)
        out.append(eng.download())
        eng.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-300)
