"""CPU tests of the host side: ingestion, RNG init, metrics, device layout, fold, generator.

These pin the parts of the drop-in `Model` that stay on the host
(src/TrigenicInteractionPredictor.py :106-170, :321-423, :447-523, :583-637)
against the reference-generated fixtures and the oracle."""
import contextlib
import io
import os
import random

import numpy as np
import pytest

from golden_util import cases, load
from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
from trigenicinteractionpredictor_amd.layout import links_to_arrays, n_observations
from trigenicinteractionpredictor_amd.model import Model

CASES = cases()


def _model(train, test):
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(train, test)
    return m


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_ingestion_matches_reference(case, name):
    meta, vec, train, test = load(case, name)
    m = _model(train, test)
    assert m.P == meta["P"]
    assert [[k, v] for k, v in m.links.items()] == meta["links"]
    assert [[k, v] for k, v in m.test_links.items()] == meta["test_links"]
    assert [m.id_gene[i] for i in range(m.P)] == meta["id_gene"]


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_initialize_parameters_bit_exact(case, name):
    meta, vec, train, test = load(case, name)
    m = _model(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"])
    np.testing.assert_array_equal(np.array(m.theta), vec["theta_0"])
    np.testing.assert_array_equal(np.array(m.pr), vec["pr_0"])


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_metrics_match_reference_on_reference_predictions(case, name):
    """Sort-based AUC == the reference's O(n+ n-) count (:611-615), exactly."""
    meta, vec, train, test = load(case, name)
    if np.isnan(vec["metrics"]).any():
        pytest.skip("reference metrics undefined (no positives or no negatives)")
    m = _model(train, test)
    m.results = [[float(p), str(k), int(r)] for p, k, r in zip(vec["pred"], vec["pred_key"], vec["pred_real"])]
    assert m.calculate_metrics() == vec["metrics"].tolist()


def test_metrics_ties_counted_as_not_greater():
    m = Model()
    m.links = {"0_1_2": [0, 1], "0_1_3": [1, 0]}
    m.test_links = {"a": [0, 1], "b": [1, 0], "c": [1, 0], "d": [0, 1]}
    m.results = [[0.5, "a", 1], [0.5, "b", 0], [0.4, "c", 0], [0.3, "d", 1]]
    prec, rec, fall, auc = m.calculate_metrics()
    # pairs (pos, neg): (0.5,0.5) tie -> 0, (0.5,0.4) 1, (0.3,0.5) 0, (0.3,0.4) 0
    assert auc == 1 / 4


def test_link_arrays_keep_key_order_and_counts():
    links = {"0_1_2": [1, 0], "10_2_9": [0, 2], "3_3_4": [2, 1], "1_5_6": [0, 1]}
    ids, counts = links_to_arrays(links)
    assert ids[1].tolist() == [10, 2, 9]         # string-sorted key order is kept
    assert ids[2].tolist() == [3, 3, 4]          # a repeated gene keeps both slots
    assert counts.tolist() == [[1, 0], [0, 2], [2, 1], [0, 1]]
    assert n_observations(counts) == 5


def test_fold_splits_are_complementary(tmp_path):
    tr, te = str(tmp_path / "tr.dat"), str(tmp_path / "te.dat")
    write_fold(FoldSpec(P=50, E=300, seed=2), tr, te)
    m = _model(tr, te)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        np.random.seed(0)
        m.fold(0.2)
        lines = lambda f: open(f).read().splitlines()
        all_tests = []
        for i in range(5):
            t, r = lines("test%d.dat" % i), lines("train%d.dat" % i)
            assert not set(t) & set(r)
            assert len(t) + len(r) == len(m.links)
            all_tests += t
        assert len(all_tests) == len(set(all_tests)) == len(m.links)
    finally:
        os.chdir(cwd)


def test_generator_format_and_coverage(tmp_path):
    tr, te = str(tmp_path / "tr.dat"), str(tmp_path / "te.dat")
    ntr, nte = write_fold(FoldSpec(P=90, E=600, seed=4, multi_frac=0.1, both_frac=0.05, dup_frac=0.1), tr, te)
    train_lines = open(tr).read().splitlines()
    assert len(train_lines) == ntr
    train_genes = set()
    for line in train_lines:
        names, r = line.split("\t")
        parts = names.split("_")
        assert parts == sorted(parts) and r in ("0", "1")
        train_genes.update(parts)
    for line in open(te).read().splitlines():
        assert set(line.split("\t")[0].split("_")) <= train_genes


def test_large_generator_numpy_path(tmp_path):
    tr, te = str(tmp_path / "tr.dat"), str(tmp_path / "te.dat")
    ntr, nte = write_fold(FoldSpec(P=5000, E=1_000_000, seed=1), tr, te)
    assert ntr + nte >= 1_000_000 - 10
    with open(tr) as f:
        first = f.readline()
    names, r = first.rstrip("\n").split("\t")
    assert len(names.split("_")) == 3 and r in ("0", "1")
