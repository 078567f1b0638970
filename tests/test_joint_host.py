"""Host half of the joint model mirror (trigenicinteractionpredictor_amd/joint.py) against the
reference `_23` fixtures, on the CPU: ingestion tables, RNG init and the `to_string()` text
(byte-exact, from the reference's own final parameters).  No GPU call."""
import os
import random

import numpy as np
import pytest

from golden_util import joint_cases, joint_load
from trigenicinteractionpredictor_amd.joint import DataType, Model

CASES = joint_cases()


def _model(meta, train, test, capsys=None):
    m = Model()
    m.get_train_test(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"], getattr(DataType, meta["interaction"]))
    return m


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_ingest_and_init_match_reference(case, name):
    meta, vec, train, test = joint_load(case, name)
    m = _model(meta, train, test)
    assert [[k, v] for k, v in m.links.items()] == meta["links"]
    assert [[k, v] for k, v in m.dlinks.items()] == meta["dlinks"]
    assert [[k, v] for k, v in m.test_links.items()] == meta["test_links"]
    assert [[k, v] for k, v in m.dtest_links.items()] == meta["dtest_links"]
    assert [m.id_gene[i] for i in range(m.P)] == meta["id_gene"]
    assert [m.gene_num_aparitions[i] for i in range(m.P)] == meta["gene_num_aparitions"]
    np.testing.assert_array_equal(np.array(m.theta), vec["theta_0"])
    np.testing.assert_array_equal(np.array(m.pr), vec["pr_0"])
    np.testing.assert_array_equal(np.array(m.qr), vec["qr_0"])


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_to_string_is_byte_identical(case, name):
    meta, vec, train, test = joint_load(case, name)
    m = _model(meta, train, test)
    last = meta["iters"][-1]
    m.theta = vec["theta_%d" % last].tolist()
    m.pr = vec["pr_%d" % last].tolist()
    m.qr = vec["qr_%d" % last].tolist()
    m.likelihood = float(vec["L_%d" % last])
    m.likelihoodVector = [[0, it, float(vec["L_%d" % it])] for it in meta["iters"]]
    assert m.to_string() == meta["text"]["to_string"]


def test_get_train_test_prints_like_the_reference(capsys):
    meta, vec, train, test = joint_load("tiny", "K2_s1")
    Model().get_train_test(train, test)
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "number of triplets, pairs %d %d" % (len(meta["links"]), len(meta["dlinks"]))
    assert out[1] == "READ DATA train %d %d" % (len(meta["links"]), len(meta["links"]))
    assert out[2] == "READ DATA train %d %d" % (len(meta["dlinks"]), len(meta["dlinks"]))
    assert out[3] == "READ DATA test %d" % len(meta["test_links"])


def test_fast_folds_write_the_reference_files(tmp_path, monkeypatch):
    """pair_fast_fold (:777-939): test fold 0 leaves dlinks; dtrain0 holds the other folds'
    pairs and every triplet; without `output` the reference ends in UnboundLocalError."""
    meta, vec, train, test = joint_load("small", "K2_s1")
    monkeypatch.chdir(tmp_path)
    m = Model()
    m.get_train_test(train, test)
    n_pairs, n_trip = len(m.dlinks), len(m.links)
    np.random.seed(3)
    m.pair_fast_fold(output=1, folds='yes')
    size = int(n_pairs * 0.2)
    assert len(m.dlinks) == n_pairs - size and len(m.dtest_links) >= size
    lines0 = open("dtest0.dat", encoding="utf-8").read().splitlines()
    assert len(lines0) == size
    tr = open("dtrain0.dat", encoding="utf-8").read().splitlines()
    assert len(tr) == (n_pairs - size) + n_trip
    for f in range(1, 5):
        assert os.path.exists("dtest%d.dat" % f)
    m2 = Model()
    m2.get_train_test(train, test)
    with pytest.raises(UnboundLocalError):
        m2.triplet_fast_fold()
