"""The joint-model oracle (oracle/joint_oracle.py, oracle/mmsbm_oracle.c) is bit-exact against
fixtures written by the reference `src/TrigenicInteractionPredictor_23.py` under the
DataType.ALL -> all spec fix (tests/golden/make_joint_golden.py): ingestion tables, RNG init,
theta / pr / qr and the log-likelihood after 1, 5, 25 iterations, the prediction table and the
metrics."""
import json
import os
import random

import numpy as np
import pytest

from golden_util import JOINT, joint_cases, joint_load
from oracle import c_oracle
from oracle.joint_oracle import ALL, DIGENIC, TRIGENIC, OracleJointModel

CASES = joint_cases()
INTERACTION = {"all": ALL, "trigenic": TRIGENIC, "digenic": DIGENIC}


def _model(meta, train, test):
    m = OracleJointModel()
    m.get_train_test(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(meta["K"], INTERACTION[meta["interaction"]])
    return m


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_joint_ingest_and_init(case, name):
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
    assert m.compute_likelihood() == float(vec["L_0"])


@pytest.mark.parametrize("case,name", [c for c in CASES if c[0] != "small"],
                         ids=["%s/%s" % c for c in CASES if c[0] != "small"])
def test_joint_python_oracle_matches_reference_bitwise(case, name):
    meta, vec, train, test = joint_load(case, name)
    m = _model(meta, train, test)
    done = 0
    for it in meta["iters"]:
        while done < it:
            m.make_iteration()
            done += 1
        np.testing.assert_array_equal(np.array(m.theta), vec["theta_%d" % it])
        np.testing.assert_array_equal(np.array(m.pr), vec["pr_%d" % it])
        np.testing.assert_array_equal(np.array(m.qr), vec["qr_%d" % it])
        assert m.compute_likelihood() == float(vec["L_%d" % it])
    m.calculate_test_set_results()
    assert [r[0] for r in m.results] == vec["pred"].tolist()
    assert [r[1] for r in m.results] == vec["pred_key"].tolist()
    assert [r[2] for r in m.results] == vec["pred_real"].tolist()
    np.testing.assert_array_equal(np.array(m.calculate_metrics()), vec["metrics"])


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_joint_c_oracle_matches_reference_bitwise(case, name):
    meta, vec, train, test = joint_load(case, name)
    m = OracleJointModel()
    m.get_train_test(train, test)
    ids3, c3 = c_oracle.links_to_arrays(m.links)
    ids2, c2 = c_oracle.links_to_arrays(m.dlinks, arity=2)
    theta, pr, qr = vec["theta_0"], vec["pr_0"], vec["qr_0"]
    done = 0
    for it in meta["iters"]:
        while done < it:
            theta, pr, qr = c_oracle.joint_make_iteration(ids3, c3, ids2, c2, theta, pr, qr)
            done += 1
        np.testing.assert_array_equal(theta, vec["theta_%d" % it])
        np.testing.assert_array_equal(pr, vec["pr_%d" % it])
        np.testing.assert_array_equal(qr, vec["qr_%d" % it])
        assert c_oracle.joint_loglik(ids3, c3, ids2, c2, theta, pr, qr) == float(vec["L_%d" % it])
    # prediction: triplets with pr, pairs with qr (:946-973)
    keys = list(m.test_links) + list(m.dtest_links)
    pred = []
    for key in keys:
        ids = np.array([[int(s) for s in key.split("_")]], dtype=np.int32)
        pred.append(float((c_oracle.predict(ids, theta, pr) if ids.shape[1] == 3
                           else c_oracle.pair_predict(ids, theta, qr))[0]))
    assert sorted(pred, reverse=True) == vec["pred"].tolist()


def test_joint_zero_degree_raises():
    with open(os.path.join(JOINT, "zerodeg.json")) as f:
        z = json.load(f)
    assert z["raises_zero_division"]
    d = os.path.join(JOINT, "tiny")
    m = OracleJointModel()
    m.get_train_test(os.path.join(d, "train.dat"), os.path.join(d, "test_zerodeg.dat"))
    random.seed(z["seed"])
    m.initialize_parameters(z["K"])
    assert m.P == z["P"]
    assert m.compute_likelihood() == z["L_0"]
    with pytest.raises(ZeroDivisionError):
        m.make_iteration()
    ids3, c3 = c_oracle.links_to_arrays(m.links)
    ids2, c2 = c_oracle.links_to_arrays(m.dlinks, arity=2)
    with pytest.raises(ZeroDivisionError):
        c_oracle.joint_make_iteration(ids3, c3, ids2, c2, np.array(m.theta), np.array(m.pr), np.array(m.qr))
