"""The C oracle restates the same binary64 operation order as the reference:
bit-exact against the reference fixtures, including the 1600-link K=10 case."""
import random

import numpy as np
import pytest

from golden_util import cases, load
from oracle import c_oracle
from oracle.mmsbm_oracle import OracleModel

CASES = cases()


@pytest.mark.parametrize("case,name", CASES, ids=["%s/%s" % c for c in CASES])
def test_c_oracle_matches_reference_bitwise(case, name):
    meta, vec, train, test = load(case, name)
    m = OracleModel()
    m.get_traintest(train, test)
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)
    theta, pr = vec["theta_0"], vec["pr_0"]
    done = 0
    for it in meta["iters"]:
        while done < it:
            theta, pr = c_oracle.make_iteration(ids, counts, theta, pr)
            done += 1
        np.testing.assert_array_equal(theta, vec["theta_%d" % it])
        np.testing.assert_array_equal(pr, vec["pr_%d" % it])
        assert c_oracle.loglik(ids, counts, theta, pr) == float(vec["L_%d" % it])
        assert c_oracle.loglik(tids, tcounts, theta, pr) == float(vec["LT_%d" % it])
    pred = c_oracle.predict(tids, theta, pr)
    assert sorted(pred.tolist(), reverse=True) == vec["pred"].tolist()


def test_c_oracle_init_matches_python_init():
    meta, vec, train, test = load("tiny", "K3_s1")
    m = OracleModel()
    m.get_traintest(train, test)
    random.seed(meta["seed"])
    m.initialize_parameters(3)
    np.testing.assert_array_equal(np.array(m.theta), vec["theta_0"])
