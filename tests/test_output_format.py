"""Output-format pin on CPU: the drop-in `Model.to_string` (src/TrigenicInteractionPredictor.py
:793-858) against the text the REFERENCE wrote for the same model state
(tests/golden/output, made by tests/golden/make_output_golden.py).  The model state is the
reference's own theta / p after 25 iterations (the golden .npz); the two engine-backed calls
inside to_string (held-out likelihood, test-set predictions) are answered by the C oracle here
(this test covers the host formatting, ranking and metrics code; tests/test_gpu_output.py runs
the whole thing on the GPU)."""
import contextlib
import io
import os

import numpy as np
import pytest

from golden_util import GOLDEN, OUTPUT_CASES, compare_output, load, output_text
from oracle import c_oracle
from trigenicinteractionpredictor_amd.model import Model


@pytest.mark.parametrize("case,K,seed", OUTPUT_CASES)
def test_to_string_matches_reference_text(case, K, seed, monkeypatch):
    meta, vec, train, test = load(case, "K%d_s%d" % (K, seed))
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(train, test)
    m.K = K
    th, pr = vec["theta_25"], vec["pr_25"]
    m._theta, m._pr = th.tolist(), pr.tolist()
    m.likelihood = float(vec["L_25"])
    ids, counts = c_oracle.links_to_arrays(m.links)
    tids, tcounts = c_oracle.links_to_arrays(m.test_links)

    def compute_likelihood(selected_set="train"):
        a, c = (ids, counts) if selected_set == "train" else (tids, tcounts)
        v = c_oracle.loglik(a, c, th, pr)
        if selected_set == "train":
            m.likelihood = v
        else:
            m.heldoutlikelihood = v
        return v

    def calculate_test_set_results():
        probs = c_oracle.predict(tids, th, pr)
        m.results = sorted(([float(p), key, 0 if n[0] else 1]
                            for p, (key, n) in zip(probs, m.test_links.items())), reverse=True)

    monkeypatch.setattr(m, "compute_likelihood", compute_likelihood)
    monkeypatch.setattr(m, "calculate_test_set_results", calculate_test_set_results)
    compare_output(m.to_string(), output_text(case, K, seed))


def test_to_file_creates_the_file_before_formatting(tmp_path, monkeypatch):
    """The reference opens (creates / truncates) the output file before calling to_string
    (:898-899): when to_string raises, an empty file stays behind, and the CLI's resume rule
    (:1256) then skips that sample."""
    m = Model()

    def boom():
        raise ZeroDivisionError("float division by zero")

    monkeypatch.setattr(m, "to_string", boom)
    path = str(tmp_path / "Sample_0_K2.csv")
    with pytest.raises(ZeroDivisionError):
        m.to_file(path)
    assert os.path.isfile(path) and os.path.getsize(path) == 0
