"""Helpers to enumerate and load the committed golden fixtures (data only)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    out = []
    for meta_path in sorted(glob.glob(os.path.join(GOLDEN, "*", "K*_s*.json"))):
        case_dir = os.path.dirname(meta_path)
        name = os.path.basename(meta_path)[:-5]
        out.append((os.path.basename(case_dir), name))
    return out


def load(case, name):
    d = os.path.join(GOLDEN, case)
    with open(os.path.join(d, name + ".json")) as f:
        meta = json.load(f)
    vec = np.load(os.path.join(d, name + ".npz"), allow_pickle=False)
    return meta, vec, os.path.join(d, "train.dat"), os.path.join(d, "test.dat")


OUTPUT_CASES = [("small", 2, 1), ("multi", 3, 4), ("tiny", 10, 1)]


def output_text(case, K, seed):
    """The reference's `to_string()` after 25 iterations (tests/golden/make_output_golden.py)."""
    with open(os.path.join(GOLDEN, "output", "%s_K%d_s%d.txt" % (case, K, seed)),
              encoding="utf-8") as f:
        return f.read()


def _floats(s):
    return [float(x) for x in s.split("\t")]


def compare_output(got, want, rtol=1e-9, gap=1e-7):
    """Line-by-line comparison of two `to_string()` texts (src/TrigenicInteractionPredictor.py
    :847-858): labels, counts, keys and real ratings exactly; likelihoods, metrics and predicted
    probabilities within `rtol`.  The test-set table is sorted by probability; where two
    reference probabilities are closer than `gap` (relative) their order is not determined by
    the algorithm (FP64 re-association), so only the multiset of rows is checked there."""
    import numpy as np
    g, w = got.split("\n"), want.split("\n")
    assert len(g) == len(w), (len(g), len(w))
    head = w.index("Predicted Interaction\tID of genes\tReal Interaction")
    for i in range(head + 1):
        if w[i].startswith(("Max Likelihood:\t", "Held-out Likelihood:\t")):
            lg, vg = g[i].split("\t")
            lw, vw = w[i].split("\t")
            assert lg == lw
            np.testing.assert_allclose(float(vg), float(vw), rtol=rtol)
        elif i > 0 and w[i - 1] == "Precision\tRecall\tFallout\tAUC":
            np.testing.assert_allclose(_floats(g[i]), _floats(w[i]), rtol=rtol)
        else:
            assert g[i] == w[i], (i, g[i], w[i])
    rows_g = [r.split("\t") for r in g[head + 1:] if r]
    rows_w = [r.split("\t") for r in w[head + 1:] if r]
    assert len(rows_g) == len(rows_w)
    pw = np.array([float(r[0]) for r in rows_w])
    pg = np.array([float(r[0]) for r in rows_g])
    np.testing.assert_allclose(pg, pw, rtol=rtol, atol=1e-300)
    # rows whose probability is isolated (both neighbours farther than `gap`) sit at the same place
    n = len(rows_w)
    for i in range(n):
        lo = i == 0 or abs(pw[i] - pw[i - 1]) > gap * abs(pw[i])
        hi = i == n - 1 or abs(pw[i] - pw[i + 1]) > gap * abs(pw[i])
        if lo and hi:
            assert rows_g[i][1:] == rows_w[i][1:], (i, rows_g[i], rows_w[i])
    assert sorted(tuple(r[1:]) for r in rows_g) == sorted(tuple(r[1:]) for r in rows_w)


# ---- joint digenic + trigenic fixtures (tests/golden/make_joint_golden.py) ----
JOINT = os.path.join(GOLDEN, "joint")


def joint_cases():
    out = []
    for meta_path in sorted(glob.glob(os.path.join(JOINT, "*", "K*_s*.json"))):
        out.append((os.path.basename(os.path.dirname(meta_path)), os.path.basename(meta_path)[:-5]))
    return out


def joint_load(case, name):
    d = os.path.join(JOINT, case)
    with open(os.path.join(d, name + ".json"), encoding="utf-8") as f:
        meta = json.load(f)
    vec = np.load(os.path.join(d, name + ".npz"), allow_pickle=False)
    return meta, vec, os.path.join(d, "train.dat"), os.path.join(d, "test.dat")
