"""Generate the ingestion fixtures (tests/golden/ingest.json) by running the REFERENCE's
`Model.get_traintest` (src/TrigenicInteractionPredictor.py:321-423) on small fold files.

Run once in the build container (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ingest_golden.py

Each case stores its input texts and the reference's resulting tables (P, id_gene, uniqueg,
links, nlinks, test_links in insertion order), its printed lines, and the exception it let
propagate, if any.  tests/test_ingest.py replays the inputs through the build's Model (native
reader or its Python fallback) and compares everything.
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
OUT = os.path.join(HERE, "ingest.json")


def random_fold(seed, n_lines=300, n_genes=40, n_test=60):
    rng = random.Random(seed)
    names = ["g%d" % rng.randrange(10 ** rng.randrange(1, 4)) for _ in range(n_genes)]
    names += ["a b", "x-1", "Z", "0"]
    lines = []
    for _ in range(n_lines):
        g = [rng.choice(names) for _ in range(3)]          # repeated genes in a triple allowed
        r = rng.choice(["0", "1", "01", "+1", " 0 ", "1 "])
        lines.append("%s\t%s" % ("_".join(g), r))
    train = "".join((" " if rng.random() < 0.1 else "") + ln + ("\t" if rng.random() < 0.1 else "")
                    + "\n" for ln in lines[n_test:])
    if seed % 2:
        train = train.rstrip("\n")                          # last line without its newline
    test = "".join(ln + "\n" for ln in lines[:n_test])
    return train, test


CASES = [("random%d" % s,) + random_fold(s) for s in range(6)] + [
    ("crlf", "a_b_c\t1\r\nd_e_f\t0\r\n", "a_b_d\t1\n"),
    ("four_genes", "a_b_c_d\t1\n", "a_b_c\t0\n"),
    ("two_genes", "a_b\t1\n", "a_b_c\t0\n"),
    ("rating_2", "a_b_c\t2\n", "a_b_c\t0\n"),
    ("rating_minus1", "a_b_c\t-1\n", "a_b_c\t0\n"),
    ("blank_line", "a_b_c\t1\n\nd_e_f\t0\n", "a_b_c\t0\n"),
    ("value_error", "a_b_c\tx\nd_e_f\t0\n", "a_b_c\t0\n"),
    ("underscore_int", "a_b_c\t1_0\n", "a_b_c\t0\n"),
    ("empty_test_rating", "a_b_c\t1\n", "a_b_c\t\n"),
    ("test_no_tab", "a_b_c\t1\n", "a_b_c 0\n"),
    ("non_ascii", "é_b_c\t1\n", "a_b_c\t0\n"),
    ("vt_separator", "a_b_c\t1\x0bd_e_f\t0\n", "a_b_c\t0\n"),
    ("ids_ge_10", "".join("g%02d_g%02d_g%02d\t%d\n" % (i, i + 1, i + 2, i % 2) for i in range(14)),
     "g00_g05_g13\t1\ng12_g00_g07\t0\n"),
    ("test_only_gene", "a_b_c\t1\n", "a_b_zz\t0\n"),
    ("empty_files", "", ""),
]


def run_reference(train_text, test_text):
    sys.path.insert(0, REF_SRC)
    import TrigenicInteractionPredictor as ref
    with tempfile.TemporaryDirectory() as d:
        tr, te = os.path.join(d, "train.dat"), os.path.join(d, "test.dat")
        for p, t in ((tr, train_text), (te, test_text)):
            with open(p, "w", encoding="utf-8", newline="") as f:
                f.write(t)
        m = ref.Model()
        out = io.StringIO()
        err = None
        with contextlib.redirect_stdout(out):
            try:
                m.get_traintest(tr, te)
            except Exception as e:  # noqa: BLE001 - the reference lets these propagate
                err = [type(e).__name__, str(e)]
    return {"stdout": out.getvalue(), "error": err, "P": m.P,
            "id_gene": [m.id_gene[i] for i in range(len(m.id_gene))],
            "uniqueg": [m.uniqueg[i] for i in range(len(m.uniqueg))],
            "links": [[k, v] for k, v in m.links.items()],
            "nlinks": [[k, v] for k, v in m.nlinks.items()],
            "test_links": [[k, v] for k, v in m.test_links.items()]}


def main():
    out = []
    for name, tr, te in CASES:
        out.append({"name": name, "train": tr, "test": te, "ref": run_reference(tr, te)})
    with open(OUT, "w", encoding="utf-8") as f:
        json.dump(out, f, indent=0, ensure_ascii=True)
    print("wrote", OUT, len(out), "cases")


if __name__ == "__main__":
    main()
