"""Generate the output-format pin by importing the REFERENCE implementation.

Run once in the build container (the reference is mounted read-only at /root/reference and
never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_output_golden.py

For a few (fold, K, seed) cases it runs 25 `make_iteration` calls on the reference `Model`,
sets `likelihood` the way the reference driver does before it writes a sample file (the train
likelihood of the last check, src/TrigenicInteractionPredictor.py:1269, then `to_file` :1275),
and stores the text of `to_string()` (:793-858) as ``output/<case>_K<K>_s<seed>.txt``.  These
files are data (the reference's output), not code: tests compare the drop-in `Model.to_string`
with them line by line.
"""
from __future__ import annotations

import contextlib
import io
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True

REF_SRC = "/root/reference/src"
# (case directory holding train.dat / test.dat, K, seed, iterations)
RUNS = [("small", 2, 1, 25), ("multi", 3, 4, 25), ("tiny", 10, 1, 25)]


def main():
    sys.path.insert(0, REF_SRC)
    import TrigenicInteractionPredictor as ref  # noqa: E402
    out_dir = os.path.join(HERE, "output")
    os.makedirs(out_dir, exist_ok=True)
    for case, K, seed, iters in RUNS:
        d = os.path.join(HERE, case)
        with contextlib.redirect_stdout(io.StringIO()):
            m = ref.Model()
            m.get_traintest(os.path.join(d, "train.dat"), os.path.join(d, "test.dat"))
        random.seed(seed)
        m.initialize_parameters(K)
        for _ in range(iters):
            m.make_iteration()
        m.compute_likelihood()                 # :1269 sets self.likelihood before :1275
        text = m.to_string()
        name = "%s_K%d_s%d.txt" % (case, K, seed)
        with open(os.path.join(out_dir, name), "w", encoding="utf-8") as f:
            f.write(text)
        print("  output/%s: %d lines" % (name, text.count("\n") + 1))


if __name__ == "__main__":
    main()
