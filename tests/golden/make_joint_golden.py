"""Generate the joint digenic + trigenic parity fixtures by importing the REFERENCE
`src/TrigenicInteractionPredictor_23.py` (run once in the build container; the reference
never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_joint_golden.py

The reference's `Model()` raises `AttributeError: ALL` (:105): the enum at :31-34 defines
`all`, not `ALL`.  The spec fix ("Joint digenic + trigenic model") reads `ALL` as
`all`; this script applies exactly that, as a class attribute alias set before the first
`Model()`, and changes nothing else.  For every case it writes the fold files (inputs) and
one `.npz` per (K, seed) with theta / pr / qr / log-likelihood after 0, 1, 5, 25
`make_iteration` calls, the test-set prediction table and metrics, and the text of
`to_string_short()` / `to_string()` after the last snapshot (as the driver
`src/trigenic_fromtesttrain_2+3.py:74-98` would write it).
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from trigenicinteractionpredictor_amd.data import JointFoldSpec, write_joint_fold  # noqa: E402

REF_SRC = "/root/reference/src"

CASES = {
    # name: (spec, [(K, seed, iterations, interaction name)])
    "tiny": (JointFoldSpec(P=40, E3=150, E2=80, seed=21, pair_only=4, ho_frac=0.3,
                           multi_frac=0.1, both_frac=0.05, pos_frac=0.2, pair_pos_frac=0.3),
             [(1, 1, [0, 1, 5], "all"), (2, 1, [0, 1, 5, 25], "all"), (3, 2, [0, 1, 5, 25], "all"),
              (10, 1, [0, 1, 5, 25], "all"), (2, 4, [0, 1, 5], "trigenic"),
              (2, 5, [0, 1, 5], "digenic")]),
    "pairs": (JointFoldSpec(P=30, E3=0, E2=120, seed=22, pair_pos_frac=0.3, multi_frac=0.1),
              [(2, 3, [0, 1, 5, 25], "all"), (3, 1, [0, 1, 5, 25], "all")]),
    "small": (JointFoldSpec(P=200, E3=1200, E2=500, seed=23, pair_only=12, ho_frac=0.1,
                            pos_frac=0.1, pair_pos_frac=0.2),
              [(2, 1, [0, 1, 5, 25], "all"), (10, 1, [0, 1, 5], "all")]),
}


def _import_reference():
    sys.path.insert(0, REF_SRC)
    import TrigenicInteractionPredictor_23 as ref  # noqa: E402
    if not hasattr(ref.DataType, "ALL"):
        # spec fix for :105 / :194 / :209 / :296 — ALL is the member the code means by `all`
        type.__setattr__(ref.DataType, "ALL", ref.DataType.all)
    return ref


def _run_case(ref, case_dir, train, test, K, seed, iters, interaction):
    quiet = io.StringIO()
    with contextlib.redirect_stdout(quiet):
        m = ref.Model()
        m.get_train_test(train, test)
    random.seed(seed)
    m.initialize_parameters(K, getattr(ref.DataType, interaction))
    out = {}
    done = 0
    for it in iters:
        while done < it:
            m.make_iteration()
            done += 1
        out["theta_%d" % it] = np.array(m.theta, dtype=np.float64)
        out["pr_%d" % it] = np.array(m.pr, dtype=np.float64)
        out["qr_%d" % it] = np.array(m.qr, dtype=np.float64)
        out["L_%d" % it] = np.float64(m.compute_likelihood())
        m.likelihoodVector.append([0, it, float(out["L_%d" % it])])
    m.calculate_test_set_results()
    out["pred"] = np.array([row[0] for row in m.results], dtype=np.float64)
    out["pred_key"] = np.array([row[1] for row in m.results])
    out["pred_real"] = np.array([row[2] for row in m.results], dtype=np.int64)
    try:
        out["metrics"] = np.array(m.calculate_metrics(), dtype=np.float64)
    except ZeroDivisionError:
        out["metrics"] = np.array([np.nan] * 4)
    texts = {}
    for name in ("to_string_short", "to_string"):
        try:
            texts[name] = getattr(m, name)()
        except ZeroDivisionError:
            texts[name] = None
    meta = {
        "K": K, "seed": seed, "iters": iters, "interaction": interaction, "P": m.P,
        "links": list(m.links.items()), "dlinks": list(m.dlinks.items()),
        "test_links": list(m.test_links.items()), "dtest_links": list(m.dtest_links.items()),
        "id_gene": [m.id_gene[i] for i in range(m.P)],
        "gene_num_aparitions": [m.gene_num_aparitions[i] for i in range(m.P)],
        "text": texts,
    }
    name = "K%d_s%d" % (K, seed)
    np.savez_compressed(os.path.join(case_dir, name + ".npz"), **out)
    with open(os.path.join(case_dir, name + ".json"), "w", encoding="utf-8") as f:
        json.dump(meta, f, ensure_ascii=False)
    print("  joint/%s/%s: L_final=%r" % (os.path.basename(case_dir), name, float(out["L_%d" % iters[-1]])))


CLI_RUNS = [  # (name, argv of src/trigenic_fromtesttrain_2+3.py without the files, seed)
    ("v0", [80, 2, 5, 2, 3], 0, 77),
    ("v1", [400, 2, 10, 2, 0], 1, 78),
]


def _run_driver(ref, case_dir, out_dir):
    """The loop of src/trigenic_fromtesttrain_2+3.py:65-107 on the reference Model, with the spec
    fix (likelihoodVector for :78/:86's vlikelihood), seed given instead of os.getpid() (:32).
    Records stdout and every output file."""
    import math
    train, test = os.path.join(case_dir, "train.dat"), os.path.join(case_dir, "test.dat")
    runs = {}
    for name, (iterations, samples, fcheck, k, sampleini), verbose, seed in CLI_RUNS:
        d = os.path.join(out_dir, name)
        os.makedirs(d, exist_ok=True)
        cwd = os.getcwd()
        os.chdir(d)
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                random.seed(seed)
                msg = "\n****************************************\n* Trigenic Interaction Predictor v 1.0 *\n**************"
                msg += "**************************\n\nDoing " + str(samples) + " samples of " + str(iterations) + " num_iterations."
                msg += "**************************\n\nStarting from sample " + str(sampleini) + " ."
                msg += "\nLikelihood will be calculated every " + str(fcheck) + " num_iterations."
                print(msg)
                model = ref.Model()
                model.get_train_test(train, test)
                print("\nStarting algorithm...")
                print(verbose)
                for sample in range(sampleini, sampleini + int(samples)):
                    print("Sample " + str(1 + sample) + ":")
                    model.initialize_parameters(k)
                    print("Parameters have been initialized")
                    like0 = model.compute_likelihood()
                    print("· Likelihood 0 is " + str(like0))
                    model.likelihoodVector.append([sample, 0, like0])
                    for iteration in range(iterations):
                        model.make_iteration()
                        if iteration % fcheck == 0:
                            like = model.compute_likelihood()
                            print("· Likelihood " + str(iteration + 1) + " is " + str(like))
                            model.likelihoodVector.append([sample, iteration + 1, like])
                            if math.fabs((like - like0) / like0) < 0.001:
                                print("\n\t****************************\n\t* Likelihood has converged *\n\t****************************")
                                outfile = 'outSamp%dK%d.csv' % (sample, k)
                                if verbose == 0:
                                    model.to_file_short(outfile)
                                elif verbose == 1:
                                    model.to_file(outfile)
                                break
                            like0 = like
            files = {f: open(f, encoding="utf-8").read() for f in sorted(os.listdir("."))}
        finally:
            os.chdir(cwd)
        for f in files:
            os.remove(os.path.join(d, f))
        os.rmdir(d)
        runs[name] = {"argv": [str(x) for x in (iterations, samples, fcheck, k, sampleini)] + [verbose, seed],
                      "stdout": buf.getvalue(), "files": files}
        print("  joint/cli/%s: files %s" % (name, sorted(files)))
    with open(os.path.join(out_dir, "driver.json"), "w", encoding="utf-8") as f:
        json.dump(runs, f, ensure_ascii=False)


def main():
    ref = _import_reference()
    if "--cli-only" in sys.argv:
        _run_driver(ref, os.path.join(HERE, "joint", "tiny"), os.path.join(HERE, "joint", "cli"))
        return
    root = os.path.join(HERE, "joint")
    for case, (spec, runs) in CASES.items():
        d = os.path.join(root, case)
        os.makedirs(d, exist_ok=True)
        train, test = os.path.join(d, "train.dat"), os.path.join(d, "test.dat")
        write_joint_fold(spec, train, test)
        for K, seed, iters, interaction in runs:
            _run_case(ref, d, train, test, K, seed, iters, interaction)
    # zero degree: a gene seen only in the test file -> ZeroDivisionError in make_iteration (:1642)
    d = os.path.join(root, "tiny")
    zt = os.path.join(d, "test_zerodeg.dat")
    with open(os.path.join(d, "test.dat"), encoding="utf-8") as f:
        lines = f.readlines()
    with open(zt, "w", encoding="utf-8") as f:
        f.writelines(lines + ["g00000_zz999\t1\n"])
    with contextlib.redirect_stdout(io.StringIO()):
        m = ref.Model()
        m.get_train_test(os.path.join(d, "train.dat"), zt)
    random.seed(9)
    m.initialize_parameters(2)
    L0 = m.compute_likelihood()
    try:
        m.make_iteration()
        raised = False
    except ZeroDivisionError:
        raised = True
    with open(os.path.join(root, "zerodeg.json"), "w") as f:
        json.dump({"K": 2, "seed": 9, "P": m.P, "L_0": L0, "raises_zero_division": raised}, f)
    print("  joint/zerodeg: raises=%s" % raised)
    _run_driver(ref, os.path.join(root, "tiny"), os.path.join(root, "cli"))


if __name__ == "__main__":
    main()
