"""The CLI driver on the GPU model: same iterations-to-convergence and output files as the
reference loop run on the oracle (src/TrigenicInteractionPredictor.py:1253-1279), and the
output header of `to_string` (:847-858) with the likelihoods within the parity tolerance."""
import contextlib
import io
import os

import numpy as np
import pytest

from test_cli import TEST, TRAIN, _reference_loop
from trigenicinteractionpredictor_amd import cli

pytestmark = pytest.mark.gpu


def test_cli_on_gpu_matches_reference_loop(tmp_path):
    out = str(tmp_path) + os.sep
    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(["-k", "3", "-i", "60", "-n", "2", "-f", "4", "-b", "6", "-t", TRAIN, "-e", TEST,
                       "-o", out, "--seed", "7"], out=lines.append)
    assert rc == 0
    ref = _reference_loop(3, 7, 2, 60, 4, 6)
    assert sum(1 for l in lines if l.startswith("· Iteration ")) == sum(r[1] for r in ref)
    for s, _, conv in ref:
        path = out + "Sample_%d_K3.csv" % s
        assert os.path.isfile(path) == conv
        if conv:
            text = open(path).read()
            assert text.startswith("Max Likelihood:\t")
            assert "Held-out Likelihood:\t" in text and "\nMetrics:\n" in text
            like = float(text.split("\n")[0].split("\t")[1])
            assert np.isfinite(like)


def test_cli_batch_mode_on_gpu_matches_reference_loop(tmp_path):
    """`--batch 2` (samples advanced together in one batched engine) against the sequential
    reference loop on the oracle: same iterations to convergence, same converged set, same file
    names; each file's header likelihood equals the oracle's at that iteration."""
    out = str(tmp_path) + os.sep
    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(["-k", "3", "-i", "60", "-n", "3", "-f", "4", "-b", "6", "-t", TRAIN, "-e", TEST,
                       "-o", out, "--seed", "7", "--batch", "2"], out=lines.append)
    assert rc == 0
    ref = _reference_loop(3, 7, 3, 60, 4, 6)
    got = [l for l in lines if l.startswith("Sample ") and "iterations" in l]
    assert [(int(l.split()[1][:-1]), int(l.split()[2])) for l in got] == [(s, it) for s, it, _ in ref]
    for s, _, conv in ref:
        path = out + "Sample_%d_K3.csv" % s
        assert os.path.isfile(path) == conv
        if conv:
            text = open(path).read()
            like = float(text.split("\n")[0].split("\t")[1])
            want = float([l for l in got if l.startswith("Sample %d:" % s)][0].split()[5])
            np.testing.assert_allclose(like, want, rtol=1e-12)
            assert "Held-out Likelihood:\t" in text and "\nTest set:\n" in text


def test_cli_gpus_2_on_one_gpu_writes_the_batch_files(tmp_path):
    """`--gpus 2 --backend gloo` (the command spawns its two ranks before any GPU call; on this
    one-GPU box both share cuda:0) writes the same Sample files, byte for byte, as one process
    with `--batch 2`: a sample's bits depend neither on its batch nor on its rank, and rank 0
    prints every sample's summary (src/run.sh:36-45, :1253-1279)."""
    import subprocess
    import sys
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    base = ["-k", "3", "-i", "60", "-n", "4", "-f", "4", "-b", "6", "-t", TRAIN, "-e", TEST, "--seed", "7"]
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(base + ["-o", str(one) + os.sep, "--batch", "2"], out=lambda *_: None)
    assert rc == 0
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-m", "trigenicinteractionpredictor_amd.cli", *base,
                        "-o", str(two) + os.sep, "--batch", "2", "--gpus", "2", "--backend", "gloo"],
                       cwd=repo, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    files = sorted(os.listdir(one))
    assert files and files == sorted(os.listdir(two))
    for f in files:
        assert (one / f).read_bytes() == (two / f).read_bytes(), f
    summary = [l for l in p.stdout.splitlines() if l.startswith("Sample ") and "iterations" in l]
    assert [int(l.split()[1][:-1]) for l in summary] == [0, 1, 2, 3]


@pytest.mark.parametrize("K,env", [(3, {"MMSBM_SK_Y": "1"})])
def test_cli_pool_writes_the_sequential_files(tmp_path, monkeypatch, K, env):
    """`--batch 8` over 16 samples (restarts.run_pool: converged slots refilled at once, the pool
    shrinking at the end) writes the Sample files of the sequential run (the drop-in Model, one
    sample at a time, :1253-1279) byte for byte.  One kernel family for both runs: SK_Y forced
    (the pool's family; the one-sample Model would take SK_U)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    seq, pool = tmp_path / "seq", tmp_path / "pool"
    seq.mkdir()
    pool.mkdir()
    base = ["-k", str(K), "-i", "80", "-n", "16", "-f", "4", "-b", "6", "-t", TRAIN, "-e", TEST, "--seed", "11"]
    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        assert cli.main(base + ["-o", str(seq) + os.sep], out=lines.append) == 0
        stats = {}
        orig = cli._pool

        def spy(*a, **k):
            from trigenicinteractionpredictor_amd.restarts import PoolStats
            st = PoolStats()
            res = orig(*a[:5], a[5], st)
            stats["s"] = st
            return res
        monkeypatch.setattr(cli, "_pool", spy)
        assert cli.main(base + ["-o", str(pool) + os.sep, "--batch", "8"], out=lambda *_: None) == 0
    files = sorted(os.listdir(seq))
    assert files and files == sorted(os.listdir(pool))
    for f in files:
        assert (seq / f).read_bytes() == (pool / f).read_bytes(), f
    st = stats["s"]
    assert st.refills >= 1 and st.slot_iterations == st.sample_iterations


def test_cli_default_batch_families_agree_within_tolerance(tmp_path, monkeypatch):
    """with the default environment a sequential run (the drop-in Model: one sample,
    SK_U) and a `--batch 4` run (SK_Y) sum in different orders, so their files are not byte
    equal; they converge after the same iterations and their likelihoods agree to the parity
    tolerance (the user-visible contract stated in the CLI help and README)."""
    for k in ("MMSBM_SK_Y", "MMSBM_SK_FUSED", "MMSBM_SK"):
        monkeypatch.delenv(k, raising=False)
    seq, bat = tmp_path / "seq", tmp_path / "bat"
    seq.mkdir()
    bat.mkdir()
    base = ["-k", "3", "-i", "80", "-n", "8", "-f", "4", "-b", "6", "-t", TRAIN, "-e", TEST, "--seed", "11"]
    l1, l2 = [], []
    with contextlib.redirect_stdout(io.StringIO()):
        assert cli.main(base + ["-o", str(seq) + os.sep], out=l1.append) == 0
        assert cli.main(base + ["-o", str(bat) + os.sep, "--batch", "4"], out=l2.append) == 0
    files = sorted(os.listdir(seq))
    assert files and files == sorted(os.listdir(bat))
    its = [l for l in l2 if l.startswith("Sample ") and "iterations" in l]
    assert sum(int(l.split()[2]) for l in its) == sum(1 for l in l1 if l.startswith("· Iteration "))
    for f in files:
        a, b = (seq / f).read_text().split("\n"), (bat / f).read_text().split("\n")
        assert len(a) == len(b)
        for x, y in zip(a[:2], b[:2]):  # Max / Held-out likelihood header lines
            np.testing.assert_allclose(float(x.split("\t")[1]), float(y.split("\t")[1]), rtol=1e-9)


@pytest.mark.parametrize("K,family", [(10, "sky"), (13, "auto")])
def test_pool_results_equal_single_sample_runs(tmp_path, K, family):
    """restarts.run_pool with 4 slots over 10 samples (refills, then shrinking): every sample's
    final theta / p / likelihood equals, bit for bit, a one-sample engine of the same family run
    for the same number of iterations, converged or not (the large-K case rarely converges on
    small data, so this compares parameters rather than files)."""
    import random
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
    from trigenicinteractionpredictor_amd.restarts import PoolStats, run_pool, stream_states
    tr, te = str(tmp_path / "tr.dat"), str(tmp_path / "te.dat")
    write_fold(FoldSpec(P=120, E=1500, seed=K), tr, te)
    m = Model()
    m.get_traintest(tr, te)

    def engine(B):
        e = EMEngine(K, m.P, B=B, family=family)
        e.set_links(0, *m._link_arrays(0))
        e.set_links(1, *m._link_arrays(1))
        return e
    random.seed(3)
    st = PoolStats()
    res = run_pool(engine(4), stream_states(m, K, range(10)), iterations=40, fcheck=3, bcheck=5,
                   keep_params=True, stats=st)
    assert sorted(r.sample for r in res) == list(range(10)) and st.refills == 6
    assert st.slot_iterations == sum(r.iterations for r in res)
    random.seed(3)
    init = {s: (th, pr) for s, th, pr in stream_states(m, K, range(10))}
    for r in res:
        one = engine(1)
        one.upload(init[r.sample][0][None], init[r.sample][1][None])
        one.iterate(r.iterations)
        th, pr = one.download()
        np.testing.assert_array_equal(th[0], r.theta)
        np.testing.assert_array_equal(pr[0], r.pr)
        assert one.loglik(0)[0] == r.loglik
