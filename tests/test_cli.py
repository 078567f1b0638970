"""The CLI driver (reference `__main__`, src/TrigenicInteractionPredictor.py:1148-1279): flag
parsing and validation, the check schedule, convergence, output naming and the skip-if-exists
resume rule — on CPU, with the oracle standing in for the GPU model."""
import contextlib
import io
import math
import os
import random

import pytest

from oracle.mmsbm_oracle import OracleModel
from trigenicinteractionpredictor_amd import cli

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny")
TRAIN, TEST = os.path.join(GOLD, "train.dat"), os.path.join(GOLD, "test.dat")


class OracleCliModel(OracleModel):
    """Oracle model with the drop-in's batch call and a minimal to_file (test stand-in)."""
    written = []

    def make_iterations(self, n):
        for _ in range(n):
            self.make_iteration()

    def to_file(self, name):
        with open(name, "w") as f:
            f.write("Max Likelihood:\t%r\n" % self.compute_likelihood())
        OracleCliModel.written.append(name)


def _reference_loop(K, seed, samples, iterations, f, b):
    """The reference __main__ per-sample loop (:1253-1279) on the oracle, one make_iteration at a
    time: (sample, iterations run, converged, final likelihood)."""
    m = OracleModel()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(TRAIN, TEST)
    random.seed(seed)
    out = []
    for s in range(samples):
        m.initialize_parameters(K)
        like0 = m.compute_likelihood()
        done = None
        for it in range(iterations):
            m.make_iteration()
            if it % f == 0 and it > b:
                like = m.compute_likelihood()
                if math.fabs((like - like0) / like0) < 0.01:
                    done = (s, it + 1, True)
                    break
                like0 = like
        out.append(done or (s, iterations, False))
    return out


def _run(argv):
    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(argv, model_factory=OracleCliModel, out=lines.append)
    return rc, lines


def test_check_points_follow_the_reference_condition():
    assert cli.check_points(10, 3, 4) == [6, 9]
    assert cli.check_points(200, 25, 100) == [125, 150, 175]
    assert cli.check_points(50, 51, 0) == []      # -f 0 with -i 50: never checks


def test_driver_matches_reference_loop(tmp_path):
    OracleCliModel.written = []
    out = str(tmp_path) + os.sep
    rc, lines = _run(["-k", "2", "-i", "40", "-n", "3", "-f", "3", "-b", "4", "-t", TRAIN,
                      "-e", TEST, "-o", out, "--seed", "5"])
    assert rc == 0
    ref = _reference_loop(2, 5, 3, 40, 3, 4)
    iters = [l for l in lines if l.startswith("· Iteration ")]
    assert len(iters) == sum(r[1] for r in ref)
    conv = [r for r in ref if r[2]]
    assert sorted(OracleCliModel.written) == sorted(out + "Sample_%d_K2.csv" % r[0] for r in conv)
    # resume: finished samples are skipped on a second run
    OracleCliModel.written = []
    rc, lines = _run(["-k", "2", "-i", "40", "-n", "3", "-f", "3", "-b", "4", "-t", TRAIN,
                      "-e", TEST, "-o", out, "--seed", "5"])
    assert rc == 0
    assert sum(1 for l in lines if l.startswith("Sample ")) == 3 - len(conv)


def test_fcheck_zero_never_writes(tmp_path):
    OracleCliModel.written = []
    rc, lines = _run(["-i", "8", "-f", "0", "-k", "2", "-n", "1", "-t", TRAIN, "-e", TEST,
                      "-o", str(tmp_path) + os.sep, "--seed", "1"])
    assert rc == 0 and OracleCliModel.written == []
    assert sum(1 for l in lines if l.startswith("· Iteration ")) == 8
    assert not any(l.startswith("· Likelihood ") for l in lines)


@pytest.mark.parametrize("argv", [["-i", "0"], ["-n", "0"], ["-s", "-1"], ["-f", "-1"], ["-b", "-2"],
                                  ["-k", "0"], ["-t", "/nonexistent.dat"], ["-o", "/nonexistent/"],
                                  ["-x"], ["-i", "abc"]])
def test_invalid_arguments_exit_2(argv):
    rc, _ = _run(argv)
    assert rc == 2


def test_help_exits_0():
    rc, _ = _run(["-h"])
    assert rc == 0


def test_batch_mode_matches_reference_loop(tmp_path):
    """--batch 2 on 3 samples (one full batch and a ragged one): same iterations to convergence,
    same converged set and output names as the sequential reference loop (:1253-1279); the batched
    engine is the C oracle here (tests/test_gpu_cli.py runs it on the GPU)."""
    from oracle_engine import OracleEngine
    from trigenicinteractionpredictor_amd.model import Model

    written = []

    class M(Model):
        def to_file(self, name_file=None):
            written.append((name_file, self.likelihood, [list(r) for r in self._theta]))

    out = str(tmp_path) + os.sep
    lines = []
    holder = {}

    def factory():
        holder["m"] = M()
        return holder["m"]

    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(["-k", "2", "-i", "40", "-n", "3", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST,
                       "-o", out, "--seed", "5", "--batch", "2"], model_factory=factory,
                      out=lines.append,
                      engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links))
    assert rc == 0
    ref = _reference_loop(2, 5, 3, 40, 3, 4)
    got = [l for l in lines if l.startswith("Sample ") and "iterations" in l]
    assert [(int(l.split()[1][:-1]), int(l.split()[2])) for l in got] == [(s, it) for s, it, _ in ref]
    assert [w[0] for w in written] == [out + "Sample_%d_K2.csv" % s for s, _, c in ref if c]


class _FileModel:
    """Model stand-in whose to_file writes the converged snapshot exactly (repr of every value),
    so two runs' files are equal byte for byte only when their results are."""

    @staticmethod
    def make():
        from trigenicinteractionpredictor_amd.model import Model

        class M(Model):
            def to_file(self, name_file=None):
                with open(name_file, "w") as f:
                    f.write("L %r\n" % self.likelihood)
                    f.write("theta %r\n" % [list(map(float, r)) for r in self._theta])
                    f.write("pr %r\n" % repr(self._pr))
        return M()


def _ranked_worker(rank, world, port, argv, queue):
    import torch.distributed as dist  # noqa: F401
    from oracle_engine import OracleEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    holder = {}

    def factory():
        holder["m"] = _FileModel.make()
        return holder["m"]

    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(argv + ["--gpus", str(world), "--backend", "gloo"], model_factory=factory,
                      out=lines.append,
                      engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links))
    queue.put((rank, rc, lines))


def test_two_rank_gloo_cli_writes_the_one_rank_files(tmp_path):
    """`--gpus 2` (two ranks, gloo, the C oracle as each rank's engine): the Sample_<n>_K<k>.csv
    files are byte-identical to a one-process `--batch` run's, and rank 0 prints every sample's
    summary line in sample order (src/run.sh:36-45, :1253-1279)."""
    import multiprocessing as mp

    from oracle_engine import OracleEngine
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    base = ["-k", "2", "-i", "40", "-n", "5", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST, "--seed", "5",
            "--batch", "2"]
    holder = {}

    def factory():
        holder["m"] = _FileModel.make()
        return holder["m"]

    lines1 = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(base + ["-o", str(one) + os.sep], model_factory=factory, out=lines1.append,
                      engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links))
    assert rc == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 250) % 1000
    argv = base + ["-o", str(two) + os.sep]
    procs = [ctx.Process(target=_ranked_worker, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (rc, lines) for r, rc, lines in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got[0][0] == 0 and got[1][0] == 0
    assert got[1][1] == []                                   # rank 1 prints nothing
    files1, files2 = sorted(os.listdir(one)), sorted(os.listdir(two))
    assert files1 and files1 == files2
    for f in files1:
        assert (one / f).read_bytes() == (two / f).read_bytes()
    summary = lambda ls: [l for l in ls if l.startswith("Sample ") and "iterations" in l]  # noqa: E731
    assert summary(got[0][1]) == summary(lines1)


def test_gpus_flag_validation():
    rc, _ = _run(["--gpus", "0"])
    assert rc == 2
    rc, _ = _run(["--gpus", "2", "--backend", "mpi"])
    assert rc == 2
