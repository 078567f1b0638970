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
from trigenicinteractionpredictor_amd.launch import free_port
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
                      engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links, B=n))
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


def _ranked_worker(rank, world, port, argv, queue, pid=None, dump_s=None):
    import faulthandler
    faulthandler.enable()  # (a rank that dies on a signal prints where)
    if dump_s:  # a rank still running near the parent's deadline prints where it is (stderr)
        faulthandler.dump_traceback_later(dump_s)
    import torch.distributed as dist  # noqa: F401
    from oracle_engine import OracleEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    real_getpid = os.getpid
    if pid is not None:                       # each rank's default seed (:1149) differs
        os.getpid = lambda: pid + rank
    holder = {}

    def factory():
        holder["m"] = _FileModel.make()
        return holder["m"]

    lines = []
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            rc = cli.main(argv + ["--gpus", str(world), "--backend", "gloo"], model_factory=factory,
                          out=lines.append,
                          engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links, B=n))
    finally:
        # the real pid again before the queue is used: multiprocessing's queue decides from
        # os.getpid() whether this process must flush its feeder thread at exit (with the fake pid
        # both ranks sometimes exited 0 without their result reaching the parent)
        os.getpid = real_getpid
    queue.put((rank, rc, lines))


def _run_ranks(world, argv, timeout, pid=None):
    """`world` gloo ranks of cli.main (spawned processes) -> {rank: (rc, lines)}; ranks still alive
    when the results are in (or when collecting them fails) are terminated, so a failing test leaves
    no process behind."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()  # (a pid-derived port collided with another xdist worker's test)
    procs = [ctx.Process(target=_ranked_worker, args=(r, world, port, argv, q, pid, timeout - 20))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            try:
                r, rc, lines = q.get(timeout=timeout)
            except Exception as e:  # (which ranks are still running, and how the others ended)
                states = [(p.pid, p.is_alive(), p.exitcode) for p in procs]
                raise AssertionError("ranks did not report: %r (pid, alive, exitcode): %r" % (e, states))
            got[r] = (rc, lines)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        return got
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(10)


def _pool_run(argv, out_dir, engines=None):
    """One-process cli.main with the C oracle as the pool's engine; returns (rc, lines)."""
    from oracle_engine import OracleEngine
    holder = {}

    def factory():
        holder["m"] = _FileModel.make()
        return holder["m"]

    def eng(n):
        e = OracleEngine(holder["m"].links, holder["m"].test_links, B=n)
        if engines is not None:
            engines.append(e)
        return e
    lines = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(argv + ["-o", str(out_dir) + os.sep], model_factory=factory, out=lines.append,
                      engine_factory=eng)
    return rc, lines


def test_pool_refills_converged_slots_and_matches_the_sequential_loop(tmp_path):
    """--batch 4 over 16 samples (restarts.run_pool): a converged sample's slot goes to the next
    pending sample at once, the slots shrink when nothing is pending, and the files equal a
    16-slot run's (no refill) byte for byte; iterations and convergence per sample are the
    sequential reference loop's (:1253-1279)."""
    base = ["-k", "2", "-i", "60", "-n", "16", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST, "--seed", "8"]
    a, b = tmp_path / "b4", tmp_path / "b16"
    a.mkdir()
    b.mkdir()
    engines = []
    rc, lines4 = _pool_run(base + ["--batch", "4"], a, engines)
    assert rc == 0 and len(engines) == 1 and engines[0].B == 4
    rc, lines16 = _pool_run(base + ["--batch", "16"], b)
    assert rc == 0
    ref = _reference_loop(2, 8, 16, 60, 3, 4)
    summary = lambda ls: [l for l in ls if l.startswith("Sample ") and "iterations" in l]  # noqa: E731
    got = [(int(l.split()[1][:-1]), int(l.split()[2])) for l in summary(lines4)]
    assert got == [(s, it) for s, it, _ in ref]
    assert summary(lines4) == summary(lines16)
    files = sorted(os.listdir(a))
    assert files == sorted("Sample_%d_K2.csv" % s for s, _, c in ref if c) and files
    assert files == sorted(os.listdir(b))
    for f in files:
        assert (a / f).read_bytes() == (b / f).read_bytes()
    log = engines[0].log
    # the pool never iterates a finished sample: slot-iterations = the samples' own iterations
    slot_its = sum(n * live for kind, n, *rest in log if kind == "iterate" for live in rest)
    assert slot_its == sum(it for _, it, _ in ref)
    shrinks = [n for kind, n, *rest in log if kind == "active"]
    assert shrinks[0] == 4 and shrinks[-1] >= 1 and sorted(shrinks, reverse=True) == shrinks


def test_two_rank_gloo_cli_writes_the_one_rank_files(tmp_path):
    """`--gpus 2` (two ranks, gloo, the C oracle as each rank's engine) with a 4-slot pool per
    rank over 16 samples: the Sample_<n>_K<k>.csv files are byte-identical to a one-process
    `--batch 4` run's, and rank 0 prints every sample's summary line in sample order (VERDICT r3
    item 5, r4 item 2; src/run.sh:36-45, :1253-1279)."""

    from oracle_engine import OracleEngine
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    base = ["-k", "2", "-i", "40", "-n", "16", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST, "--seed", "5",
            "--batch", "4"]
    holder = {}

    def factory():
        holder["m"] = _FileModel.make()
        return holder["m"]

    lines1 = []
    with contextlib.redirect_stdout(io.StringIO()):
        rc = cli.main(base + ["-o", str(one) + os.sep], model_factory=factory, out=lines1.append,
                      engine_factory=lambda n: OracleEngine(holder["m"].links, holder["m"].test_links, B=n))
    assert rc == 0
    got = _run_ranks(2, base + ["-o", str(two) + os.sep], 240)
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


def test_two_ranks_without_seed_replay_rank0_stream(tmp_path):
    """under an external launcher a rank given no --seed seeds from its own pid (:1149);
    the ranks take rank 0's seed, so the files equal a one-process run seeded with it."""
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    base = ["-k", "2", "-i", "40", "-n", "6", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST, "--batch", "2"]
    rc, lines1 = _pool_run(base + ["--seed", "4100"], one)
    assert rc == 0
    got = _run_ranks(2, base + ["-o", str(two) + os.sep], 240, pid=4100)
    assert got[0][0] == 0 and got[1][0] == 0
    files = sorted(os.listdir(one))
    assert files and files == sorted(os.listdir(two))
    for f in files:
        assert (one / f).read_bytes() == (two / f).read_bytes()


def test_first_failing_rank_ends_the_launch():
    """the self-spawn launcher watches every rank; when rank 1 exits 1 while rank 0
    would wait (in a barrier, here a sleep), rank 0 is terminated and the launch returns 1 at
    once instead of after rank 0's timeout."""
    import sys
    import time

    from trigenicinteractionpredictor_amd.launch import spawn_ranks
    t0 = time.time()
    rc = spawn_ranks([sys.executable, "-c", "import os, sys, time\n"
                      "sys.exit(1) if os.environ['RANK'] == '1' else time.sleep(120)"], 2)
    assert rc == 1 and time.time() - t0 < 30


def test_nccl_ranks_beyond_visible_gpus_are_refused(monkeypatch):
    """with the nccl backend --gpus above the visible GPUs is exit code 2 (RCCL takes
    one GPU per rank); gloo may share."""
    from trigenicinteractionpredictor_amd import launch
    monkeypatch.setattr(launch, "visible_gpus", lambda: 1)
    rc, lines = _run(["--gpus", "2", "-t", TRAIN, "-e", TEST, "-k", "2"])
    assert rc == 2 and any("visible" in l for l in lines)


def test_eight_rank_gloo_cli_config3_topology(tmp_path):
    """BASELINE config 3's topology on CPU: 64 restarts, `--batch 8`, eight
    gloo ranks (one per GPU of the node in the real run), the C oracle as each rank's engine and
    the reference's check schedule / convergence rule (:1262-1279).  The Sample files equal a
    one-process `--batch 8` run's byte for byte, rank 0's gathered summary lists all 64 samples
    in sample order, and the other ranks print nothing (src/run.sh:36-45, :1253-1279)."""
    one, eight = tmp_path / "one", tmp_path / "eight"
    one.mkdir()
    eight.mkdir()
    base = ["-k", "3", "-i", "40", "-n", "64", "-f", "3", "-b", "4", "-t", TRAIN, "-e", TEST, "--seed", "20",
            "--batch", "8"]
    rc, lines1 = _pool_run(base, one)
    assert rc == 0
    got = _run_ranks(8, base + ["-o", str(eight) + os.sep], 400)
    assert all(got[r][0] == 0 for r in range(8))
    assert all(got[r][1] == [] for r in range(1, 8))
    summary = lambda ls: [l for l in ls if l.startswith("Sample ") and "iterations" in l]  # noqa: E731
    s8 = summary(got[0][1])
    assert [int(l.split()[1][:-1]) for l in s8] == list(range(64))
    assert s8 == summary(lines1)
    files = sorted(os.listdir(one))
    assert files and files == sorted(os.listdir(eight))
    for f in files:
        assert (one / f).read_bytes() == (eight / f).read_bytes()
