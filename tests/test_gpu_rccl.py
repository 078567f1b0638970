"""RCCL on the one GPU of the test box: a world-size-1 `nccl` process group
created with `device_id`, as bench.py / cli.py create it for N ranks, then every collective the
multi-GPU paths issue — the device all-gather of the result rows (restarts.gather_rows /
gather_results), the replay check, and the link-shard all-reduce of the P*K + K^3*R accumulator
buffer (linkshard.LinkShardedEM).  A world of one makes each collective an identity, so the
results must equal the plain single-GPU runs bit for bit; what is exercised is RCCL itself
(communicator init on the MI355X, device buffers, the stream handshake).

The reference has no collective: its samples are separate OS processes (src/run.sh:36-45,
src/TrigenicInteractionPredictor.py:1253-1279) and its accumulation is one loop (:986-1028)."""
import contextlib
import io
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dev
    dist.barrier()
    dist.destroy_process_group()


def _model(tmp_path):
    from trigenicinteractionpredictor_amd import Model
    from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
    tr, te = str(tmp_path / "train.dat"), str(tmp_path / "test.dat")
    write_fold(FoldSpec(P=300, E=6000, seed=21), tr, te)
    m = Model()
    with contextlib.redirect_stdout(io.StringIO()):
        m.get_traintest(tr, te)
    return m


def _factory(m, K, dev):
    from trigenicinteractionpredictor_amd import EMEngine

    def make(B):
        e = EMEngine(K, m.P, B=B, device=dev)
        e.set_links(0, *m._link_arrays(0))
        e.set_links(1, *m._link_arrays(1))
        return e
    return make


def test_rccl_gather_rows_and_replay(nccl_group, tmp_path):
    """fixed_run -> gather_rows over RCCL (device buffers) -> replay_check, as bench.py's N-rank
    path runs them: the gathered rows are the local rows and the replay is bitwise equal."""
    from trigenicinteractionpredictor_amd.restarts import (fixed_run, gather_rows, init_samples,
                                                           replay_check, result_rows, rows_digest)
    dev = nccl_group
    m = _model(tmp_path)
    ids = [0, 1, 2]
    th, pr = init_samples(m, 10, ids, seed=4)
    make = _factory(m, 10, dev)
    L = fixed_run(make(3), th, pr, 7, chunks=(2, 1))
    rows = result_rows(ids, L)
    got = gather_rows(rows, 3, device=dev)
    assert np.array_equal(got.view(np.int64), rows.view(np.int64))
    chk = replay_check(got, m, 10, 4, 7, make)
    assert chk["bitwise_equal"] and chk["digest"] == rows_digest(rows)


def test_rccl_restart_driver_gather_results(nccl_group, tmp_path):
    """restarts.run_restarts with the group initialised: the per-sample results travel through
    gather_results' RCCL all-gather and equal the driver run without a group."""
    import torch.distributed as dist
    from trigenicinteractionpredictor_amd.restarts import init_samples, run_samples, run_restarts
    dev = nccl_group
    m = _model(tmp_path)
    got = run_restarts(m, 4, 3, seed=6, iterations=40, fcheck=5, bcheck=10,
                       engine_factory=_factory(m, 4, dev), device=dev)
    assert dist.is_initialized()
    th, pr = init_samples(m, 4, [0, 1, 2], seed=6)
    want = run_samples(_factory(m, 4, dev)(3), [0, 1, 2], th, pr, 40, 5, 10)
    assert [(g.sample, g.iterations, g.converged, g.loglik, g.heldout) for g in got] == \
           [(w.sample, w.iterations, w.converged, w.loglik, w.heldout) for w in want]


@pytest.mark.parametrize("K", [10, 20])
def test_rccl_linkshard_allreduce_equals_plain_iteration(nccl_group, tmp_path, K):
    """LinkShardedEM with the group up issues one RCCL all-reduce of the P*K + K^3*R buffer per
    iteration (world 1: an identity); theta / p / L equal the plain engine's bit for bit."""
    from trigenicinteractionpredictor_amd.linkshard import LinkShardedEM
    from trigenicinteractionpredictor_amd.restarts import init_samples
    dev = nccl_group
    m = _model(tmp_path)
    th, pr = init_samples(m, K, [0, 1], seed=2)
    make = _factory(m, K, dev)
    ids, counts = m._link_arrays(0)
    tids, tcounts = m._link_arrays(1)
    from trigenicinteractionpredictor_amd import EMEngine
    runner = LinkShardedEM(EMEngine(K, m.P, B=2, device=dev), ids, counts, tids, tcounts)
    assert runner.dist_on and runner.world == 1 and runner.buf.is_cuda
    runner.upload(np.stack(th), np.stack(pr))
    runner.iterate(3)
    t1, p1 = runner.download()
    L1 = runner.loglik(0)
    # the plain path: accumulate + mstep without a collective gives the same sums as fin; the
    # same split on the plain engine is the reference for the bits
    plain = make(2)
    plain.upload(np.stack(th), np.stack(pr))
    import torch
    nth = torch.zeros((2, m.P, K), dtype=torch.float64, device=dev)
    S = torch.zeros((2, 2, K ** 3), dtype=torch.float64, device=dev)
    for _ in range(3):
        plain.accumulate(nth, S)
        plain.mstep(nth, S)
    t2, p2 = plain.download()
    assert np.array_equal(t1.view(np.int64), t2.view(np.int64))
    assert np.array_equal(p1.view(np.int64), p2.view(np.int64))
    assert np.array_equal(np.asarray(L1).view(np.int64), plain.loglik(0).view(np.int64))


def _bench(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_bench_process_group_one_gpu():
    """bench.py --gpus 1 --process-group: the nccl init with device_id (bench.py's N-rank line),
    the RCCL gather of the rows and the replay check on the one GPU."""
    rec = _bench("--process-group", "--samples", "2", "--steps", "5", "--warmup", "2",
                 "--no-cpu-baseline", "--roofline-launches", "5")
    assert rec["process_group"] == "nccl" and rec["world_size"] == 1
    assert rec["gathered_samples"] == 2
    assert rec["samples"]["replay_check"]["bitwise_equal"]


def test_bench_process_group_link_shard_one_gpu():
    """bench.py --gpus 1 --process-group --shard links: one RCCL all-reduce per iteration."""
    rec = _bench("--process-group", "--shard", "links", "--K", "20", "--steps", "3", "--warmup", "1",
                 "--no-cpu-baseline", "--roofline-launches", "3")
    assert rec["process_group"] == "nccl" and rec["scaling"] == "strong"
    assert np.isfinite(rec["final_loglik"])
