"""bench.py's N-rank launch path on CPU: `--gpus 2` without a launcher starts two ranks (one per
GPU on the box; here gloo and no GPU work), and the end-of-run all-gather collects every rank's
samples (the reference's process-level sample parallelism, src/run.sh:36-45)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    return p


def test_gpus_2_launches_two_ranks_and_gathers():
    p = _run("--gpus", "2", "--backend", "gloo", "--launch-check", "--samples", "3")
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2
    assert rec["gathered_rows"] == 6 and rec["samples"] == list(range(6))


def test_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-check"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
