"""Self-spawned ranks for `cli.py --gpus N` and `bench.py --gpus N`: one OS process per GPU, as the
reference scales by one process per batch of samples (src/run.sh:36-45).

The parent starts the ranks before it touches a GPU, with the environment torch.distributed.run
would give them (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR / MASTER_PORT on
127.0.0.1), and waits on ALL of them at once: the first rank to fail has the survivors terminated
(they would otherwise sit in a barrier or collective until its timeout) and its exit code is
returned.  Pure Python, no torch import and no HIP call (visible_gpus reads sysfs): safe before
any GPU call.
"""
from __future__ import annotations

import glob
import os
import socket
import subprocess
import time


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    return dict(os.environ if base is None else base, RANK=str(rank), LOCAL_RANK=str(rank),
                WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port))


def wait_ranks(procs, poll_s: float = 0.05) -> int:
    """Wait for every process; on the first non-zero exit terminate the others.  Returns 0 or the
    first failure's code (a signal death -s as 128 + s)."""
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in alive:
                    q.terminate()
        if alive:
            time.sleep(poll_s)
    return rc


def spawn_ranks(cmd, n: int) -> int:
    """Start `cmd` (argv list) as ranks 0..n-1 of one process group and wait for them."""
    port = free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(r, n, port)) for r in range(n)]
    return wait_ranks(procs)


def visible_gpus():
    """GPUs this process may use, counted without touching HIP (the launcher runs this before it
    spawns the ranks, and must not initialise the GPU in the parent): the KFD topology nodes with
    a GPU id, capped by the *_VISIBLE_DEVICES lists the HIP runtime honours.  None when the
    topology is not readable (the ranks then check with the runtime's own count)."""
    files = glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")
    if not files:
        return None
    n = 0
    for f in files:
        try:
            with open(f) as fh:
                n += int(fh.read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n
