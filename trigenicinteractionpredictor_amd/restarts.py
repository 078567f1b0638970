"""Independent EM restarts ("samples") sharded across ranks — SURVEY.md §8e.

The reference runs samples one after another in one process (`__main__`,
src/TrigenicInteractionPredictor.py:1253-1279) and scales by launching more
processes (`src/run.sh:36-45`).  Here one process per GPU owns a contiguous
block of the global sample ids and advances all of them at once in one batched
engine (theta [B][P][K], p [B][R][K^3]); there is no per-iteration
communication.  At the end the per-sample results are gathered over the process
group (RCCL over xGMI for `nccl`, `gloo` in the CPU tests).

RNG: like the reference, one stdlib `random` stream is seeded once and every
sample's `initialize_parameters` consumes the next P*K + K^3*R draws, so
sample s gets the same initial state whether it runs alone, batched or on
another rank (a rank replays the draws of the samples before its block).

Per-sample driver semantics are the reference's (:1262-1279): initial
likelihood, then `make_iteration`; at iterations with `it % fcheck == 0 and
it > bcheck` the train likelihood is compared with the previous check and the
sample stops (converges) when |(L - L0) / L0| < 0.01.  A batched sample that
has converged keeps its snapshot; later batch iterations do not change it.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field

import numpy as np

TRAIN, TEST = 0, 1


def shard_samples(n_samples: int, world: int, rank: int) -> list[int]:
    """Contiguous, balanced block of global sample ids for `rank`."""
    base, extra = divmod(n_samples, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def init_samples(model, K: int, sample_ids: list[int], seed: int):
    """Initial (theta, pr) of each sample id; draws are consumed in global sample order."""
    random.seed(seed)
    want = set(sample_ids)
    thetas, prs = {}, {}
    for s in range(max(sample_ids) + 1 if sample_ids else 0):
        model.initialize_parameters(K)
        if s in want:
            thetas[s] = np.array(model._theta, dtype=np.float64)
            prs[s] = np.array(model._pr, dtype=np.float64)
    return [thetas[s] for s in sample_ids], [prs[s] for s in sample_ids]


@dataclass
class SampleResult:
    sample: int
    iterations: int
    converged: bool
    loglik: float
    heldout: float
    theta: np.ndarray = field(default=None, repr=False)
    pr: np.ndarray = field(default=None, repr=False)


def run_samples(engine, sample_ids, thetas, prs, iterations=10000, fcheck=25, bcheck=100,
                keep_params=False):
    """Drive the batched engine with the reference's per-sample convergence rule.

    `engine` provides upload(thetas, prs), iterate(n), loglik(which) -> [B], download().
    """
    B = len(sample_ids)
    engine.upload(np.stack(thetas), np.stack(prs))
    like0 = np.array(engine.loglik(TRAIN), dtype=np.float64)
    done = [None] * B
    it = 0
    while it < iterations and any(d is None for d in done):
        # next check iteration (reference checks right after make_iteration #it)
        nxt = it
        while nxt < iterations and not (nxt % fcheck == 0 and nxt > bcheck):
            nxt += 1
        n = min(nxt, iterations - 1) - it + 1
        engine.iterate(n)
        it += n
        if it - 1 == nxt and nxt < iterations:
            like = np.array(engine.loglik(TRAIN), dtype=np.float64)
            snap = None
            for s in range(B):
                if done[s] is not None:
                    continue
                if math.fabs((like[s] - like0[s]) / like0[s]) < 0.01:
                    if snap is None:
                        snap = engine.download() if keep_params else (None, None)
                        held = np.array(engine.loglik(TEST), dtype=np.float64)
                    done[s] = SampleResult(sample_ids[s], it, True, float(like[s]), float(held[s]),
                                           None if snap[0] is None else snap[0][s],
                                           None if snap[1] is None else snap[1][s])
                like0[s] = like[s]
    if any(d is None for d in done):
        like = np.array(engine.loglik(TRAIN), dtype=np.float64)
        held = np.array(engine.loglik(TEST), dtype=np.float64)
        snap = engine.download() if keep_params else (None, None)
        for s in range(B):
            if done[s] is None:
                done[s] = SampleResult(sample_ids[s], it, False, float(like[s]), float(held[s]),
                                       None if snap[0] is None else snap[0][s],
                                       None if snap[1] is None else snap[1][s])
    return done


def gather_results(results: list[SampleResult], n_samples: int, group=None, device=None):
    """All-gather (sample, iterations, converged, loglik, heldout) of every rank.

    One collective at the end of the run (no data-path communication); on GPU
    ranks with the nccl backend this is an RCCL all-gather over xGMI."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = -(-n_samples // world)
    buf = torch.full((width, 5), float("nan"), dtype=torch.float64)
    for i, r in enumerate(results):
        buf[i] = torch.tensor([r.sample, r.iterations, float(r.converged), r.loglik, r.heldout],
                              dtype=torch.float64)
    if device is not None:
        buf = buf.to(device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    rows = torch.cat(out).cpu().numpy()
    rows = rows[~np.isnan(rows[:, 0])]
    rows = rows[np.argsort(rows[:, 0], kind="stable")]
    return [SampleResult(int(r[0]), int(r[1]), bool(r[2]), float(r[3]), float(r[4])) for r in rows]


def run_restarts(model, K, n_samples, seed, iterations=10000, fcheck=25, bcheck=100,
                 engine_factory=None, group=None, device=None):
    """Shard `n_samples` restarts over the process group (or run all locally), drive them,
    and return every sample's result on every rank (sorted by sample id)."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    ids = shard_samples(n_samples, world, rank)
    local = []
    if ids:
        thetas, prs = init_samples(model, K, ids, seed)
        if engine_factory is None:
            from .engine import EMEngine
            from .layout import links_to_arrays

            def engine_factory(B):
                eng = EMEngine(K, model.P, B=B, R=model.R, eps=model.eps, device=device)
                eng.set_links(TRAIN, *links_to_arrays(model.links, model.R))
                eng.set_links(TEST, *links_to_arrays(model.test_links, model.R))
                return eng
        local = run_samples(engine_factory(len(ids)), ids, thetas, prs, iterations, fcheck, bcheck)
    if not dist_on:
        return local
    return gather_results(local, n_samples, group=group, device=device)


# ------------------------------------------------------------------ fixed-length runs (bench.py)
# bench.py runs every rank's block of samples for a fixed number of iterations (no convergence
# stop), gathers (sample id, final train log-likelihood) from every rank and, on rank 0, replays
# all samples as ONE batch on one engine: a sample's bits do not depend on its batch or its rank
# (DESIGN.md), so the gathered values must equal the replay bit for bit.  The digest names the
# per-sample results of a run, so runs at different GPU counts can be compared.

def fixed_run(engine, thetas, prs, iterations: int, chunks=()):
    """Upload, run `iterations` EM iterations (in the given chunk sizes when they are given),
    and return the final train log-likelihood of every sample."""
    engine.upload(np.stack(thetas), np.stack(prs))
    done = 0
    for n in chunks:
        engine.iterate(n)
        done += n
    if iterations > done:
        engine.iterate(iterations - done)
    return np.array(engine.loglik(TRAIN), dtype=np.float64)


def result_rows(sample_ids, loglik) -> np.ndarray:
    """[n][2] float64 rows (sample id, final log-likelihood)."""
    return np.stack([np.asarray(sample_ids, dtype=np.float64),
                     np.asarray(loglik, dtype=np.float64)], axis=1).reshape(-1, 2)


def gather_rows(rows: np.ndarray, n_samples: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's rows (one collective: RCCL all-gather over xGMI under nccl),
    sorted by sample id."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = -(-n_samples // world)
    buf = torch.full((width, 2), float("nan"), dtype=torch.float64)
    buf[:rows.shape[0]] = torch.from_numpy(np.ascontiguousarray(rows))
    if device is not None:
        buf = buf.to(device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    got = torch.cat(out).cpu().numpy()
    got = got[~np.isnan(got[:, 0])]
    return got[np.argsort(got[:, 0], kind="stable")]


def rows_digest(rows: np.ndarray) -> str:
    """sha256 (16 hex digits) of the rows sorted by sample id, as float64 bytes."""
    import hashlib
    r = np.ascontiguousarray(rows[np.argsort(rows[:, 0], kind="stable")], dtype=np.float64)
    return hashlib.sha256(r.tobytes()).hexdigest()[:16]


def replay_check(rows: np.ndarray, model, K: int, seed: int, iterations: int, engine_factory,
                 chunks=()) -> dict:
    """Replay every gathered sample as one batch (engine_factory(B)) from the same RNG stream and
    compare bit for bit.  -> {"samples", "digest", "replay_digest", "bitwise_equal"}."""
    ids = [int(s) for s in rows[:, 0]]
    thetas, prs = init_samples(model, K, ids, seed)
    L = fixed_run(engine_factory(len(ids)), thetas, prs, iterations, chunks)
    rep = result_rows(ids, L)
    return {"samples": len(ids), "digest": rows_digest(rows), "replay_digest": rows_digest(rep),
            "bitwise_equal": bool(np.array_equal(rows[:, 1].view(np.int64), rep[:, 1].view(np.int64)))}
