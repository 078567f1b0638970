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


def family_for_batch(batch: int) -> str:
    """The small-K kernel family for a run configured with `batch` samples per engine
    (include/mmsbm.h mmsbm_set_family): SK_Y from 2 (the throughput winner), SK_U for one sample
    (the latency winner).  Fixed per run, so a ragged last batch, a rank with a smaller share or a
    shrinking pool gives its samples the same bits as the full batches."""
    return "sky" if int(batch) >= 2 else "sku"


def next_stop(it: int, iterations: int, fcheck: int, bcheck: int):
    """(iterations to run from `it` to the next stop, whether that stop is a check): the reference
    checks after make_iteration #c when c % fcheck == 0 and c > bcheck (:1268), and a sample ends
    after `iterations` iterations (:1264)."""
    c = max(it, bcheck + 1)
    c = -(-c // fcheck) * fcheck
    if c < iterations:
        return c + 1 - it, True
    return iterations - it, False


@dataclass
class PoolStats:
    """What a pool run cost: slot_iterations = sum over iterate calls of (iterations x live
    slots); sample_iterations = the iterations the samples needed (sum of SampleResult.iterations);
    calls = engine.iterate calls; refills = slots handed to a pending sample; shrinks = active-prefix
    reductions."""
    slot_iterations: int = 0
    sample_iterations: int = 0
    calls: int = 0
    refills: int = 0
    shrinks: int = 0


def run_pool(engine, states, iterations=10000, fcheck=25, bcheck=100, keep_params=False,
             on_done=None, stats: PoolStats = None):
    """Drive samples through a B-slot engine with the reference's per-sample loop (:1259-1279),
    retiring each sample at convergence (or after `iterations`) and handing its slot to the next
    pending one at once, as the reference's process starts its next sample (:1253-1279) and
    run.sh keeps every core busy (src/run.sh:12,16,45).

    `states` yields (sample id, theta [P][K], pr [K][K][K][R]) in sample order; it is consumed
    lazily, one sample per free slot, so initial states are drawn in sample order (:1260) whenever
    they are drawn.  Every slot keeps its own iteration count and check schedule; one engine.iterate
    call advances all live slots to the nearest stop of any of them.  When nothing is pending a
    finished slot takes the last live slot's parameters (a device copy) and the active prefix
    shrinks (engine.set_active), so no GPU time goes to finished samples.  A sample's bits do not
    depend on its slot or its batch-mates (one kernel family per run), so every result equals the
    sequential run's.  `engine` provides B, upload_slot, download_slot, move_slot, set_active,
    iterate, loglik.  on_done(result) is called as each sample finishes; returns the results in
    finishing order."""
    B = engine.B
    src = iter(states)
    slots = [None] * B       # per slot: [sample id, iterations run, previous check likelihood]
    pending_done = False

    def fill(b):
        nonlocal pending_done
        if pending_done:
            return False
        try:
            sid, th, pr = next(src)
        except StopIteration:
            pending_done = True
            return False
        engine.upload_slot(b, th, pr)
        slots[b] = [sid, 0, None]
        return True

    n_act = 0
    while n_act < B and fill(n_act):
        n_act += 1
    if n_act == 0:
        return []
    engine.set_active(n_act)
    like = engine.loglik(TRAIN)
    for b in range(n_act):
        slots[b][2] = float(like[b])
    out = []
    stats = stats if stats is not None else PoolStats()
    while n_act:
        stops = [next_stop(slots[b][1], iterations, fcheck, bcheck) for b in range(n_act)]
        n = min(st[0] for st in stops)
        if n > 0:
            engine.iterate(n)
            stats.calls += 1
            stats.slot_iterations += n * n_act
        for b in range(n_act):
            slots[b][1] += n
        like = held = None
        finished = []                  # (slot, converged, likelihood)
        for b in range(n_act):
            steps, check = stops[b]
            if steps != n:
                continue
            if check:
                if like is None:
                    like = engine.loglik(TRAIN)
                if math.fabs((like[b] - slots[b][2]) / slots[b][2]) < 0.01:
                    finished.append((b, True, float(like[b])))
                    continue
                slots[b][2] = float(like[b])
            if slots[b][1] >= iterations:
                if like is None:
                    like = engine.loglik(TRAIN)
                finished.append((b, False, float(like[b])))
        if not finished:
            continue
        held = engine.loglik(TEST)
        for b, conv, L in finished:
            th = pr = None
            if keep_params:
                th, pr = engine.download_slot(b)
            r = SampleResult(slots[b][0], slots[b][1], conv, L, float(held[b]), th, pr)
            stats.sample_iterations += r.iterations
            out.append(r)
            if on_done is not None:
                on_done(r)
            slots[b] = None
        refilled = []
        for b, _, _ in finished:       # slot order = the order pending samples are drawn in
            if fill(b):
                refilled.append(b)
                stats.refills += 1
        live = [b for b in range(n_act) if slots[b] is not None]
        if len(live) < n_act:          # nothing pending: compact the live slots to the front
            for e in range(len(live)):
                if slots[e] is None:
                    h = max(b for b in range(e + 1, n_act) if slots[b] is not None)
                    engine.move_slot(e, h)
                    slots[e], slots[h] = slots[h], None
                    refilled = [e if x == h else x for x in refilled]
            n_act = len(live)
            stats.shrinks += 1
            if n_act:
                engine.set_active(n_act)
        if refilled:
            like = engine.loglik(TRAIN)
            for b in refilled:
                slots[b][2] = float(like[b])
    return out


def run_samples(engine, sample_ids, thetas, prs, iterations=10000, fcheck=25, bcheck=100,
                keep_params=False):
    """The batched engine over exactly these samples (one slot each) with the reference's
    per-sample convergence rule; results in sample order.  See run_pool."""
    res = run_pool(engine, zip(sample_ids, thetas, prs), iterations, fcheck, bcheck, keep_params)
    order = {s: i for i, s in enumerate(sample_ids)}
    return sorted(res, key=lambda r: order[r.sample])


def stream_states(model, K: int, samples, mine=None):
    """(sample, theta, pr) for the samples in `mine` (default: all), drawing every sample's initial
    state from the one stdlib stream in `samples` order (:1260), lazily."""
    for s in samples:
        model.initialize_parameters(K)
        if mine is None or s in mine:
            yield s, np.array(model._theta, dtype=np.float64), np.array(model._pr, dtype=np.float64)


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
                 engine_factory=None, group=None, device=None, batch=None):
    """Shard `n_samples` restarts over the process group (or run all locally), drive them in one
    pool per rank (run_pool: `batch` slots, default the rank's whole share) and return every
    sample's result on every rank (sorted by sample id).  The kernel family follows `batch`, or
    n_samples when no batch is given, so the results do not depend on the world size."""
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
            family = family_for_batch(batch if batch else n_samples)

            def engine_factory(B):
                eng = EMEngine(K, model.P, B=B, R=model.R, eps=model.eps, device=device, family=family)
                eng.set_links(TRAIN, *links_to_arrays(model.links, model.R))
                eng.set_links(TEST, *links_to_arrays(model.test_links, model.R))
                return eng
        slots = min(batch or len(ids), len(ids))
        local = run_pool(engine_factory(slots), zip(ids, thetas, prs), iterations, fcheck, bcheck)
        local.sort(key=lambda r: r.sample)
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
