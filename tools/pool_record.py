"""Restart pool vs round 4's block driver (measurement aid): fold0 stand-in,
K=10, 64 samples, the reference's schedule (-i 10000 -f 25 -b 100), --batch 8 on one GPU.

  block: round 4's cli.run_batch - blocks of 8 samples in sample order, each block iterated until
         its slowest sample converges (finished slots keep iterating);
  pool:  restarts.run_pool - a converged sample's slot goes to the next pending sample at once,
         the active prefix shrinks when nothing is pending.

Both drivers give every sample the same iterations and the same likelihood bits (one kernel
family, SK_Y); the record holds the slot-iterations each paid and the wall time.

    python tools/pool_record.py [--samples 64] [--batch 8] [--K 10]
"""
import argparse
import contextlib
import io
import json
import math
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def block_driver(engine, states, iterations, fcheck, bcheck):
    """Round 4's restarts.run_samples on one block (every slot iterates until all converge);
    -> ({sample: (iterations, converged, L)}, slot-iterations)."""
    ids = [s for s, _, _ in states]
    B = len(ids)
    engine.upload(np.stack([t for _, t, _ in states]), np.stack([p for _, _, p in states]))
    like0 = np.array(engine.loglik(0), dtype=np.float64)
    done = [None] * B
    it = 0
    cost = 0
    while it < iterations and any(d is None for d in done):
        nxt = it
        while nxt < iterations and not (nxt % fcheck == 0 and nxt > bcheck):
            nxt += 1
        n = min(nxt, iterations - 1) - it + 1
        engine.iterate(n)
        cost += n * B
        it += n
        if it - 1 == nxt and nxt < iterations:
            like = np.array(engine.loglik(0), dtype=np.float64)
            for s in range(B):
                if done[s] is None and math.fabs((like[s] - like0[s]) / like0[s]) < 0.01:
                    done[s] = (it, True, float(like[s]))
                like0[s] = like[s]
    like = np.array(engine.loglik(0), dtype=np.float64)
    for s in range(B):
        if done[s] is None:
            done[s] = (it, False, float(like[s]))
    return dict(zip(ids, done)), cost


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--iterations", type=int, default=10000)
    ap.add_argument("--fcheck", type=int, default=25)
    ap.add_argument("--bcheck", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import torch
    import bench
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.restarts import PoolStats, family_for_batch, run_pool, stream_states
    tr, te = bench.make_fold(1500, 90000, 0)
    with contextlib.redirect_stdout(io.StringIO()):
        m = Model()
        m.get_traintest(tr, te)
    fam = family_for_batch(a.batch)

    def engine(B):
        e = EMEngine(a.K, m.P, B=B, family=fam)
        e.set_links(0, *m._link_arrays(0))
        e.set_links(1, *m._link_arrays(1))
        return e
    random.seed(a.seed)
    states = list(stream_states(m, a.K, range(a.samples)))
    # warm both paths (code objects, plans) outside the timed runs
    e8 = engine(a.batch)
    e8.upload(np.stack([t for _, t, _ in states[:a.batch]]), np.stack([p for _, _, p in states[:a.batch]]))
    e8.iterate(3)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    blk, blk_cost = {}, 0
    for lo in range(0, a.samples, a.batch):
        part = states[lo:lo + a.batch]
        r, c = block_driver(engine(len(part)) if len(part) != a.batch else e8, part, a.iterations,
                            a.fcheck, a.bcheck)
        blk.update(r)
        blk_cost += c
    torch.cuda.synchronize()
    t_block = time.perf_counter() - t0

    st = PoolStats()
    t0 = time.perf_counter()
    res = run_pool(e8, iter(states), a.iterations, a.fcheck, a.bcheck, stats=st)
    torch.cuda.synchronize()
    t_pool = time.perf_counter() - t0
    pool = {r.sample: (r.iterations, r.converged, r.loglik) for r in res}
    same = all(pool[s] == blk[s] for s in blk)
    its = [pool[s][0] for s in sorted(pool)]
    print(json.dumps({
        "workload": "fold0 stand-in (P=1500, 72k train observations), K=%d, %d samples, --batch %d, "
                    "-i %d -f %d -b %d, family %s" % (a.K, a.samples, a.batch, a.iterations, a.fcheck,
                                                       a.bcheck, fam),
        "sample_iterations": int(sum(its)),
        "iterations_per_sample": {"min": min(its), "median": float(np.median(its)), "max": max(its)},
        "converged": int(sum(1 for s in pool if pool[s][1])),
        "block_driver": {"slot_iterations": blk_cost, "seconds": t_block},
        "pool": {"slot_iterations": st.slot_iterations, "seconds": t_pool, "iterate_calls": st.calls,
                 "refills": st.refills, "shrinks": st.shrinks},
        "slot_iterations_saved": blk_cost - st.slot_iterations,
        "saved_frac": 1.0 - st.slot_iterations / blk_cost,
        "speedup": t_block / t_pool,
        "results_bitwise_equal": same,
        "build_id": __import__("trigenicinteractionpredictor_amd._lib", fromlist=["build_id"]).build_id(),
    }, indent=1))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
