"""Fixed cost of one mmsbm_iterate call vs its per-iteration cost (measurement aid): times
iterate(n) for several n on the fold0 stand-in at K=10 after a warmup and fits t(n) = a + b n.

    python tools/overhead_probe.py [--K 10] [--reps 20] [--graph G]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.restarts import init_samples
    tr, te = bench.make_fold(1500, 90000, 0)
    with contextlib.redirect_stdout(io.StringIO()):
        m = Model()
        m.get_traintest(tr, te)
    th, pr = init_samples(m, args.K, [0], 1)
    eng = EMEngine(args.K, m.P, B=1)
    eng.set_links(0, *m._link_arrays(0))
    eng.set_links(1, *m._link_arrays(1))
    eng.upload(np.stack(th), np.stack(pr))
    eng.iterate(50)
    torch.cuda.synchronize()
    ns = [1, 2, 5, 10, 20, 50, 100, 200]
    res = {}
    for n in ns:
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.iterate(n)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[n] = float(np.median(ts)) * 1e6
    a, b = np.polyfit(np.array(ns, float), np.array([res[n] for n in ns]), 1)[::-1]
    # the host side alone: launches queued without waiting (the GPU drains them afterwards)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(200)
    t_host = (time.perf_counter() - t0) * 1e6
    torch.cuda.synchronize()
    print(json.dumps({"median_us": res, "fit_fixed_us": a, "fit_per_iter_us": b,
                      "host_submit_200_us": t_host, "plan": eng.plan_info(0)["small_k"]}))


if __name__ == "__main__":
    main()
