#!/usr/bin/env python3
"""Joint digenic + trigenic EM throughput (src/TrigenicInteractionPredictor_23.py :1572-1687 on
the GPU: trigenicinteractionpredictor_amd/joint.py JointEngine), one GPU.

    python tools/bench_joint.py [--P 1500] [--E3 90000] [--E2 30000] [--K 10] [--samples 1]
                                [--steps 200] [--warmup 20]

Prints one JSON line: joint EM-iterations/s (whole iterations: the fused pair half, then the
triplet iteration whose theta update adds the pair sums), the split between the
triplet and the pair half (HIP events around each half over the timed loop's last iterations),
and the pair kernels' algorithmic bytes per iteration.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import random
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1500)
    ap.add_argument("--E3", type=int, default=90000)
    ap.add_argument("--E2", type=int, default=30000)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--samples", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--split-iters", type=int, default=20)
    a = ap.parse_args()

    import torch
    from trigenicinteractionpredictor_amd import _lib
    from trigenicinteractionpredictor_amd.data import JointFoldSpec, write_joint_fold
    from trigenicinteractionpredictor_amd.joint import JointEngine, Model, _pair_arrays
    from trigenicinteractionpredictor_amd.layout import links_to_arrays

    d = tempfile.mkdtemp(prefix="mmsbm_joint_")
    tr, te = os.path.join(d, "train.dat"), os.path.join(d, "test.dat")
    write_joint_fold(JointFoldSpec(P=a.P, E3=a.E3, E2=a.E2, seed=7, pair_only=a.P // 30), tr, te)
    with contextlib.redirect_stdout(io.StringIO()):
        m = Model()
        m.get_train_test(tr, te)
    K, B = a.K, a.samples
    random.seed(1)
    inits = []
    for _ in range(B):
        m.initialize_parameters(K)
        inits.append((np.array(m._theta), np.array(m._pr), np.array(m._qr)))
    torch.cuda.set_device(0)
    eng = JointEngine(K, m.P, B=B)
    ids3, c3 = links_to_arrays(m.links, 2)
    ids2, c2 = _pair_arrays(m.dlinks, 2)
    eng.set_links(_lib.SET_TRAIN, ids3, c3, ids2, c2)
    eng.upload(*[np.stack([x[i] for x in inits]) for i in range(3)])
    eng.iterate(a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.iterate(a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L = eng.loglik(0)
    # split: events around one pair launch + one triplet iteration, through the building blocks
    # (the pair launch alone = mmsbm_pairs_accumulate, which also adds its S2 tail)
    lib, s = eng.lib, torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    th, pr, qr = eng.theta.data_ptr(), eng.pr.data_ptr(), eng.qr.data_ptr()
    nth, S2 = eng.nth.data_ptr(), eng.S2.data_ptr()
    acc = np.zeros(2)
    for _ in range(a.split_iters):
        ev[0].record(s)
        _lib.check(lib.mmsbm_pairs_accumulate(eng.pctx, th, qr, nth, S2, s.cuda_stream))
        ev[1].record(s)
        _lib.check(lib.mmsbm_joint_iterate(eng.tri.ctx, eng.pctx, th, pr, qr, nth, 1, s.cuda_stream))
        ev[2].record(s)
        torch.cuda.synchronize()
        acc += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])]
    acc = acc / a.split_iters * 1e3
    info = eng.plan_info(0)
    n_ent = info["pair_entries"]
    # pair half, algorithmic bytes per iteration: each entry's record (8 B) and its other gene's
    # theta row (8 K B); the genes' theta rows, ntheta written, qr read and written
    pair_bytes = B * (n_ent * (8 + 8 * K) + 2 * 8 * m.P * K + 2 * 8 * 2 * K * K)
    print(json.dumps({
        "metric": "joint EM-iterations/sec (digenic + trigenic, _23)", "value": a.steps * B / el,
        "unit": "EM-iterations/s", "ms_per_step": el / a.steps * 1e3, "steps": a.steps, "dtype": "f64",
        "config": {"P": m.P, "E_triplets": len(m.links), "E_pairs": len(m.dlinks), "K": K,
                   "samples": B, "data": "synthetic joint fold (data.JointFoldSpec)"},
        "split_us": {"pair_launch_with_s2_tail": acc[0], "joint_iteration": acc[1]},
        "pair_plan": {k: v for k, v in info.items() if k.startswith("pair_")},
        "pair_bytes_per_iteration": pair_bytes,

        "final_loglik": float(L[0]),
    }), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
