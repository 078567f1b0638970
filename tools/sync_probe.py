"""Where the fixed cost of one timed call goes (measurement aid): the driver's
20-step line pays ~20 us of start/finish cost on top of 20 iterations.  Times, on the fold0
stand-in at K=10 (medians over --reps):

  sync_idle      torch.cuda.synchronize() on an idle device
  empty_k        one empty torch kernel + synchronize
  iterate(n)     EMEngine.iterate(n) + synchronize, n = 1, 2, 20, 200
  fit            t(n) = fixed + n * per_iter over n = 1..200

    python tools/sync_probe.py [--spin] [--reps 50]

--spin calls hipSetDeviceFlags(hipDeviceScheduleSpin) before torch touches the device (host waits
spin instead of sleeping on an interrupt); ROC_ACTIVE_WAIT_TIMEOUT in the environment sets how
long the HIP runtime spins before it sleeps.
"""
import argparse
import contextlib
import ctypes
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(f, reps):
    import torch
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--K", type=int, default=10)
    a = ap.parse_args()
    flags_rc = None
    if a.spin:
        hip = ctypes.CDLL("libamdhip64.so")
        flags_rc = int(hip.hipSetDeviceFlags(ctypes.c_uint(1)))  # hipDeviceScheduleSpin
    import torch
    import bench
    from trigenicinteractionpredictor_amd import EMEngine, Model
    from trigenicinteractionpredictor_amd.restarts import init_samples
    tr, te = bench.make_fold(1500, 90000, 0)
    with contextlib.redirect_stdout(io.StringIO()):
        m = Model()
        m.get_traintest(tr, te)
    th, pr = init_samples(m, a.K, [0], 1)
    eng = EMEngine(a.K, m.P, B=1)
    eng.set_links(0, *m._link_arrays(0))
    eng.set_links(1, *m._link_arrays(1))
    eng.upload(np.stack(th), np.stack(pr))
    eng.iterate(50)
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    res = {"sync_idle": med(lambda: None, a.reps), "empty_k": med(lambda: x.add_(1.0), a.reps)}
    ns = [1, 2, 20, 200]
    it = {n: med(lambda: eng.iterate(n), a.reps if n < 200 else 10) for n in ns}
    b, c = np.polyfit(np.array(ns, float), np.array([it[n] for n in ns]), 1)
    # the driver's short line: idle host gap, W warmup iterations, 20 timed (one shot each, median
    # over shots): how much of its excess is the GPU waking from idle
    short = {}
    for gap_ms in (0, 2, 20, 200):
        for w in (5, 50):
            ts = []
            for _ in range(7):
                torch.cuda.synchronize()
                time.sleep(gap_ms / 1000)
                eng.iterate(w)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.iterate(20)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            short["gap%dms_w%d" % (gap_ms, w)] = 20 / float(np.median(ts))
    print(json.dumps({"short_20_rate": short, "spin": a.spin, "hipSetDeviceFlags_rc": flags_rc,
                      "ROC_ACTIVE_WAIT_TIMEOUT": os.environ.get("ROC_ACTIVE_WAIT_TIMEOUT"),
                      "us": res, "iterate_us": it, "fit_fixed_us": c, "fit_per_iter_us": b,
                      "rate_20": 20 / it[20] * 1e6}))


if __name__ == "__main__":
    main()
