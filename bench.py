#!/usr/bin/env python3
"""Benchmark: EM-iterations/sec on the fold0 stand-in, K=10 (BASELINE.json metric, configs[1]).

A "step" is one EM iteration (`Model.make_iteration`, src/TrigenicInteractionPredictor.py
:984-1043) of every sample resident on a GPU over the fold0-shaped synthetic train set
(P=1,500 genes, 72,000 train links, 18,000 test links).  Samples
(independent EM restarts, :1253) shard across ranks with no data-path collective (weak
scaling); the final log-likelihoods are gathered over RCCL at the end (:1262-1279 analogue).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--K 10] [--samples 1]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` is measured live with HIP events on the launch stream:
the dominant kernel (the E-step) is launched back to back right after the timed region and
its average duration divides the algorithmic FLOPs of one launch; `kernel_us` also gives each
kernel's in-loop time from event pairs around the warmup iterations' launches (those include the
dependent-launch boundary; the timed steps run without events).  `cpu_baseline` times the
pure-Python CPU restatement of the reference path (oracle/, test infrastructure) on a bounded
sample of the same workload, on this host, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import random
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector and matrix: 256 CU x 128 FLOP/clk x 2.4 GHz (spec)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--samples", type=int, default=1, help="samples (restarts) per GPU")
    ap.add_argument("--P", type=int, default=1500)
    ap.add_argument("--E", type=int, default=90000, help="unique triples, train + test")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--hub", default="",
                    help="FRAC,SHARE: hub-heavy synthetic fold (SHARE of the triples take one gene "
                         "from the first FRAC of the genes; data.FoldSpec.hub_*), e.g. 0.02,0.3")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl",
                    help="collective backend: nccl (= RCCL over xGMI); gloo only to rehearse "
                         "several ranks sharing one GPU")
    ap.add_argument("--no-events", action="store_true", help="do not time kernels (overhead probe)")
    ap.add_argument("--roofline-launches", type=int, default=1000,
                    help="back-to-back E-step launches timed for the roofline")
    ap.add_argument("--shard", choices=("samples", "links"), default="samples",
                    help="samples: independent restarts per rank (weak scaling, the default); "
                         "links: ONE batch of samples whose train links are split over the ranks, "
                         "one all-reduce of the accumulators per iteration (strong scaling, "
                         "SURVEY.md 8e secondary)")
    ap.add_argument("--event-stride", type=int, default=1,
                    help="time the kernels of every n-th warmup iteration with HIP events")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and run the end-of-run gather without any GPU work "
                         "(CPU test of the N-rank launch path, with --backend gloo)")
    ap.add_argument("--process-group", action="store_true",
                    help="create the process group at --gpus 1 too (world size 1): the nccl init "
                         "with device_id, the RCCL all-gather of the result rows, the replay check "
                         "and, with --shard links, the per-iteration RCCL all-reduce all run on the "
                         "one GPU (VERDICT r3 item 4)")
    ap.add_argument("--test-frac", type=float, default=0.2,
                    help="share of the E unique triples that go to the test file (config 5 runs "
                         "with 0: all E links train)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="processes for the aggregate CPU baseline (default: the host cores this "
                         "process may use, at most 16)")
    return ap.parse_args()


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N copies of this script, one rank per GPU (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT as torch.distributed.run sets them), BEFORE this
    process touches any GPU, and return the first failure's exit code (a failed rank has the
    others terminated: they would wait in a barrier).  Rank 0 prints the JSON line.
    (The reference scales the same way, one OS process per batch of samples: src/run.sh:36-45.)"""
    from trigenicinteractionpredictor_amd.launch import spawn_ranks as spawn
    return spawn([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], n)


KERNEL_NAMES = {"pass_a": "pass_kernel<%d, PASS_A> (stream 0: V, Z, Z', d, c, the j / k Y entries, M0 "
                          "partial rows; FP64 MFMA)",
                "gene": "gm_kernel<%d> (X rows and S partials from the M0 partial rows, FP64 MFMA)",
                "fused": "fused E-step: sk_pass_kernel<%d, SK_U> (all three streams: V, Z, d, c, M, X; "
                         "stream 0 also the S partials); FP64 MFMA",
                "fused_sky": "fused E-step: sky_pass_kernel<%d> (SK_Y, stream 0: V, Z, Z', d, c, Y entries, "
                             "M, X, S partials); FP64 MFMA",
                "pass_b": "sk_pass_kernel<%d, SK_B> (streams 1/2: M1, M2, X)",
                "fin": "fin: sk_fin_kernel<%d> / upd_kernel (theta and p update)"}


def kernel_work(plan, K, P, R, B, E_obs):
    """Algorithmic (FLOPs, HBM bytes) of one launch of each kernel of the iteration, keyed by the
    engine's kernel labels (EMEngine.LABELS; DESIGN.md "Roofline accounting"): per observation
    2K^2 per K^2 contraction (Z, Z', M) and 2K (d); per pivot-gene table or contraction 2K^3;
    bytes = the records, Y entries, partial rows and parameters each launch must move once."""
    K2, K3 = K * K, K ** 3
    rows0, rows = plan["rows_stream0"], plan["rows"]
    prows = plan["partial_rows"]
    prow0 = plan["partial_rows_stream0"]
    genes_a = plan["v_genes"]
    params = 8.0 * (P * K + R * K3)
    if plan.get("small_k") == 3:
        # the stream-0 small-K E-step with Y entries (csrc/sk.h SK_Y): per observation Z, Z', M
        # (2K^2 each) and d; per stretch a V table and an X contraction, per stretch an S update;
        # bytes: records + their Y entry indices, 2K words of Y entries per observation, X partials,
        # S partials.  fin: per gene its X partial rows and Y entries, per cell the S partials.
        wga = plan["wg_stream0"]
        n_y = plan.get("y_entries", 2 * E_obs)
        u_fl = E_obs * (6.0 * K2 + 2.0 * K) + prow0 * 3 * 2.0 * K3
        u_by = 24.0 * rows0 + 8.0 * K * n_y + 8.0 * K * prow0 + 8.0 * K3 * wga + params
        f_fl = 1.0 * prow0 * K + 1.0 * n_y * K + R * K3 * wga + 3.0 * P * K + 3.0 * R * K3
        f_by = 8.0 * K * prow0 + 8.0 * K * n_y + 8.0 * K3 * wga + 2 * params + 4.0 * 8 * P
        return {"fused": (u_fl * B, u_by * B), "fin": (f_fl * B, f_by * B)}
    if plan.get("small_k") == 2:
        # the fused small-K E-step (csrc/sk.h SK_U): every stream's observations get Z, d, c and
        # M (each stream forms its own c); per stretch of any stream a V table and an X
        # contraction, per stream-0 stretch an S update; bytes: all records, X partials, S partials
        wga = plan["wg_stream0"]
        u_fl = 3.0 * E_obs * (4.0 * K2 + 2.0 * K) + prows * 2 * 2.0 * K3 + prow0 * 2.0 * K3
        u_by = 16.0 * rows + 8.0 * K * prows + 8.0 * K3 * wga + params
        f_fl = 1.0 * prows * K + R * K3 * wga + 3.0 * P * K + 3.0 * R * K3
        f_by = 8.0 * K * prows + 8.0 * K3 * wga + 2 * params + 4.0 * 6 * P
        return {"fused": (u_fl * B, u_by * B), "fin": (f_fl * B, f_by * B)}
    if plan.get("small_k"):
        # small-K kernels (csrc/sk.h): per stream-0 stretch a V table, an X contraction and an S
        # update (2K^3 each); per stream-1/2 stretch an X contraction; bytes: records, row12 and
        # the c scatter, X partials (K per partial row), S partials (K^3 per stream-0 workgroup)
        wga = plan["wg_stream0"]
        a_fl = E_obs * (4.0 * K2 + 2.0 * K) + prow0 * 3 * 2.0 * K3
        a_by = 24.0 * rows0 + 16.0 * E_obs + 8.0 * K * prow0 + 8.0 * K3 * wga + params
        b_fl = E_obs * 4.0 * K2 + (prows - prow0) * 2.0 * K3
        b_by = 24.0 * (rows - rows0) + 8.0 * K * (prows - prow0) + params
        f_fl = 1.0 * prows * K + R * K3 * wga + 3.0 * P * K + 3.0 * R * K3
        f_by = 8.0 * K * prows + 8.0 * K3 * wga + 2 * params + 4.0 * 6 * P
        return {"pass_a": (a_fl * B, a_by * B), "pass_b": (b_fl * B, b_by * B), "fin": (f_fl * B, f_by * B)}
    # large-K kernels (csrc/mmsbm.hip): pass A per observation Z, Z', M (2K^2 each) + d, per
    # workgroup gene a V table; it reads the records + their Y entry indices and writes 2K words
    # of Y entries per observation and the K^2 stream-0 partial rows.  The gene kernel: per
    # (gene, rating) with stream-0 rows an X0 contraction (2K^3; at most P R), per partial row an
    # S update (2K^3), per Y entry K adds; it reads the partial rows twice and the Y entries once,
    # writes x0, ysum and the S partials.  The update: theta from x0 + ysum, p from the S partials.
    n_sp = plan["wg_spartial"]
    n_y = plan.get("y_entries", 2 * E_obs)
    xg = min(P * R, prow0)
    a_fl = E_obs * (6.0 * K2 + 2.0 * K) + genes_a * 2.0 * K3
    a_by = 16.0 * rows0 + 8.0 * rows0 + 8.0 * K * n_y + 8.0 * K2 * prow0 + params
    g_fl = xg * 2.0 * K3 + prow0 * 2.0 * K3 + n_y * K
    g_by = 2 * 8.0 * K2 * prow0 + 8.0 * K * n_y + 8.0 * K3 * n_sp + 2 * 8.0 * P * K + params
    f_fl = 3.0 * P * K + n_sp * R * K3 + 3.0 * R * K3
    f_by = 3 * 8.0 * P * K + 8.0 * K3 * n_sp + 2 * params
    return {"pass_a": (a_fl * B, a_by * B), "gene": (g_fl * B, g_by * B), "fin": (f_fl * B, f_by * B)}


def s8d_work(K, P, R, B, E_obs):
    """SURVEY.md 8d's algorithmic work of one EM iteration of B samples: F = 8 K^3 per observed
    (link, r) (the reference's lattice) + the M-step 2 P K + 3 K^3 R, and the compulsory HBM
    bytes B_hbm = 16 E_obs + 2 * 8 P K + 3 * 8 K^3 R (records once, theta read + written,
    p / S)."""
    flops = (8.0 * K ** 3 * E_obs + 2.0 * P * K + 3.0 * K ** 3 * R) * B
    hbm = (16.0 * E_obs + 16.0 * P * K + 24.0 * K ** 3 * R) * B
    return flops, hbm


def pmc_traffic(build_id, K, E_obs, B):
    """L2->fabric bytes per launch from a PMC record under profiles/ taken with THIS build
    (tools/pmc_to_traffic.py stamps each record with the profiled library's build id, and states
    its basis: Infinity-Cache hits included, FETCH doubled for wide-stream kernels only); None when
    no record names this build.  Round-5 records (HBM-labelled, FETCH doubled everywhere) are
    not used."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            with open(f) as fh:
                rec = json.load(fh)
        except (OSError, ValueError):
            continue
        if (rec.get("build_id") == build_id and rec.get("K") == K and rec.get("E_obs") == E_obs
                and rec.get("B") == B and rec.get("l2_fabric_bytes_per_launch")):
            best = (os.path.relpath(f, REPO), rec)
    return best


def roofline_record(K, P, R, B, E_obs, plan, iter_s, b2b, build_id):
    """The bench line's `roofline` (DESIGN.md "Roofline accounting").  Headline: SURVEY 8d's
    binding roof for K >= 3, FP64: achieved = 8d FLOPs of one iteration / the measured iteration
    time (the timed region), against the FP64 MFMA peak.  Beside it: the FLOPs the engine really
    executes (its factorisation does far fewer), the 8d compulsory HBM bytes against the HBM
    peak, and the longest kernel of the iteration timed alone back to back with HIP events."""
    f8, b8 = s8d_work(K, P, R, B, E_obs)
    work = kernel_work(plan, K, P, R, B, E_obs)
    exe = sum(fl for fl, _ in work.values())
    tf = f8 / iter_s / 1e12
    dom = max(b2b, key=b2b.get)
    dom_s = b2b[dom] / 1e3
    dfl, dby = work[dom]
    pmc = pmc_traffic(build_id, K, E_obs, B)
    traffic = None
    if pmc is not None:
        traffic = sum(pmc[1]["l2_fabric_bytes_per_launch"].get(k, 0.0) for k in work)
    exe_tf = exe / iter_s / 1e12
    # the 8d credit counts the reference's 8 K^3 per observation; where that exceeds the FP64
    # peak (K >= 20 here: the factorisation does far less work) it says nothing about utilisation,
    # so the headline becomes the executed FLOPs and the credit stays beside it
    credited = tf <= FP64_PEAK_TFLOPS
    head = tf if credited else exe_tf
    return {"bound": "mfma", "achieved": head, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": head / FP64_PEAK_TFLOPS,
            "frac_credited": tf / FP64_PEAK_TFLOPS,
            "frac_executed": exe_tf / FP64_PEAK_TFLOPS,
            "frac_basis": ("SURVEY 8d credited FLOPs" if credited else
                           "executed FLOPs (the 8d credit exceeds the FP64 peak)"),
            "credited": {"achieved": tf, "frac": tf / FP64_PEAK_TFLOPS},
            "traffic": traffic,
            "traffic_unit": "L2->fabric bytes per iteration, all kernels (PMC FETCH_SIZE + WRITE_SIZE: "
                            "Infinity-Cache hits included, so an upper bound on HBM bytes; FETCH x 2 "
                            "only for wide-stream kernels)",
            "traffic_basis": None if pmc is None else pmc[1].get("basis"),
            "traffic_per_kernel": None if pmc is None else pmc[1]["l2_fabric_bytes_per_launch"],
            "tcc_hit_rate": None if pmc is None else pmc[1].get("tcc_hit_rate"),
            "traffic_source": None if pmc is None else pmc[0],
            "traffic_build_id": None if pmc is None else pmc[1]["build_id"],
            "per": "one EM iteration of all %d sample(s): %.4g FLOPs credited by SURVEY 8d "
                   "(8 K^3 per observation + the M-step) / %.3f us measured" % (B, f8, iter_s * 1e6),
            "credited_flops_per_iteration": f8,
            "executed": {"flops_per_iteration": exe, "achieved": exe / iter_s / 1e12,
                         "peak": FP64_PEAK_TFLOPS, "frac": exe / iter_s / 1e12 / FP64_PEAK_TFLOPS},
            "hbm": {"bytes_per_iteration": b8, "achieved": b8 / iter_s / 1e9, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": b8 / iter_s / 1e9 / HBM_PEAK_GBS,
                    "traffic_over_compulsory": None if traffic is None else traffic / b8},
            "dominant_kernel": {"kernel": KERNEL_NAMES["fused_sky" if dom == "fused" and plan.get("small_k") == 3
                                                    else dom] % K, "avg_launch_us": dom_s * 1e6,
                                "executed_flops_per_launch": dfl, "algorithmic_bytes_per_launch": dby,
                                "tflops": dfl / dom_s / 1e12, "mfma_frac": dfl / dom_s / 1e12 / FP64_PEAK_TFLOPS,
                                "gbs": dby / dom_s / 1e9, "hbm_frac": dby / dom_s / 1e9 / HBM_PEAK_GBS,
                                "traffic_per_launch": None if pmc is None else
                                pmc[1]["l2_fabric_bytes_per_launch"].get(dom)}}


def make_fold(P, E, rank, hub="", test_frac=0.2):
    from trigenicinteractionpredictor_amd.data import FoldSpec, write_fold
    d = tempfile.mkdtemp(prefix="mmsbm_bench_r%d_" % rank)
    tr, te = os.path.join(d, "train0.dat"), os.path.join(d, "test0.dat")
    hf, hs = (float(x) for x in hub.split(",")) if hub else (0.0, 0.0)
    write_fold(FoldSpec(P=P, E=E, seed=7, hub_frac=hf, hub_share=hs, test_frac=test_frac), tr, te)
    return tr, te


def _port_rate(train, test, K, seed, seconds, full):
    """One CPU process: seconds per EM iteration of the pure-Python restatement of :984-1043.
    full: time whole make_iteration calls (cheap K); else the per-link loop (:987-1012, all of
    the cost) on the first n links, n sized so the sample takes ~`seconds`, scaled to every
    link, plus the M-step (:1016-1043) timed whole.  -> (s_per_iter, links_timed, links)."""
    import contextlib
    import io
    from oracle.mmsbm_oracle import OracleModel
    with contextlib.redirect_stdout(io.StringIO()):
        m = OracleModel()
        m.get_traintest(train, test)
    random.seed(seed)
    m.initialize_parameters(K)
    items = list(m.links.items())
    E = len(items)
    if full:
        n_it = 0
        t0 = time.perf_counter()
        while n_it < 1 or time.perf_counter() - t0 < seconds:
            m.make_iteration()
            n_it += 1
        return (time.perf_counter() - t0) / n_it, E, E
    t0 = time.perf_counter()
    m.accumulate(items[:32])
    per_link = (time.perf_counter() - t0) / 32
    n = max(32, min(E, int(seconds / per_link)))
    t0 = time.perf_counter()
    m.accumulate(items[:n])
    t_loop = time.perf_counter() - t0
    full_deg = [0] * m.P
    for key in m.links:
        for x in key.split("_"):
            full_deg[int(x)] += 1
    nth = [[1.0] * K for _ in range(m.P)]
    npr = [[[[0.5] * m.R for _ in range(K)] for _ in range(K)] for _ in range(K)]
    t0 = time.perf_counter()
    m.finish(nth, npr, full_deg)
    t_fin = time.perf_counter() - t0
    return t_loop * E / n + t_fin, n, E


def _port_worker(a):
    return _port_rate(*a)


def cpu_baseline(train, test, K, seed, seconds, cores):
    """The reference path's CPU baseline: the oracle's pure-Python restatement,
    one process per core, each on its own sample (the reference's own scaling model, src/run.sh
    :12,16).  Single-core rate alone, then `cores` processes at once (aggregate); config 1's K=2
    rate from whole iterations.  Runs before this process touches the GPU."""
    import multiprocessing as mp
    one, n, E = _port_rate(train, test, K, seed, seconds, False)
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        many = pool.map(_port_worker, [(train, test, K, seed + c, seconds, False) for c in range(cores)])
    agg = sum(1.0 / r[0] for r in many)
    k2, _, _ = _port_rate(train, test, 2, seed, min(seconds, 5.0), True)
    rec = {"value": agg, "unit": "EM-iterations/s", "cores": cores, "kind": "port",
           "single_core_value": 1.0 / one,
           "config1_K2_single_core_value": 1.0 / k2,
           "sample": ("oracle/mmsbm_oracle.py (pure-Python restatement of :984-1043), %s %s. "
                      "K=%d: the per-link loop timed on %d of %d train links (%.0f s) and scaled "
                      "x%.2f to the whole set, M-step timed whole: %.1f s/iteration on 1 core; "
                      "%d processes at once, each its own sample: aggregate %.4f iterations/s. "
                      "K=2 (config 1): whole iterations, %.2f s each on 1 core"
                      % (platform.python_implementation(), platform.python_version(), K, n, E,
                         seconds, E / n, one, cores, agg, k2))}
    cal = os.path.join(REPO, "profiles", "cpu_calibration.json")
    if os.path.exists(cal):
        with open(cal) as f:
            rec["calibration"] = json.load(f)     # restatement vs the reference's own loop
    return rec


def launch_check(args, world, rank):
    """The N-rank path without GPU work: every rank takes its block of sample ids, and the
    end-of-run gather (RCCL all_gather under nccl) collects them on every rank."""
    import torch
    import torch.distributed as dist
    from trigenicinteractionpredictor_amd.restarts import shard_samples
    if world > 1:
        dist.init_process_group(args.backend)
    ids = shard_samples(args.samples * world, world, rank)
    mine = torch.tensor([[rank, s] for s in ids], dtype=torch.float64)
    if world > 1:
        rows = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        rows = torch.cat(rows)
    else:
        rows = mine
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world,
                          "world_size": dist.get_world_size() if world > 1 else 1,
                          "gathered_rows": int(rows.shape[0]),
                          "samples": sorted(int(x) for x in rows[:, 1].tolist())}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    if args.launch_check:
        launch_check(args, world, rank)
        return 0
    if args.backend == "nccl" and world > 1:
        import torch               # (a rank: it uses its GPU anyway)
        n_vis = torch.cuda.device_count()
        if world > n_vis:          # RCCL: one GPU per rank of a communicator
            print("bench.py: %d nccl ranks need %d GPUs, %d visible" % (world, world, n_vis),
                  file=sys.stderr)
            return 2
    train, test = make_fold(args.P, args.E, rank, args.hub, args.test_frac)
    cpu_rec = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = args.cpu_cores or min(len(os.sched_getaffinity(0)), 16)
        cpu_rec = cpu_baseline(train, test, args.K, args.seed, args.cpu_baseline_seconds, cores)

    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll = dev if args.backend == "nccl" else torch.device("cpu")  # where collectives run
    dist_on = world > 1 or args.process_group
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            import socket
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            if "MASTER_PORT" not in os.environ:
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from trigenicinteractionpredictor_amd import EMEngine, Model, _lib
    from trigenicinteractionpredictor_amd.layout import links_to_arrays, n_observations
    build_id = _lib.build_id()

    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        host = Model()
        host.get_traintest(train, test)
    K, B = args.K, args.samples
    links_mode = args.shard == "links"
    # restart sharding: global sample s = rank*B + b; one RNG stream seeded once, like :1149/:1260.
    # link sharding: every rank holds the same B samples (s = 0..B-1) and 1/world of the links.
    first = 0 if links_mode else rank * B
    from trigenicinteractionpredictor_amd.restarts import (family_for_batch, gather_rows, init_samples,
                                                           replay_check, result_rows, rows_digest)
    sample_ids = list(range(first, first + B))
    thetas, prs = init_samples(host, K, sample_ids, args.seed)
    # the small-K kernel family follows the configured samples per GPU (SK_U for one, SK_Y from
    # two; include/mmsbm.h mmsbm_set_family), and the replay below uses the same family
    family = family_for_batch(B)
    eng = EMEngine(K, host.P, B=B, device=dev, family=family)
    ids, counts = host._link_arrays(0)           # the native reader's arrays (links order)
    tids, tcounts = host._link_arrays(1)
    if links_mode:
        from trigenicinteractionpredictor_amd.linkshard import LinkShardedEM, shard_links
        runner = LinkShardedEM(eng, ids, counts, tids, tcounts)
        lo, hi = shard_links(ids.shape[0], world, rank)
        E_obs = n_observations(counts[lo:hi])      # this rank's observations
    else:
        eng.set_links(0, ids, counts)
        eng.set_links(1, tids, tcounts)
        runner = eng
        E_obs = n_observations(counts)
    runner.upload(np.stack(thetas), np.stack(prs))
    plan = eng.plan_info(0)

    # per-kernel in-loop times come from event pairs in the (untimed) warmup iterations: an
    # event record between two dependent launches costs the loop ~1-2 us, so the timed region
    # runs without them
    # (the first warmup iteration runs without them: it includes the code objects' lazy load)
    first_w = min(1, args.warmup)
    runner.iterate(first_w)
    eng.timing(0 if args.no_events else args.event_stride)
    runner.iterate(args.warmup - first_w)
    torch.cuda.synchronize(dev)
    labels = eng.kernels()
    in_loop = {k: eng.timing_result(k) for k in labels}
    eng.timing(False)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    runner.iterate(args.steps)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist_on:
        dist.barrier()
    # each kernel of the iteration alone, back to back on the launch stream (per-launch duration
    # for the roofline; the in-loop events above also time the dependent-launch boundary)
    b2b = {k: eng.time_kernel(k, args.roofline_launches) for k in labels}
    elapsed = t1 - t0
    L = runner.loglik(0)
    rows = result_rows(sample_ids, L)
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if not links_mode:   # RCCL all-gather of (sample, final L) over xGMI
            rows = gather_rows(rows, B * world, device=coll)
    n_gathered = int(rows.shape[0])
    scale_check = None
    if rank == 0 and dist_on and not links_mode:
        # every sample replayed as ONE batch on this GPU: within one kernel family a sample's bits
        # do not depend on its batch or rank, so the gathered values must equal the replay bit for bit
        def factory(nb):
            e = EMEngine(K, host.P, B=nb, device=dev, family=family)
            e.set_links(0, ids, counts)
            e.set_links(1, tids, tcounts)
            return e
        scale_check = replay_check(rows, host, K, args.seed, args.warmup + args.steps, factory)

    if rank == 0:
        iters_total = args.steps * B * (1 if links_mode else world)
        value = iters_total / elapsed
        iter_s = elapsed / args.steps
        roofline = roofline_record(K, host.P, 2, B, E_obs, plan, iter_s, b2b, build_id)
        wl = ("fold0 stand-in" if (args.P, args.E) == (1500, 90000) else
              "synthetic P=%d, E=%d" % (host.P, args.E))
        if args.hub:
            wl += " (hub-heavy degrees %s)" % args.hub
        line = {
            "metric": "EM-iterations/sec + final log-likelihood, fold0 K=%d" % K,
            "value": value,
            "unit": "EM-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if links_mode else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic fold0 stand-in (real fold0 is a Git-LFS pointer)",
            "config": {"workload": ("%s, K=%d, %d sample(s) link-sharded over %d GPU(s)"
                                    % (wl, K, B, world)) if links_mode else
                                   "%s, K=%d, %d sample(s)/GPU" % (wl, K, B), "K": K,
                       "P": host.P, "E_train": int(ids.shape[0]), "E_test": int(tids.shape[0]),
                       "E_obs": E_obs, "samples_per_gpu": B,
                       "parallelism": ("link-sharded x%d" if links_mode else "restart-sharded x%d") % world},
            "world_size": dist.get_world_size() if dist_on else 1,
            "process_group": dist.get_backend() if dist_on else None,
            "gathered_samples": n_gathered,
            "final_loglik": float(rows[0, 1]),
            "final_loglik_best": float(rows[:, 1].max()),
            "samples": {"digest": rows_digest(rows),
                        "rows": rows.tolist() if n_gathered <= 64 else None,
                        "replay_check": scale_check},
            "build_id": build_id,
            "roofline": roofline,
            # both bases of the roofline fraction, whichever `roofline.frac` reports
            "frac_credited": roofline["frac_credited"],
            "frac_executed": roofline["frac_executed"],
            "kernel_family": {0: "large-K", 1: "small-K two-pass", 2: "SK_U", 3: "SK_Y"}[plan["small_k"]],
            "iteration": {"us": iter_s * 1e6},
            # the kernels the iteration launches (EMEngine.kernels(): the fused small-K E-step
            # has no pass B, the large-K iteration runs pass A, the gene kernel and the update)
            "kernel_us": {k: {"back_to_back": b2b[k] * 1e3,
                              "in_loop": in_loop[k][0] * 1e3 / max(in_loop[k][1], 1)}
                          for k in labels},
            "plan": plan,
            "cpu_baseline": cpu_rec,
        }
        if cpu_rec is not None:
            line["vs_cpu_baseline"] = value / cpu_rec["value"]
        print(json.dumps(line), flush=True)
    rc = 0
    if scale_check is not None and not scale_check["bitwise_equal"]:
        print("bench.py: gathered per-sample results differ from the one-GPU replay", file=sys.stderr)
        rc = 3
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
