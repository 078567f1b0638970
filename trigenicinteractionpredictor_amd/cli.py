"""Command-line driver: the reference's `__main__` (src/TrigenicInteractionPredictor.py:1148-1279)
on the GPU `Model`.

    python -m trigenicinteractionpredictor_amd.cli -k 10 -t train0.dat -e test0.dat -o out/ \
        [-i 10000] [-n 100] [-s 0] [-f 25] [-b 100] [--seed S]

Same flags, defaults, validation, exit codes and per-sample semantics as the reference:
  * `random.seed(os.getpid())` once (:1149) unless --seed is given (an addition, for
    reproducible runs); samples consume the stdlib stream one after another;
  * a sample whose `Sample_<n>_K<k>.csv` exists is skipped (:1256-1257, the resume rule);
  * the likelihood is checked after iteration `it` when `it % f == 0 and it > b` (:1268) and
    the sample stops when |(L - L0) / L0| < 0.01 (:1272), writing its file only then (:1275);
  * `-f 0` sets f = iterations + 1 with the iterations value parsed so far (:1192-1193), so
    the check never fires and no file is written — kept, not "fixed";
  * the K = 1 warning never prints (`int(arg == 1)`, :1224) — kept.
The iterations between two checks run as one `Model.make_iterations(n)` call (no host round
trip per iteration); the per-iteration lines are printed after the batch, with the same text.

`--gpus N` is the reference's process-level sample parallelism (src/run.sh:36-45, one OS process
per batch of samples) as one process per GPU: without a launcher the command starts N copies of
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them) before it
touches a GPU, and every rank takes a contiguous block of the pending samples (`run_ranked`).
Each rank replays the one RNG stream through the draws of the samples before its block, so a
sample starts from the state the one-process run gives it, runs with the reference's check
schedule and convergence rule (:1262-1279) on its own GPU, and writes its own
`Sample_<n>_K<k>.csv`.  One all-gather at the end (RCCL over xGMI under nccl) brings every
sample's result to rank 0, which prints the summary.  A sample's bits depend neither on its batch
nor on its rank, so the files equal a one-process run's byte for byte.  (At K <= 12 the kernel
family follows `--batch`: B = 1 sums in SK_U's order, B >= 2 in SK_Y's, so files written with
different `--batch` values agree to ~1e-12 relative, not byte for byte; include/mmsbm.h
mmsbm_set_family.)
"""
from __future__ import annotations

import getopt
import math
import os
import random
import sys

USAGE = """
Usage:
python -m trigenicinteractionpredictor_amd.cli [-h|--help] [-i|--num_iterations=] <iterations>
    [-n|--num_samples=] <samples> [-s|--sample_ini=] <first sample id>
    [-f|--fcheck=] <likelihood check frequency, 0: never> [-b|--bcheck=] <first check after>
    [-o|--out=] <output path prefix> [-t|--train=] <train file> [-e|--test=] <test file>
    [-k|--k=] <number of groups> [--seed=] <RNG seed, default: the process id>
    [--batch=] <samples advanced together on the GPU, default 1; at K <= 12 a batch of 2 or more
               runs the batched kernel family, whose files agree with --batch 1 to ~1e-12, not
               byte for byte>
    [--gpus=] <processes, one per GPU, over which the samples are sharded, default 1>
    [--backend=] <collective backend of --gpus: nccl (RCCL, default) or gloo>

Defaults: iterations {it}, samples {s}, check frequency {f}, train file {t}, K {k}.
"""


MAX_K = 32   # MMSBM_MAX_K (include/mmsbm.h): largest K the kernels are compiled for


class ArgError(Exception):
    pass


def parse(argv, defaults):
    cfg = dict(defaults)
    try:
        opts, _ = getopt.getopt(argv, "hi:n:s:f:b:o:t:e:k:",
                                ["help", "num_iterations=", "num_samples=", "sample_ini=", "fcheck=",
                                 "bcheck=", "out=", "train=", "test=", "k=", "seed=", "batch=", "gpus=",
                                 "backend="])
    except getopt.GetoptError:
        print("Argument error. Aborting")
        raise ArgError()
    for opt, arg in opts:          # in order: -f 0 uses the iterations parsed before it
        if opt in ("-h", "--help"):
            print(USAGE.format(it=cfg["iterations"], s=cfg["samples"], f=cfg["fcheck"],
                               t=cfg["train"], k=cfg["k"]))
            cfg["help"] = True
            return cfg
        try:
            if opt in ("-i", "--num_iterations"):
                if int(arg) < 1:
                    print("\n\nERROR: Number of num_iterations should be a integer positive number!")
                    raise ArgError()
                cfg["iterations"] = int(arg)
            elif opt in ("-n", "--num_samples"):
                if int(arg) < 1:
                    print("\n\nERROR: Number of samples should be a integer positive number")
                    raise ArgError()
                cfg["samples"] = int(arg)
            elif opt in ("-s", "--sample_ini"):
                if int(arg) < 0:
                    print("\n\nERROR: Number of samples should be a integer positive number!")
                    raise ArgError()
                cfg["sample_ini"] = int(arg)
            elif opt in ("-f", "--fcheck"):
                if int(arg) < 0:
                    print("\n\nERROR: frequency of checking should be a integer positive number or 0!")
                    raise ArgError()
                cfg["fcheck"] = cfg["iterations"] + 1 if int(arg) == 0 else int(arg)
            elif opt in ("-b", "--bcheck"):
                if int(arg) < 0:
                    print("\n\nERROR: Threshold to start checking likelihood should be a integer "
                          "positive number or 0!")
                    raise ArgError()
                cfg["bcheck"] = int(arg)
            elif opt in ("-o", "--out"):
                if not os.path.exists(str(arg)):
                    print("\n\nERROR: The selected path does not exist.")
                    raise ArgError()
                cfg["out"] = arg
            elif opt in ("-t", "--train"):
                if not os.path.isfile(arg):
                    print("\n\nERROR: The selected file does not exist.")
                    raise ArgError()
                cfg["train"] = arg
            elif opt in ("-e", "--test"):
                if not os.path.isfile(arg):
                    print("\n\nERROR: The selected file does not exist.")
                    raise ArgError()
                cfg["test"] = arg
            elif opt in ("-k", "--k"):
                if int(arg) < 1:
                    print("\n\nERROR: Number of groups should be a positive integer number different from 0")
                    raise ArgError()
                if int(arg) > MAX_K:     # the engine's compiled kernel set (include/mmsbm.h)
                    print("\n\nERROR: Number of groups K=%d is above the engine's maximum %d"
                          % (int(arg), MAX_K))
                    raise ArgError()
                cfg["k"] = int(arg)
            elif opt == "--seed":
                cfg["seed"] = int(arg)
            elif opt == "--batch":
                if int(arg) < 1:
                    print("\n\nERROR: batch size should be a positive integer number")
                    raise ArgError()
                cfg["batch"] = int(arg)
            elif opt == "--gpus":
                if int(arg) < 1:
                    print("\n\nERROR: number of GPUs should be a positive integer number")
                    raise ArgError()
                cfg["gpus"] = int(arg)
            elif opt == "--backend":
                if arg not in ("nccl", "gloo"):
                    print("\n\nERROR: backend should be nccl or gloo")
                    raise ArgError()
                cfg["backend"] = arg
        except ValueError:
            raise ArgError()
    return cfg


def check_points(iterations, fcheck, bcheck):
    """Iteration indices after which the reference checks the likelihood (:1268)."""
    return [it for it in range(iterations) if it % fcheck == 0 and it > bcheck]


def run_sample(model, cfg, sample, outfile, out=print):
    """One sample of the reference loop (:1259-1279); returns (iterations run, converged)."""
    out("Sample " + str(sample) + ":")
    model.initialize_parameters(cfg["k"])
    out("Parameters have been initialized")
    like0 = model.compute_likelihood()
    out("· Initial Likelihood is " + str(like0))
    iterations, f, b = cfg["iterations"], cfg["fcheck"], cfg["bcheck"]
    checks = check_points(iterations, f, b)
    it = 0
    for c in checks + [iterations - 1]:
        if c < it:
            continue
        model.make_iterations(c - it + 1)
        for i in range(it, c + 1):
            out("· Iteration " + str(i))
        it = c + 1
        if c in checks:
            like = model.compute_likelihood()
            out("· Likelihood " + str(c + 1) + " is " + str(like))
            if math.fabs((like - like0) / like0) < 0.01:
                out("\n\t**************************\n\t* Likelihood has converged *\n\t**************************")
                model.to_file(outfile)
                return it, True
            like0 = like
        if it >= iterations:
            break
    return it, False


DEFAULTS = {"iterations": 10000, "samples": 100, "sample_ini": 0, "fcheck": 25, "bcheck": 100,
            "train": "train0.dat", "test": "test0.dat", "out": "", "k": 1, "seed": None, "batch": 1,
            "gpus": 1, "backend": "nccl"}


def _write_result(model, cfg, r):
    """A converged sample's file (:1275) from its theta / p snapshot and converged likelihood."""
    model.theta = r.theta.tolist()
    model.pr = r.pr.tolist()
    model.likelihood = r.loglik
    model.to_file(cfg["out"] + "Sample_" + str(r.sample) + "_K" + str(cfg["k"]) + ".csv")


def _summary(r):
    return ("Sample " + str(r.sample) + ": " + str(r.iterations) + " iterations, likelihood "
            + str(r.loglik) + (" (converged)" if r.converged else ""))


def _default_engine_factory(model, K, family):
    from .engine import EMEngine

    def factory(n):
        eng = EMEngine(K, model.P, B=n, R=model.R, eps=model.eps, family=family)
        eng.set_links(0, *model._link_arrays(0))
        eng.set_links(1, *model._link_arrays(1))
        return eng
    return factory


def _pool(model, cfg, samples, mine, engine_factory, on_done, stats=None):
    """One engine of min(--batch, len(mine)) slots over the samples in `mine` (restarts.run_pool):
    a converged sample's file is written at once (:1275) and its slot goes to the next pending
    sample.  The kernel family follows the configured --batch (restarts.family_for_batch), so
    every sample's bits are those of the one-process run whatever its share."""
    from .restarts import family_for_batch, run_pool, stream_states
    K = cfg["k"]
    n = min(cfg["batch"], len(mine))
    if n == 0:
        return []
    if engine_factory is None:
        engine_factory = _default_engine_factory(model, K, family_for_batch(cfg["batch"]))
    return run_pool(engine_factory(n), stream_states(model, K, samples, mine), cfg["iterations"],
                    cfg["fcheck"], cfg["bcheck"], keep_params=True, on_done=on_done, stats=stats)


def run_batch(model, cfg, samples, out=print, engine_factory=None, stats=None):
    """`--batch B`: the pending samples share one B-slot engine (restarts.run_pool): the
    reference's per-sample check schedule and convergence rule (:1262-1279) for each sample; a
    converged sample is written through `Model.to_file` (:1275) as soon as it converges, with its
    converged train likelihood as `likelihood` (:1269), and its slot takes the next pending sample
    at once.  Initial states come from the one RNG stream in sample order (:1260).  The summary
    lines print in sample order at the end.  Returns [(sample, iterations, converged)]."""
    def done(r):
        if r.converged:
            _write_result(model, cfg, r)
    res = sorted(_pool(model, cfg, samples, set(samples), engine_factory, done, stats),
                 key=lambda r: r.sample)
    for r in res:
        out(_summary(r))
    return [(r.sample, r.iterations, r.converged) for r in res]


def run_ranked(model, cfg, samples, out=print, engine_factory=None, group=None, device=None, stats=None):
    """`--gpus N`, one rank: this rank's contiguous block of the pending `samples` (the same list
    on every rank) in one `--batch`-slot pool (restarts.run_pool: the reference's per-sample check
    schedule and convergence rule, converged samples written by this rank at once, freed slots
    refilled from the block); then one all-gather (restarts.gather_results: RCCL over xGMI under
    nccl) of every rank's (sample, iterations, converged, likelihood, held-out likelihood).  Rank 0
    prints one summary line per sample, in sample order, as run_batch does.  Returns the gathered
    results."""
    import torch.distributed as dist
    from .restarts import gather_results, shard_samples
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    mine = {samples[i] for i in shard_samples(len(samples), world, rank)}

    def done(r):
        if r.converged:
            _write_result(model, cfg, r)
    local = _pool(model, cfg, samples, mine, engine_factory, done, stats)
    rows = gather_results(local, len(samples), group=group, device=device)
    if rank == 0:
        for r in rows:
            out(_summary(r))
    return rows


def spawn_ranks(n, argv):
    """`--gpus N` without a launcher: N copies of this command, one rank per GPU, started before
    this process touches a GPU; every rank is watched at once and the first failure ends the
    others (launch.wait_ranks).  The parent's seed is passed on, so every rank replays the same
    RNG stream (:1149 seeds it once per run)."""
    from .launch import spawn_ranks as spawn
    if not any(a == "--seed" or a.startswith("--seed=") for a in argv):
        argv = list(argv) + ["--seed", str(os.getpid())]
    return spawn([sys.executable, "-m", "trigenicinteractionpredictor_amd.cli", *argv], n)


def _too_many_ranks(cfg, out):
    """RCCL takes one GPU per rank: --gpus above the visible GPUs would put two ranks of one
    communicator on one device (refused or hung), so it is an argument error (gloo ranks may
    share a GPU: a rehearsal mode).  The launching parent counts GPUs from sysfs (no HIP call
    before the ranks exist; launch.visible_gpus); a rank, which uses the GPU anyway, asks the
    runtime."""
    if cfg["backend"] != "nccl":
        return False
    if "WORLD_SIZE" in os.environ:
        import torch
        n = torch.cuda.device_count()
    else:
        from .launch import visible_gpus
        n = visible_gpus()
        if n is None:          # topology unreadable: the ranks check
            return False
    if cfg["gpus"] > n:
        out("\n\nERROR: --gpus %d with the nccl backend needs %d GPUs, %d visible (--backend gloo "
            "shares GPUs)" % (cfg["gpus"], cfg["gpus"], n))
        return True
    return False


def main(argv=None, model_factory=None, out=print, engine_factory=None):
    argv = sys.argv[1:] if argv is None else argv
    cfg = dict(DEFAULTS)
    cfg["seed"] = os.getpid()                                    # :1149
    try:
        cfg = parse(argv, cfg)
    except ArgError:
        return 2
    if cfg.get("help"):
        return 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if cfg["gpus"] > 1 and _too_many_ranks(cfg, out):
        return 2
    if cfg["gpus"] > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(cfg["gpus"], argv)                   # before any GPU call
    if world != cfg["gpus"]:
        out("\n\nERROR: WORLD_SIZE=%d but --gpus %d" % (world, cfg["gpus"]))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    group_on = world > 1
    device = None
    if group_on:
        import torch
        import torch.distributed as dist
        if cfg["backend"] == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", device_id=device)
        else:
            if torch.cuda.is_available():           # ranks sharing the box's GPUs (rehearsal)
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
            dist.init_process_group("gloo")
        # one RNG stream for the run (:1149): under an external launcher a rank given no --seed
        # seeded from its own pid, so every rank takes rank 0's seed
        box = [cfg["seed"]]
        dist.broadcast_object_list(box, src=0)
        cfg["seed"] = box[0]
        if rank != 0:
            out = _quiet
    try:
        return _main_ranked(cfg, model_factory, out, engine_factory, group_on, device)
    finally:
        if group_on:
            import torch.distributed as dist
            dist.barrier()
            dist.destroy_process_group()


def _quiet(*_a, **_k):
    return None


def _main_ranked(cfg, model_factory, out, engine_factory, group_on, device):
    random.seed(cfg["seed"])
    if int(cfg["fcheck"]) > int(cfg["iterations"]):
        out("\n\nWARNING: the likelihood frequency checking is bigger that the number of num_iterations "
            "per sample.")
        out("likelihood will only be calculated at the end of every sample (equivalent to --check=0 or -c 0)\n")
    msg = ("\n****************************************\n* Trigenic Interaction Predictor (MI355X) *"
           "\n****************************************\n\nDoing " + str(cfg["samples"]) + " samples of "
           + str(cfg["iterations"]) + " num_iterations.\nTrain-file is " + str(cfg["train"])
           + "\n Test-file is " + str(cfg["test"]) + "\n Output directory is " + str(cfg["out"])
           + "\nK value (number of groups) is " + str(cfg["k"]) + ".\nLikelihood will be computed every "
           + str(cfg["fcheck"]) + " num_iterations after iteration number " + str(cfg["bcheck"]))
    out(msg)
    if model_factory is None:
        from .model import Model as model_factory
    model = model_factory()
    model.get_traintest(cfg["train"], cfg["test"])
    out("\nStarting algorithm...")
    pending = []
    for sample in range(cfg["sample_ini"], cfg["sample_ini"] + int(cfg["samples"])):
        outfile = cfg["out"] + "Sample_" + str(sample) + "_K" + str(cfg["k"]) + ".csv"
        if os.path.isfile(outfile):                              # :1256-1257
            continue
        if cfg["batch"] > 1 or group_on:
            pending.append(sample)
        else:
            run_sample(model, cfg, sample, outfile, out)
    if group_on:
        import torch.distributed as dist
        dist.barrier()           # every rank has its pending list before any rank writes a file
        run_ranked(model, cfg, pending, out, engine_factory, device=device)
    elif pending:
        run_batch(model, cfg, pending, out, engine_factory)
    return 0


if __name__ == "__main__":
    sys.exit(main())
