"""Link sharding of ONE EM sample across ranks — SURVEY.md §8e, secondary mode (config 5:
one sample of a 10M-link set spread over the GPUs of a node).

The reference accumulates every train link into `ntheta` / `npr` (`make_iteration`,
src/TrigenicInteractionPredictor.py:986-1012) and only then normalises (:1016-1028).  The
accumulation is a sum over links, so each rank owns a contiguous 1/N block of the train links
and accumulates only those:

    nth[B][P][K]   per gene, the sum of its local c-scaled Y / Z / W rows  (mmsbm_accumulate)
    S[B][R][K^3]   the S lattice sums                                      (npr = p S)

`nth` and `S` live in ONE device buffer, summed over ranks with one all-reduce per iteration
(RCCL over xGMI for `nccl`: P*K + K^3*R doubles, 12.4 MB at P=50k, K=30), after which every
rank applies the same M-step (mmsbm_mstep) and holds identical theta / p.  The degree
(`counter`, :986-994) is taken over ALL train links, so a gene seen only in another rank's
block still divides by its true degree, and a gene with no train link anywhere raises
ZeroDivisionError on every rank, as :1018 does.

`LinkShardedEM` has the upload / iterate / loglik / download interface of `EMEngine`, so the
restart driver's convergence loop (`restarts.run_pool`) runs it unchanged; likelihoods are
summed over ranks the same way (the test links are sharded too).
"""
from __future__ import annotations

import numpy as np

TRAIN, TEST = 0, 1


def shard_links(n_links: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) block of the links (dict insertion order) for `rank`."""
    base, extra = divmod(n_links, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def train_degree(ids: np.ndarray, P: int) -> np.ndarray:
    """The reference's `counter` (:986-994) over all train links: occurrences per gene in
    the three slots, a repeated gene counted each time."""
    return np.bincount(ids.ravel().astype(np.int64), minlength=P)[:P].astype(np.int32)


class LinkShardedEM:
    """One (batch of) sample(s) whose train / test links are split over the process group.

    `engine` is an EMEngine (or a CPU stand-in with the same methods) of shape B, P, K, R.
    Without an initialised process group it runs alone and is the plain iteration."""

    def __init__(self, engine, ids, counts, tids, tcounts, group=None):
        import torch
        import torch.distributed as dist
        self.dist_on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = dist.get_world_size(group) if self.dist_on else 1
        self.rank = dist.get_rank(group) if self.dist_on else 0
        self.engine = engine
        ids, counts = np.asarray(ids, np.int32), np.asarray(counts, np.int32)
        tids, tcounts = np.asarray(tids, np.int32), np.asarray(tcounts, np.int32)
        lo, hi = shard_links(ids.shape[0], self.world, self.rank)
        tlo, thi = shard_links(tids.shape[0], self.world, self.rank)
        self.n_local = hi - lo
        engine.set_links(TRAIN, ids[lo:hi], counts[lo:hi], deg=train_degree(ids, engine.P))
        engine.set_links(TEST, tids[tlo:thi], tcounts[tlo:thi])
        B, P, K, R = engine.B, engine.P, engine.K, engine.R
        n_th = B * P * K
        self.buf = torch.zeros(n_th + B * R * K ** 3, dtype=torch.float64, device=engine.device)
        self.nth = self.buf[:n_th].view(B, P, K)
        self.S = self.buf[n_th:].view(B, R, K ** 3)
        self.B = B
        self.active = B
        self.device = engine.device

    def _sum(self, t):
        """Sum over ranks in place (one collective, also in a world of one when a process group
        exists: bench.py --process-group runs the RCCL all-reduce on one GPU); gloo reduces a host
        copy."""
        if not self.dist_on:
            return t
        import torch.distributed as dist
        if t.is_cuda and dist.get_backend(self.group) == "gloo":
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    # ----------------------------------------------- EMEngine-compatible interface
    def upload(self, theta, pr):
        self.engine.upload(theta, pr)

    def download(self):
        return self.engine.download()

    # sample slots (restarts.run_pool): every rank holds the same B samples, so slot operations
    # are local and identical on every rank
    def upload_slot(self, b, theta, pr):
        self.engine.upload_slot(b, theta, pr)

    def download_slot(self, b):
        return self.engine.download_slot(b)

    def move_slot(self, dst, src):
        self.engine.move_slot(dst, src)

    def set_active(self, n):
        """Shrink (or restore) the active prefix: accumulate / mstep cover samples [0, n) only, so
        the collective does too (the inactive slots' sums are stale and are never reduced)."""
        self.engine.set_active(n)
        self.active = int(n)

    def iterate(self, n_iters: int = 1):
        a = self.active
        for _ in range(int(n_iters)):
            self.engine.accumulate(self.nth, self.S)
            if a == self.B:
                self._sum(self.buf)          # one collective over the whole buffer
            else:                            # the active prefix of each part (B is the leading dim)
                self._sum(self.nth[:a])
                self._sum(self.S[:a])
            self.engine.mstep(self.nth, self.S)

    def loglik(self, which: int = TRAIN) -> np.ndarray:
        import torch
        local = torch.as_tensor(np.asarray(self.engine.loglik(which), dtype=np.float64))
        if self.dist_on and getattr(self.buf, "is_cuda", False):
            import torch.distributed as dist
            if dist.get_backend(self.group) != "gloo":
                local = local.to(self.buf.device)
        return self._sum(local).cpu().numpy()

    def synchronize(self):
        sync = getattr(self.engine, "synchronize", None)
        if sync is not None:
            sync()
