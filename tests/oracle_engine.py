"""CPU stand-in for EMEngine built on the C oracle (test infrastructure only): same
upload / iterate / loglik / download interface, one sample at a time, so the
restart driver and its gloo sharding can be tested without a GPU."""
import numpy as np

from oracle import c_oracle


class _Slots:
    """EMEngine's sample-slot interface (restarts.run_pool) over per-sample host arrays."""

    def _slots(self, B):
        if getattr(self, "theta", None) is None or len(self.theta) != B:
            self.theta, self.pr = [None] * B, [None] * B
        self.B = B
        self.active = getattr(self, "active", B)

    def upload_slot(self, b, theta, pr):
        self.theta[b] = np.array(theta, dtype=np.float64)
        self.pr[b] = np.array(pr, dtype=np.float64)

    def download_slot(self, b):
        return self.theta[b].copy(), self.pr[b].copy()

    def move_slot(self, dst, src):
        if dst != src:
            self.theta[dst], self.pr[dst] = self.theta[src].copy(), self.pr[src].copy()

    def set_active(self, n):
        assert 0 < n <= self.B
        self.active = n
        self.log.append(("active", n))

    def _live(self):
        return range(min(self.active, len(self.theta)))


class OracleEngine(_Slots):
    def __init__(self, links, test_links, B=None):
        self.ids, self.counts = c_oracle.links_to_arrays(links)
        self.tids, self.tcounts = c_oracle.links_to_arrays(test_links)
        self.log = []          # ("iterate", n, live slots) / ("active", n): what the driver asked
        self.theta = None
        if B is not None:
            self._slots(B)

    def upload(self, theta, pr):
        self.theta = [np.array(t) for t in theta]
        self.pr = [np.array(p) for p in pr]
        self.B = self.active = len(self.theta)

    def iterate(self, n):
        self.log.append(("iterate", n, self.active))
        for _ in range(n):
            for s in self._live():
                self.theta[s], self.pr[s] = c_oracle.make_iteration(self.ids, self.counts,
                                                                    self.theta[s], self.pr[s])

    def loglik(self, which):
        ids, counts = (self.ids, self.counts) if which == 0 else (self.tids, self.tcounts)
        out = np.full(len(self.theta), np.nan)
        for s in self._live():
            out[s] = c_oracle.loglik(ids, counts, self.theta[s], self.pr[s]) if ids.shape[0] else 0.0
        return out

    def download(self):
        return np.stack(self.theta), np.stack(self.pr)


class OracleShardEngine(_Slots):
    """CPU stand-in for the link-sharded EMEngine methods (set_links with a global degree,
    accumulate, mstep) on oracle/shard_oracle.py, B batched samples."""

    def __init__(self, K, P, B=1, R=2, eps=1e-10):
        self.K, self.P, self.B, self.R, self.eps = K, P, B, R, eps
        self.device = "cpu"
        self.sets = {}
        self.deg = None
        self.log = []
        self.theta = None
        self._slots(B)

    def set_links(self, which, ids, counts, deg=None):
        self.sets[which] = (np.asarray(ids, np.int32), np.asarray(counts, np.int32))
        if which == 0:
            self.deg = np.asarray(deg if deg is not None else
                                  np.bincount(np.asarray(ids).ravel(), minlength=self.P)[:self.P])

    def upload(self, theta, pr):
        self.theta = [np.array(t, dtype=np.float64) for t in theta]
        self.pr = [np.array(p, dtype=np.float64) for p in pr]

    def download(self):
        return np.stack(self.theta), np.stack(self.pr)

    def accumulate(self, nth, S):
        import torch
        from oracle import shard_oracle
        ids, counts = self.sets[0]
        for b in self._live():
            n, s = shard_oracle.accumulate(ids, counts, self.theta[b], self.pr[b], self.eps)
            nth[b].copy_(torch.from_numpy(n))
            S[b].copy_(torch.from_numpy(s))

    def mstep(self, nth, S):
        from oracle import shard_oracle
        for b in self._live():
            self.theta[b], self.pr[b] = shard_oracle.mstep(self.theta[b], self.pr[b], nth[b].numpy(),
                                                           S[b].numpy(), self.deg, self.eps)

    def loglik(self, which):
        ids, counts = self.sets[which]
        out = np.full(self.B, np.nan)
        for b in self._live():
            out[b] = c_oracle.loglik(ids, counts, self.theta[b], self.pr[b]) if ids.shape[0] else 0.0
        return out


class OracleJointEngine:
    """CPU stand-in for joint.JointEngine on the C oracle's joint iteration (bit-exact with the
    reference `_23`): lets the joint Model, its text output and cli23 run on the CPU."""

    def __init__(self, K, P, B=1, R=2, eps=1e-10, device=None):
        self.K, self.P, self.B, self.R, self.eps = K, P, B, R, eps
        self.sets = {}

    def set_links(self, which, ids3, counts3, ids2, counts2):
        self.sets[which] = tuple(np.ascontiguousarray(a, dtype=np.int32)
                                 for a in (np.reshape(ids3, (-1, 3)), np.reshape(counts3, (-1, self.R)),
                                           np.reshape(ids2, (-1, 2)), np.reshape(counts2, (-1, self.R))))

    def upload(self, theta, pr, qr):
        self.theta = [np.array(t, dtype=np.float64) for t in theta]
        self.pr = [np.array(p, dtype=np.float64) for p in pr]
        self.qr = [np.array(q, dtype=np.float64) for q in qr]

    def download(self):
        return np.stack(self.theta), np.stack(self.pr), np.stack(self.qr)

    def iterate(self, n=1):
        for _ in range(int(n)):
            for s in range(len(self.theta)):
                self.theta[s], self.pr[s], self.qr[s] = c_oracle.joint_make_iteration(
                    *self.sets[0], self.theta[s], self.pr[s], self.qr[s])

    def loglik(self, which=0):
        return np.array([c_oracle.joint_loglik(*self.sets[which], t, p, q)
                         for t, p, q in zip(self.theta, self.pr, self.qr)])

    def predict(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        f = c_oracle.predict if ids.shape[1] == 3 else c_oracle.pair_predict
        lat = self.pr if ids.shape[1] == 3 else self.qr
        return np.stack([f(ids, t, q) for t, q in zip(self.theta, lat)])

    def close(self):
        pass
