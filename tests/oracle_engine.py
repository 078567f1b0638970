"""CPU stand-in for EMEngine built on the C oracle (test infrastructure only): same
upload / iterate / loglik / download interface, one sample at a time, so the
restart driver and its gloo sharding can be tested without a GPU."""
import numpy as np

from oracle import c_oracle


class OracleEngine:
    def __init__(self, links, test_links):
        self.ids, self.counts = c_oracle.links_to_arrays(links)
        self.tids, self.tcounts = c_oracle.links_to_arrays(test_links)

    def upload(self, theta, pr):
        self.theta = [np.array(t) for t in theta]
        self.pr = [np.array(p) for p in pr]

    def iterate(self, n):
        for _ in range(n):
            for s in range(len(self.theta)):
                self.theta[s], self.pr[s] = c_oracle.make_iteration(self.ids, self.counts,
                                                                    self.theta[s], self.pr[s])

    def loglik(self, which):
        ids, counts = (self.ids, self.counts) if which == 0 else (self.tids, self.tcounts)
        if ids.shape[0] == 0:
            return np.zeros(len(self.theta))
        return np.array([c_oracle.loglik(ids, counts, t, p) for t, p in zip(self.theta, self.pr)])

    def download(self):
        return np.stack(self.theta), np.stack(self.pr)
