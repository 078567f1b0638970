"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Pure-Python CPU restatement of the joint digenic + trigenic EM of
AleixMT/TrigenicInteractionPredictor, `src/TrigenicInteractionPredictor_23.py`,
under the spec fix written in DESIGN.md ("Joint digenic + trigenic model"):
`DataType.ALL` (:105, :194, :209, :296), which the enum (:31-34) does not
define, reads as `DataType.all`.  Nothing else is changed.

Loop order and binary64 operation order follow the reference, so this is
bit-identical to the reference under CPython; `tests/test_joint_oracle.py`
checks it against fixtures written by importing the reference
(`tests/golden/make_joint_golden.py`).

Cited reference lines (all in src/TrigenicInteractionPredictor_23.py):
  ingestion        `get_train_test`              :393-546
  RNG init         `initialize_parameters`       :123-220
  EM step          `make_iteration`              :1572-1687
  log-likelihood   `compute_likelihood`          :1534-1562
  prediction       `do_prediction`               :946-973
  test-set table   `calculate_test_set_results`  :983-1004
  metrics          `calculate_metrics`           :1018-1076
"""
from __future__ import annotations

import math
import random
import re

from oracle.mmsbm_oracle import EPS, R, OracleModel

HO_DELTA = "hoΔ"   # the filler allele removed from every key (:405-410)

ALL, TRIGENIC, DIGENIC = 0, 3, 2   # DataType values (:31-34)


class OracleJointModel(OracleModel):
    """The `_23` Model state (:43-105): the triplet state plus the pair lattice qr and dlinks."""

    def __init__(self):
        super().__init__()
        self.qr = []
        self.dlinks = {}
        self.dtest_links = {}
        self.gene_num_aparitions = self.uniqueg
        self.data_type = ALL

    # --- :393-546 -------------------------------------------------------
    def _register_names(self, names):
        ids = []
        for g in names:
            if g not in self.gene_id:
                n = len(self.id_gene)
                self.gene_id[g] = n
                self.id_gene[n] = g
                self.uniqueg[n] = 0
            n = self.gene_id[g]
            self.uniqueg[n] += 1
            ids.append(str(n))
        ids.sort()
        return "_".join(ids)

    @staticmethod
    def _names(field):
        names = field.split("_")
        if HO_DELTA in names:
            names.remove(HO_DELTA)   # first occurrence only (list.remove)
        return names

    def get_train_test(self, trainfile, testfile):
        with open(trainfile, encoding="utf-8") as f:
            for line in f.readlines():
                fields = line.strip().split("\t")
                names = self._names(fields[0])
                r = int(fields[1])
                key = self._register_names(names)
                if len(names) == 3:
                    self.links.setdefault(key, [0] * 2)[r] += 1
                if len(names) == 2:
                    self.dlinks.setdefault(key, [0] * 2)[r] += 1
        with open(testfile, encoding="utf-8") as f:
            for line in f.readlines():
                fields = re.split(r"\t+", line)
                names = self._names(fields[0])
                r = int(fields[1])
                key = self._register_names(names)
                # every test line lands in test_links (:511-516); triplets a second time (:518-525),
                # pairs also in dtest_links (:526-533)
                self.test_links.setdefault(key, [0] * 2)[r] += 1
                if len(names) == 3:
                    self.test_links[key][r] += 1
                if len(names) == 2:
                    self.dtest_links.setdefault(key, [0] * 2)[r] += 1
        self.P = len(self.id_gene)

    # --- :123-220 -------------------------------------------------------
    def initialize_parameters(self, k=2, interaction=ALL, rand=random.random):
        K = self.K = int(k)
        Rn = self.R
        self.data_type = interaction
        self.theta = [[rand() for _ in range(K)] for _ in range(self.P)]
        self.pr = [[[[rand() for _ in range(Rn)] for _ in range(K)] for _ in range(K)] for _ in range(K)]
        self.qr = [[[rand() for _ in range(Rn)] for _ in range(K)] for _ in range(K)]
        for g in range(self.P):
            s = 0.
            for v in self.theta[g]:
                s += v
            if s < self.eps:
                self.theta[g] = [rand() for _ in range(K)]
            s = sum(self.theta[g])
            row = self.theta[g]
            for a in range(K):
                row[a] = row[a] / s if s != 0 else row[a] / (s + self.eps)
        if interaction in (ALL, TRIGENIC):
            for a in range(K):
                for b in range(K):
                    for c in range(K):
                        self._normalise_cell(self.pr[a][b][c])
        if interaction in (ALL, DIGENIC):
            for a in range(K):
                for b in range(K):
                    self._normalise_cell(self.qr[a][b])

    def _normalise_cell(self, cell):
        s = 0.
        for r in range(self.R):
            s += cell[r]
        for r in range(self.R):
            cell[r] = cell[r] / s if s != 0 else cell[r] / (s + self.eps)

    # --- :1534-1562 -----------------------------------------------------
    def compute_likelihood(self, selected_set="train"):
        total = super().compute_likelihood("train")
        K, Rn, th, qr = self.K, self.R, self.theta, self.qr
        for key, n in self.dlinks.items():
            s1, s2 = key.split("_")
            t1, t2 = th[int(s1)], th[int(s2)]
            d = [self.eps] * Rn
            for a in range(K):
                for b in range(K):
                    for r in range(Rn):
                        d[r] += t1[a] * t2[b] * qr[a][b][r]
            for r in range(Rn):
                total += n[r] * math.log(d[r])
        self.likelihood = total
        return total

    # --- :1572-1687 -----------------------------------------------------
    def make_iteration(self):
        nth, npr, deg = self.accumulate(self.links.items())
        nqr = self.accumulate_pairs(self.dlinks.items(), nth, deg)
        self.finish(nth, npr, deg)
        for a in range(self.K):
            for b in range(self.K):
                acc = nqr[a][b]
                s = self.eps
                for r in range(self.R):
                    s += acc[r]
                for r in range(self.R):
                    acc[r] /= s
        self.qr = nqr

    def accumulate_pairs(self, items, nth, deg):
        """Pair loop of :1608-1635, adding into the triplet loop's ntheta / counter."""
        K, Rn, th, qr = self.K, self.R, self.theta, self.qr
        nqr = [[[0.] * Rn for _ in range(K)] for _ in range(K)]
        for key, n in items:
            s1, s2 = key.split("_")
            g1, g2 = int(s1), int(s2)
            t1, t2 = th[g1], th[g2]
            deg[g1] += 1
            deg[g2] += 1
            d = [self.eps] * Rn
            for a in range(K):
                for b in range(K):
                    for r in range(Rn):
                        d[r] += t1[a] * t2[b] * qr[a][b][r]
            n1, n2 = nth[g1], nth[g2]
            for a in range(K):
                for b in range(K):
                    acc = nqr[a][b]
                    for r in range(Rn):
                        w = (t1[a] * t2[b] * qr[a][b][r]) / d[r]
                        n1[a] += w * n[r]
                        n2[b] += w * n[r]
                        acc[r] += w * n[r]
        return nqr

    # --- :946-1076 ------------------------------------------------------
    def do_prediction_ids(self, ids):
        K, th = self.K, self.theta
        p = 0
        if len(ids) == 3:
            i1, i2, i3 = ids
            for a in range(K):
                for b in range(K):
                    for c in range(K):
                        p += th[i1][a] * th[i2][b] * th[i3][c] * self.pr[a][b][c][1]
        if len(ids) == 2:
            i1, i2 = ids
            for a in range(K):
                for b in range(K):
                    p += th[i1][a] * th[i2][b] * self.qr[a][b][1]
        return p

    def calculate_test_set_results(self):
        self.results = []
        for table in (self.test_links, self.dtest_links):
            for key, n in table.items():
                real = 0 if n[0] else 1
                ids = [int(s) for s in key.split("_")]
                self.results.append([self.do_prediction_ids(ids), key, real])
        self.results.sort()
        self.results.reverse()

    def calculate_metrics(self):
        npos = sum(1 for n in self.links.values() if n[1] == 1)
        npos += sum(1 for n in self.dlinks.values() if n[1] == 1)
        frac = npos / (len(self.links) + len(self.dlinks))
        want = int(frac * len(self.test_links))
        cut = 0
        for idx, row in enumerate(self.results):
            if idx == want:
                cut = row[0]
                break
        pos = [row for row in self.results if row[2]]
        neg = [row for row in self.results if not row[2]]
        better = 0
        for p in pos:
            for q in neg:
                if p[0] > q[0]:
                    better += 1
        auc = better / (len(pos) * len(neg))
        tp = fp = fn = tn = 0
        for row in self.results:
            if row[0] >= cut:
                if row[2]:
                    tp += 1
                else:
                    fp += 1
            elif row[2]:
                fn += 1
            else:
                tn += 1
        return [tp / (tp + fp), tp / (tp + fn), fp / (fp + tn), auc]
