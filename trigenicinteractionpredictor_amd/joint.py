"""Joint digenic + trigenic model — drop-in for the reference class `Model` of
`src/TrigenicInteractionPredictor_23.py` (AleixMT/TrigenicInteractionPredictor).

The reference module cannot be instantiated as written: `Model()` raises `AttributeError: ALL`
because the enum (:31-34) defines `all` while :105, :194, :209 and :296 name `ALL`.  This mirror
implements the spec fix recorded in DESIGN.md ("Joint digenic + trigenic model"):

  1. `DataType.ALL` reads as `DataType.all` (:105, :194, :209, :296);
  2. `compare_links` reads the other model's `nLinks` (:1503 names `nlinks`, which `_23` lacks);
  3. the sample driver (`cli23.py`, for `src/trigenic_fromtesttrain_2+3.py`) appends to
     `likelihoodVector` (:78, :86 name `vlikelihood`) and starts at sample 0 on the default path
     (:53 sets `itini`, :72 reads `sampleini`).

Everything else keeps the reference's behaviour, including its quirks: a test triplet is
counted twice in `test_links` (:511-525), a test pair lands in both `test_links` and
`dtest_links` (:511-533), `to_string` prints no test table, `pair_fast_fold` without `output`
ends in `UnboundLocalError` (:938).

The EM hot path (`make_iteration` :1572-1687, `compute_likelihood` :1534-1562) and the bulk
test-set prediction (`do_prediction` :946-973 as used by `calculate_test_set_results`
:983-1004) run as HIP kernels: the triplet lattice on the engine of include/mmsbm.h, the pair
lattice on include/mmsbm_pairs.h (`JointEngine`).  There is no CPU fallback.
"""
from __future__ import annotations

import codecs
import random
import re
from enum import Enum

import numpy as np

from . import _lib
from .layout import links_to_arrays
from .tracked import TrackedLinks, TrackedTable, version_of

HO_DELTA = "hoΔ"   # the filler allele removed from every key (:318-323, :405-410)


class DataType(Enum):
    """:31-34."""
    all = 0
    trigenic = 3
    digenic = 2


def _pair_arrays(links: dict, R: int = 2):
    """`dlinks`-like dict ("i_j" -> counts) in insertion order -> (ids int32[E][2], counts)."""
    E = len(links)
    ids = np.empty((E, 2), dtype=np.int32)
    counts = np.zeros((E, R), dtype=np.int32)
    for e, (key, n) in enumerate(links.items()):
        a, b = key.split("_")
        ids[e] = (int(a), int(b))
        counts[e] = n[:R]
    return ids, counts


class JointEngine:
    """Device state of the joint model: the triplet engine (theta, pr) plus the pair context
    (qr f64[B][R][K^2]).  One iteration = triplet accumulate, pair accumulate into the same
    ntheta, M-step of theta / pr with the joint counter, qr M-step (include/mmsbm_pairs.h)."""

    def __init__(self, K: int, P: int, B: int = 1, R: int = 2, eps: float = 1e-10, device=None,
                 family="sku"):
        import ctypes

        import torch

        from .engine import EMEngine
        self._ct = ctypes
        # the triplet half keeps one small-K kernel family for every B (the three-stream fused
        # E-step, whose fin adds the pair sums and runs the q cells), so batched joint samples keep
        # their one-sample bits
        self.tri = EMEngine(K, P, B=B, R=R, eps=eps, device=device, family=family)
        self.lib, self.device = self.tri.lib, self.tri.device
        self.K, self.P, self.B, self.R, self.eps = self.tri.K, self.tri.P, self.tri.B, self.tri.R, self.tri.eps
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.mmsbm_pairs_create(self.device.index, ctypes.byref(ctx)))
        self.pctx = ctx
        _lib.check(self.lib.mmsbm_pairs_set_shape(self.pctx, self.K, self.R, self.B, self.P, self.eps))
        z = dict(dtype=torch.float64, device=self.device)
        self.qr = torch.zeros((self.B, self.R, self.K * self.K), **z)
        self.nth = torch.zeros((self.B, self.P, self.K), **z)
        self.S = torch.zeros((self.B, self.R, self.K ** 3), **z)
        self.S2 = torch.zeros((self.B, self.R, self.K * self.K), **z)
        self.pworkspace = None
        self._sets = set()
        self._torch = torch

    @property
    def theta(self):
        return self.tri.theta

    @property
    def pr(self):
        return self.tri.pr

    def set_links(self, which: int, ids3, counts3, ids2, counts2):
        """Triplet (ids int32[E3][3]) and pair (ids int32[E2][2]) tables of one set.  For the
        train set the degree is the joint `counter` (:1574-1617): triplet slots + pair slots."""
        ids3 = np.ascontiguousarray(ids3, dtype=np.int32).reshape(-1, 3)
        ids2 = np.ascontiguousarray(ids2, dtype=np.int32).reshape(-1, 2)
        counts3 = np.ascontiguousarray(counts3, dtype=np.int32).reshape(-1, self.R)
        counts2 = np.ascontiguousarray(counts2, dtype=np.int32).reshape(-1, self.R)
        deg = None
        if which == _lib.SET_TRAIN:
            deg = (np.bincount(ids3.ravel(), minlength=self.P)[:self.P]
                   + np.bincount(ids2.ravel(), minlength=self.P)[:self.P]).astype(np.int32)
        self.tri.set_links(which, ids3, counts3, deg=deg)
        hp = lambda a: a.ctypes.data_as(self._ct.c_void_p) if a.size else None
        _lib.check(self.lib.mmsbm_pairs_set_links(self.pctx, which, hp(ids2), hp(counts2), int(ids2.shape[0])))
        self._sets.add(which)
        nbytes = self._ct.c_int64()
        _lib.check(self.lib.mmsbm_pairs_workspace_bytes(self.pctx, self._ct.byref(nbytes)))
        need = max(int(nbytes.value), 256)
        if self.pworkspace is None or self.pworkspace.numel() < need:
            self.pworkspace = self._torch.empty(need, dtype=self._torch.uint8, device=self.device)
        _lib.check(self.lib.mmsbm_pairs_set_workspace(self.pctx, self.pworkspace.data_ptr(),
                                                      self.pworkspace.numel()))

    def upload(self, theta, pr, qr):
        """theta [B][P][K]; pr [B][K][K][K][R]; qr [B][K][K][R] (the reference nestings)."""
        self.tri.upload(theta, pr)
        qr = np.asarray(qr, dtype=np.float64).reshape(self.B, self.K * self.K, self.R)
        self.qr.copy_(self._torch.from_numpy(np.ascontiguousarray(qr.transpose(0, 2, 1))))

    def download(self):
        """-> theta [B][P][K], pr [B][K][K][K][R], qr [B][K][K][R] (host numpy)."""
        th, pr = self.tri.download()
        qr = self.qr.cpu().numpy().transpose(0, 2, 1).reshape(self.B, self.K, self.K, self.R)
        return th, pr, np.ascontiguousarray(qr)

    def _stream(self):
        return self._torch.cuda.current_stream(self.device).cuda_stream

    def iterate(self, n_iters: int = 1):
        """n joint iterations (mmsbm_joint_iterate): per iteration the pair launch (pair sums,
        S2 partials), then the triplet iteration whose fin adds the pair sums before the
        division by the joint counter and applies the qr M-step."""
        if _lib.SET_TRAIN not in self._sets:
            raise RuntimeError("train links not set")
        _lib.check(self.lib.mmsbm_joint_iterate(self.tri.ctx, self.pctx, self.theta.data_ptr(),
                                                self.pr.data_ptr(), self.qr.data_ptr(), self.nth.data_ptr(),
                                                int(n_iters), self._stream()))

    def iterate_unfused(self, n_iters: int = 1):
        """The same iterations through the accumulate / M-step halves (include/mmsbm_pairs.h):
        the building blocks a link-sharded joint run would all-reduce between."""
        s = self._stream()
        th, pr, qr = self.theta.data_ptr(), self.pr.data_ptr(), self.qr.data_ptr()
        nth, S, S2 = self.nth.data_ptr(), self.S.data_ptr(), self.S2.data_ptr()
        _lib.check(self.lib.mmsbm_set_theta_addend(self.tri.ctx, None))
        for _ in range(int(n_iters)):
            _lib.check(self.lib.mmsbm_accumulate(self.tri.ctx, th, pr, nth, S, s))
            _lib.check(self.lib.mmsbm_pairs_accumulate(self.pctx, th, qr, nth, S2, s))
            _lib.check(self.lib.mmsbm_mstep(self.tri.ctx, th, pr, nth, S, s))
            _lib.check(self.lib.mmsbm_pairs_qstep(self.pctx, qr, S2, s))

    def loglik(self, which: int = _lib.SET_TRAIN) -> np.ndarray:
        """Triplet + pair log-likelihood of set `which` per sample (:1534-1562)."""
        L3 = self.tri.loglik_async(which) if which in self.tri._sets else None
        L2 = self._torch.empty(self.B, dtype=self._torch.float64, device=self.device)
        _lib.check(self.lib.mmsbm_pairs_loglik(self.pctx, which, self.theta.data_ptr(), self.qr.data_ptr(),
                                               L2.data_ptr(), self._stream()))
        out = L2.cpu().numpy()
        return out if L3 is None else L3.cpu().numpy() + out

    def predict(self, ids: np.ndarray) -> np.ndarray:
        """P(r=1) for each row of ids int32[n][3] (pr) or int32[n][2] (qr) -> [B][n] (host)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        if ids.shape[1] == 3:
            return self.tri.predict(ids)
        n = int(ids.shape[0])
        out = self._torch.empty((self.B, max(n, 1)), dtype=self._torch.float64, device=self.device)
        if n:
            ids_d = self._torch.from_numpy(ids).to(self.device)
            _lib.check(self.lib.mmsbm_pairs_predict(self.pctx, ids_d.data_ptr(), n, self.theta.data_ptr(),
                                                    self.qr.data_ptr(), out.data_ptr(), self._stream()))
        return out[:, :n].cpu().numpy()

    def plan_info(self, which: int = _lib.SET_TRAIN) -> dict:
        v = (self._ct.c_int64 * 7)()
        _lib.check(self.lib.mmsbm_pairs_plan_info(self.pctx, which, v))
        info = dict(zip(("pair_observations", "pair_entries", "pair_parts", "pair_em_wgs", "pair_wg_genes_max",
                         "pair_wg_parts_max", "pair_ll_wgs"), [int(x) for x in v]))
        info.update(self.tri.plan_info(which))
        return info

    def close(self):
        if getattr(self, "pctx", None):
            self.lib.mmsbm_pairs_destroy(self.pctx)
            self.pctx = None
        if getattr(self, "tri", None) is not None:
            self.tri.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Model:
    """`Model` of src/TrigenicInteractionPredictor_23.py (:37-1697) under the spec fix."""

    Engine = JointEngine   # device engine class (tests substitute a CPU checker engine)
    # the train tables the device copy is built from; in-place edits change their version
    # (tracked.py), as the reference re-reads them on every call (:1572-1617)
    links = TrackedTable()
    dlinks = TrackedTable()

    def __init__(self, device=None):
        self.nTheta = []
        self._theta = []
        self.id_gene = {}
        self.gene_id = {}
        self._pr = []
        self.npr = []
        self._qr = []
        self.nqr = []
        self.nLinks = {}
        self.links = {}
        self.ndlinks = {}
        self.dlinks = {}
        self.test_links = {}
        self.dtest_links = {}
        self.results = []
        self.gene_num_aparitions = {}
        self.likelihood = 0
        self.likelihoodVector = []
        self.R = 2
        self.K = 0
        self.P = 0
        self.eps = 1e-10
        self.dataType = DataType.all       # :105 after the spec fix
        self._device = device
        self._engine = None
        self._engine_key = None
        self._host_fresh = True
        self._dev_fresh = False

    # ------------------------------------------------------------------ state
    def _pull(self):
        if self._host_fresh:
            return
        th, pr, qr = self._engine.download()
        self._theta, self._pr, self._qr = th[0].tolist(), pr[0].tolist(), qr[0].tolist()
        self._host_fresh = True

    def _param(name):  # noqa: N805 — property factory for theta / pr / qr
        def get(self):
            self._pull()
            self._dev_fresh = False   # the caller may edit the lists in place
            return getattr(self, name)

        def put(self, value):
            self._pull()
            setattr(self, name, value)
            self._dev_fresh = False
        return property(get, put)

    theta = _param("_theta")
    pr = _param("_pr")
    qr = _param("_qr")
    del _param

    def links_changed(self):
        """Declare an edit of the link dicts the tables cannot see (a key added to or removed
        from a dict assigned to `links` / `dlinks`; tracked.TrackedLinks): the tables re-read
        their source dicts and the device tables are rebuilt on the next call (the reference
        re-reads the dicts on every call)."""
        for t in (self.links, self.dlinks):
            t.resync()
        self._engine_key = None

    # copy.deepcopy / pickle: no device engine in the copy, tables tracked again
    def __getstate__(self):
        self._pull()
        state = dict(self.__dict__)
        state.update(_engine=None, _engine_key=None, _dev_fresh=False, _host_fresh=True)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        for name in ("_tracked_links", "_tracked_dlinks"):
            t = self.__dict__.get(name)
            if t is not None and not isinstance(t, TrackedLinks):
                self.__dict__[name] = TrackedLinks(t)

    def _ensure_engine(self):
        key = (self.K, self.P, version_of(self.links), version_of(self.dlinks))
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._pull()
                self._engine.close()
            eng = self.Engine(self.K, self.P, B=1, R=self.R, eps=self.eps, device=self._device)
            eng.set_links(_lib.SET_TRAIN, *links_to_arrays(self.links, self.R), *_pair_arrays(self.dlinks, self.R))
            self._engine = eng
            self._engine_key = key
            self._dev_fresh = False
        return self._engine

    def _push(self):
        eng = self._ensure_engine()
        if not self._dev_fresh:
            self._pull()
            eng.upload(np.array(self._theta, dtype=np.float64).reshape(1, self.P, self.K),
                       np.array(self._pr, dtype=np.float64)[None], np.array(self._qr, dtype=np.float64)[None])
            self._dev_fresh = True
        return eng

    @property
    def engine(self):
        return self._push()

    # ------------------------------------------------------------ :123-220
    def initialize_parameters(self, k=2, interaction=DataType.all):
        try:
            self.K = int(k)
        except ValueError:
            self.K = 2
        self.dataType = interaction
        self.likelihoodVector = []
        K, R, rnd = self.K, self.R, random.random
        self._theta = [[rnd() for _ in range(K)] for _ in range(self.P)]
        self.nTheta = [[0.0] * K for _ in range(self.P)]
        self._pr = [[[[rnd() for _ in range(R)] for _ in range(K)] for _ in range(K)] for _ in range(K)]
        self.npr = [[[[0.] * R for _ in range(K)] for _ in range(K)] for _ in range(K)]
        self._qr = [[[rnd() for _ in range(R)] for _ in range(K)] for _ in range(K)]
        self.nqr = [[[0.] * R for _ in range(K)] for _ in range(K)]
        for g in range(self.P):
            total = 0.
            for v in self._theta[g]:
                total += v
            if total < self.eps:
                self._theta[g] = [rnd() for _ in range(K)]
            total = sum(self._theta[g])
            row = self._theta[g]
            for a in range(K):
                row[a] = row[a] / total if total != 0 else row[a] / (total + self.eps)
        if self.dataType in (DataType.all, DataType.trigenic):
            for plane in self._pr:
                for line in plane:
                    for cell in line:
                        self._normalise(cell)
        if self.dataType in (DataType.all, DataType.digenic):
            for line in self._qr:
                for cell in line:
                    self._normalise(cell)
        self._host_fresh = True
        self._dev_fresh = False

    def _normalise(self, cell):
        total = 0.
        for v in cell:
            total += v
        for r in range(self.R):
            cell[r] = cell[r] / total if total != 0 else cell[r] / (total + self.eps)

    # ------------------------------------------------------- :266-546 (host)
    def _register(self, names, gid):
        ids = []
        for g in names:
            if g not in self.gene_id:
                self.gene_id[g] = gid
                self.id_gene[gid] = g
                self.gene_num_aparitions[gid] = 0
                gid += 1
            n = self.gene_id[g]
            self.gene_num_aparitions[n] += 1
            ids.append(str(n))
        return ids, gid

    @staticmethod
    def _add(table, key, r):
        row = table.get(key)
        if row is None:
            table[key] = [0] * 2
            row = table[key]   # a tracked table stores its own row object
        row[r] += 1

    @staticmethod
    def _drop_filler(names):
        try:
            names.remove(HO_DELTA)
        except ValueError:
            pass

    def _store(self, names, ids, r, trip, ntrip, pair, npair):
        names.sort()
        ids.sort()
        key, nkey = '_'.join(ids), '_'.join(names)
        if len(names) == 3:
            self._add(trip, key, r)
            self._add(ntrip, nkey, r)
        if len(names) == 2:
            self._add(pair, key, r)
            self._add(npair, nkey, r)

    def get_input(self, file_path, cutoff_value=-0.08, discard=0):
        try:
            gid = 0
            with codecs.open(file_path, encoding='utf-8', mode='r') as fileref:
                line = fileref.readline()
                raw = len(re.split(r'\t+', line)) == 12
                for line in fileref.readlines():
                    fields = re.split(r'\t+', line)
                    if raw:
                        fields.pop(5)
                    if self.dataType != DataType.all and fields[4] != self.dataType.name:
                        continue
                    if float(fields[6]) >= 0.05:
                        r = 0
                    elif float(fields[5]) < cutoff_value:
                        r = 1
                    elif discard:
                        continue
                    else:
                        r = 0
                    names = fields[1].split('+')
                    names.append(fields[3])
                    self._drop_filler(names)
                    ids, gid = self._register(names, gid)
                    self._store(names, ids, r, self.links, self.nLinks, self.dlinks, self.ndlinks)
                self.P = len(self.id_gene)
        except ValueError as error:
            print(error)
        except IOError as error:
            print('Error, file does not exist or can\'t be read')
            print(error)

    def get_train_test(self, train_file_path, test_file_path):
        try:
            gid = 0
            with codecs.open(train_file_path, encoding='utf-8', mode='r') as file_ref:
                for line in file_ref.readlines():
                    fields = line.strip().split('\t')
                    names = fields[0].split('_')
                    self._drop_filler(names)
                    rating = int(fields[1])
                    ids, gid = self._register(names, gid)
                    self._store(names, ids, rating, self.links, self.nLinks, self.dlinks, self.ndlinks)
                self.P = len(self.id_gene)
            print('number of triplets, pairs', len(self.links), len(self.dlinks))
            with codecs.open(test_file_path, encoding='utf-8', mode='r') as file_ref:
                for line in file_ref.readlines():
                    fields = re.split(r'\t+', line)
                    names = fields[0].split('_')
                    self._drop_filler(names)
                    rating = int(fields[1])
                    ids, gid = self._register(names, gid)
                    names.sort()
                    ids.sort()
                    key = '_'.join(ids)
                    self._add(self.test_links, key, rating)          # every line (:511-516)
                    if len(names) == 3:
                        self._add(self.test_links, key, rating)      # triplets once more (:518-525)
                    if len(names) == 2:
                        self._add(self.dtest_links, key, rating)     # :526-533
                self.P = len(self.id_gene)
        except ValueError as error:
            print(error)
        except IOError as error:
            print('Error, file does not exist or can\'t be read')
            print(error)
        print('READ DATA train', len(self.links), len(self.nLinks))
        print('READ DATA train', len(self.dlinks), len(self.ndlinks))
        print('READ DATA test', len(self.test_links))

    # --------------------------------------------------------- :548-939 (host)
    def triplet_fold(self):
        test_set_size = int(len(self.links) / 5)
        array_links = list(self.links.keys())
        loop = 0
        while loop < test_set_size:
            try:
                triplet = np.random.choice(array_links)
                names = []
                for identifier in triplet.split("_"):
                    if self.gene_num_aparitions[int(identifier)] == 1:
                        raise ValueError("Triplet " + triplet + " has at least one gene with just one "
                                         "aparition. Choosing randomly another")
                    self.gene_num_aparitions[int(identifier)] -= 1
                    names.append(self.id_gene[int(identifier)])
                rating = 0 if self.links[triplet][0] else 1
                row = self.test_links.setdefault(triplet, [0] * 2)
                row[rating] += 1
                names.sort()
                self.nLinks.pop('_'.join(names))
                self.links.pop(triplet)
                array_links.remove(triplet)
                loop += 1
            except ValueError:
                pass

    def _fast_fold(self, table, ntable, test_table, other_table, fraction, output, folds, prefix,
                   train_other_first):
        """Shared body of triplet_fast_fold (:614-775) and pair_fast_fold (:777-939)."""
        test_set_size = int(len(table) * fraction)
        rest = len(table) % test_set_size
        num_folds = int(1 / fraction)
        keys = list(table.keys())
        other_keys = list(other_table.keys())
        np.random.shuffle(keys)
        handles = []
        if output:
            base_train = codecs.open(prefix + 'train.dat', encoding='utf-8', mode="w+")
            base_test = codecs.open(prefix + 'test.dat', encoding='utf-8', mode="w+")
            of_ta = [codecs.open(prefix + 'test%d.dat' % i, encoding='utf-8', mode="w+") for i in range(num_folds)]
            of_tra = [codecs.open(prefix + 'train%d.dat' % i, encoding='utf-8', mode="w+")
                      for i in range(num_folds)]
            handles = [base_train, base_test] + of_ta + of_tra
        test, train = [], []
        for i in range(num_folds):
            test.append(keys[test_set_size * i:test_set_size * (i + 1)])
            if i > 0:
                train += test[i]
        for j in range(rest):
            print(test_set_size * num_folds + j, len(keys))
            test[num_folds - 1].append(keys[test_set_size * num_folds + j])
        train += keys[test_set_size * num_folds:]

        def line(tab, key):
            rating = 0 if tab[key][0] else 1
            names = sorted(self.id_gene[int(i)] for i in key.split("_"))
            return '_'.join(names), rating

        for key in test[0]:
            rating = 0 if table[key][0] else 1
            test_table[key] = [0] * 2
            test_table[key][rating] += 1
            for identifier in key.split("_"):
                self.gene_num_aparitions[int(identifier)] -= 1
            str_names = '_'.join(sorted(self.id_gene[int(i)] for i in key.split("_")))
            ntable.pop(str_names)
            table.pop(key)
            if output:
                of_ta[0].write(str_names + '\t' + str(rating) + '\n')
        print('remaining test sets')
        for f in range(1, num_folds):
            print('fold', f, len(test[f]))
            for key in test[f]:
                str_names, rating = line(table, key)
                if output:
                    of_ta[f].write(str_names + '\t' + str(rating) + '\n')
        for key in train:
            if output:
                str_names, rating = line(table, key)
                of_tra[0].write(str_names + '\t' + str(rating) + '\n')
        for key in other_keys:
            if output:
                str_names, rating = line(other_table, key)
                of_tra[0].write(str_names + '\t' + str(rating) + '\n')
        for h in handles:
            h.close()
        if not output:
            # :774 / :938 close handles that only exist when `output` is set
            raise UnboundLocalError("local variable 'outf_train' referenced before assignment")

    def triplet_fast_fold(self, fraction=0.2, output=None, folds=None):
        self._fast_fold(self.links, self.nLinks, self.test_links, self.dlinks, fraction, output, folds, '',
                        False)

    def pair_fast_fold(self, fraction=0.2, output=None, folds=None):
        self._fast_fold(self.dlinks, self.ndlinks, self.dtest_links, self.links, fraction, output, folds, 'd',
                        False)

    # ------------------------------------------------------ hot path (GPU)
    def make_iteration(self):
        """One joint EM iteration on the GPU (:1572-1687).  ZeroDivisionError when a gene has no
        train triplet or pair, like :1642."""
        eng = self._push()
        eng.iterate(1)
        self._host_fresh = False

    def make_iterations(self, n):
        eng = self._push()
        eng.iterate(int(n))
        self._host_fresh = False

    def compute_likelihood(self):
        eng = self._push()
        self.likelihood = float(eng.loglik(_lib.SET_TRAIN)[0])
        return self.likelihood

    # ------------------------------------------------------- :946-1076
    def do_prediction(self, ids):
        try:
            ids = [int(i) for i in ids]
        except ValueError:
            ids = [self.gene_id[i] for i in ids]
        if len(ids) not in (2, 3):
            return 0
        for n, g in enumerate(ids):   # list indexing of theta (:955, :961)
            if not -self.P <= g < self.P:
                raise IndexError("list index out of range")
            ids[n] = g % self.P
        return float(self._push().predict(np.array([ids], dtype=np.int32))[0, 0])

    def calculate_test_set_results(self):
        rows = []
        for table in (self.test_links, self.dtest_links):
            for key, n in table.items():
                rows.append((key, 0 if n[0] else 1, [int(s) for s in key.split("_")]))
        probs = [0] * len(rows)   # a key of another arity predicts the int 0 (:948, :964)
        eng = self._push() if rows else None
        for arity in (3, 2):
            sel = [i for i, row in enumerate(rows) if len(row[2]) == arity]
            if sel:
                p = eng.predict(np.array([rows[i][2] for i in sel], dtype=np.int32))[0]
                for i, v in zip(sel, p):
                    probs[i] = float(v)
        self.results = [[probs[i], rows[i][0], rows[i][1]] for i in range(len(rows))]
        self.results.sort()
        self.results.reverse()

    def calculate_metrics(self):
        positives = sum(1 for n in self.links.values() if n[1] == 1)
        positives += sum(1 for n in self.dlinks.values() if n[1] == 1)
        positives_fraction = positives / (len(self.links) + len(self.dlinks))
        positives_number = int(positives_fraction * len(self.test_links))
        cut_value = 0
        if positives_number < len(self.results):
            cut_value = self.results[positives_number][0]
        pos = np.array([row[0] for row in self.results if row[2]], dtype=np.float64)
        neg = np.sort(np.array([row[0] for row in self.results if not row[2]], dtype=np.float64))
        better = int(np.searchsorted(neg, pos, side='left').sum())   # pairs with pos > neg (:1050-1053)
        auc = better / (len(pos) * len(neg))
        tp = fp = fn = tn = 0
        for row in self.results:
            if row[0] >= cut_value:
                if row[2]:
                    tp += 1
                else:
                    fp += 1
            elif row[2]:
                fn += 1
            else:
                tn += 1
        return [tp / (tp + fp), tp / (tp + fn), fp / (fp + tn), auc]

    # ------------------------------------------------------- :1231-1488
    def _head(self):
        text = "Max Likelihood:\t" + str(self.likelihood) + "\n"
        text += "Number of genes (P):\t" + str(self.P) + "\n"
        text += "Number of links:\t" + str(len(self.links)) + "\n"
        text += "Number of groups of genes (K):\n" + str(self.K) + "\n"
        text += "Number of possible ratings (R):\n" + str(self.R) + "\n\n"
        return text

    def _genes(self):
        text = "\nLIST OF REGISTERED GENES\n"
        text += "Gene_ID\tGene_name\tnumAparitions\n"
        for gid in self.id_gene:
            text += str(gid) + "\t" + self.id_gene[gid] + "\t" + str(self.gene_num_aparitions[gid]) + '\n'
        return text

    def _matrix(self, header, top):
        K = self.K
        txt = ''
        for i in range(K):
            txt += str(i) + "\n\t" + "".join(str(a) + "\t\t" for a in range(K)) + "\n\t" + "0\t1\t" * K + "\n"
            for j in range(K):
                cells = top[i][j] if header == 3 else [top[i][j]]
                txt += str(j) + "\t" + "".join("{0:.6f}".format(c[r]) + "\t" for c in cells
                                              for r in range(self.R)) + "\n"
            txt += "\n\n"
        return txt

    def to_string(self):
        text = self._head()
        text += "Likelihood vector: \n" + "Sample\titeration\tlikelihood\n"
        for num_sample, num_iteration, num_likelihood in self.likelihoodVector:
            text += str(num_sample) + "\t" + str(num_iteration) + "\t" + str(num_likelihood) + "\n"
        text += self._genes()
        text += "\nMATRIX OF PROBABILITIES PR\n" + self._matrix(3, self.pr)
        text += "\nMATRIX OF PROBABILITIES QR\n" + self._matrix(2, self.qr)
        text += "\nTHETA VECTOR\n" + '\n\t' + "".join(str(a) + "\t" for a in range(self.K))
        theta = self.theta
        for p in range(self.P):
            text += "\n" + str(p) + "\t" + "".join("{0:.12f}".format(v) + "\t" for v in theta[p])
        text += '\n'
        return text

    def to_string_short(self):
        text = self._head()
        self.calculate_test_set_results()
        text += "\nTest set:" + '\nPredicted Interaction\tID of genes\tReal Interaction\n'
        for row in self.results:
            text += str(row[0]) + '\t' + str(row[1]) + '\t' + str(row[2]) + '\n'
        metrics = self.calculate_metrics()
        text += "\nMetrics:\nPrecision\tRecall\tFallout\tAUC\n"
        text += str(metrics[0]) + "\t" + str(metrics[1]) + "\t" + str(metrics[2]) + "\t" + str(metrics[3])
        text += self._genes()
        return text

    def _write(self, name_file, producer):
        try:
            if name_file is None:
                name_file = "out.txt"
            fileref = codecs.open(name_file, encoding='utf-8', mode="w+")   # opened first (:1470)
            data = producer()
            fileref.write(data)
            fileref.close()
        except IOError:
            print("I/O error")

    def to_file(self, name_file=None):
        self._write(name_file, self.to_string)

    def to_file_short(self, name_file=None):
        self._write(name_file, self.to_string_short)

    # ------------------------------------------------------- :1499-1719
    def compare_links(self, arg_model):
        return [link for link in self.nLinks.keys() if link not in arg_model.nLinks.keys()]

    def compare_genes(self, arg_model):
        return [gene for gene in self.gene_id.keys() if gene not in arg_model.gene_id.keys()]

    def compare_dataset(self, arg_model):
        if not self.compare_links(arg_model):
            print("First dataset is subgraph of second dataset for links")
            node = 1
        else:
            print("First dataset is not subgraph of second dataset for links")
            node = 0
        if not self.compare_genes(arg_model):
            print("First dataset is subgraph of second dataset for nodes")
            link = 1
        else:
            print("First dataset is not subgraph of second dataset for nodes")
            link = 0
        return link and node
