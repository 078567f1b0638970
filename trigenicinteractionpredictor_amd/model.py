"""`Model` — drop-in for the reference class `Model`
(AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py:33).

Same attribute names, method names, argument meaning and error behaviour.
The EM hot path (`make_iteration` :984-1043, `compute_likelihood` :952-974)
and the bulk test-set prediction (`do_prediction` :530-547 as used by
`calculate_test_set_results` :557-569) run as HIP kernels through
libmmsbm.so; there is no CPU fallback.  Ingestion, RNG initialisation, fold
splitting and text output stay on the host, as in the reference.

`theta` and `pr` are materialised as the reference's nested Python lists on
first access after the device moved them on; handing the lists out marks the
device copy stale, so in-place edits are uploaded before the next iteration
(the reference's `to_string`/`do_prediction` read them directly).
"""
from __future__ import annotations

import codecs
import random
import re

import numpy as np

from . import _lib
from .layout import links_to_arrays
from .tracked import TrackedLinks, tracked, version_of


NATIVE_INGEST = True   # get_traintest's native reader for canonical files (ingest.py)


class Model:
    def __init__(self, device=None):
        self._links_version = 0
        self._fold = None               # native parse backing the lazy link dicts (ingest.py)
        self._fold_v = [None, None]     # table version that still equals the parsed arrays
        self.ntheta = []
        self._theta = []
        self.id_gene = {}
        self.gene_id = {}
        self._pr = []
        self.npr = []
        self.nlinks = {}
        self.links = {}
        self.test_links = {}
        self.results = []
        self.uniqueg = {}
        self.likelihood = 0
        self.heldoutlikelihood = 0
        self.vlikelihood = []
        self.R = 2
        self.K = 0
        self.P = 0
        self.eps = 1e-10
        self._device = device
        self._engine = None
        self._engine_key = None
        self._host_fresh = True   # host lists hold the newest parameters
        self._dev_fresh = False   # device tensors hold the newest parameters

    # ------------------------------------------------------------------ state
    def _pull(self):
        if self._host_fresh:
            return
        th, pr = self._engine.download()
        self._theta = th[0].tolist()
        self._pr = pr[0].tolist()
        self._host_fresh = True

    @property
    def theta(self):
        self._pull()
        self._dev_fresh = False   # the caller may edit the lists in place
        return self._theta

    @theta.setter
    def theta(self, value):
        self._pull()
        self._theta = value
        self._dev_fresh = False

    @property
    def pr(self):
        self._pull()
        self._dev_fresh = False
        return self._pr

    @pr.setter
    def pr(self, value):
        self._pull()
        self._pr = value
        self._dev_fresh = False

    # ---------------------------------------------- link tables (lazy after a native parse)
    # After get_traintest's native reader, `links` / `nlinks` / `test_links` are built as the
    # reference's dicts on first access; until then the engine reads the parsed arrays.  The
    # tables are TrackedLinks (tracked.py): every in-place edit (`links[k][r] += 1`,
    # `links[k] = [..]`, `del links[k]`, ...) changes their version, and so does assigning a new
    # table.  The device copy is rebuilt whenever the versions differ from the ones it was built
    # from, as the reference re-reads the dicts on every call (:987, :959).
    @property
    def links(self):
        if self._links is None:
            self._links = TrackedLinks(self._fold.links_dict())
            self._fold_v[0] = self._links.version.n
        return self._links

    @links.setter
    def links(self, value):
        # a plain dict is aliased, not copied (tracked.TrackedLinks): `m.links = d` then
        # `d[k][r] += 1` reaches the device like the reference's shared object would
        self._links = tracked(value)
        self._fold_v[0] = None

    @property
    def test_links(self):
        if self._test_links is None:
            self._test_links = TrackedLinks(self._fold.test_links_dict())
            self._fold_v[1] = self._test_links.version.n
        return self._test_links

    @test_links.setter
    def test_links(self, value):
        self._test_links = tracked(value)
        self._fold_v[1] = None

    @property
    def nlinks(self):
        if self._nlinks is None:
            self._nlinks = self._fold.nlinks_dict()
        return self._nlinks

    @nlinks.setter
    def nlinks(self, value):
        self._nlinks = value

    def links_changed(self):
        """Declare an edit the tables cannot see: a key added to or deleted from a dict that was
        assigned to `links` / `test_links` (row edits such as `d[k][1] += 1` are seen without
        it).  The tables re-read their source dicts and the device copy is rebuilt on the next
        call."""
        for t in (self._links, self._test_links):
            if isinstance(t, TrackedLinks):
                t.resync()
        self._links_version += 1

    # copy.deepcopy / pickle: the device engine is not copied (the copy builds its own on first
    # use, from freshly pulled host parameters) and the tables come back tracked
    def __getstate__(self):
        self._pull()
        state = dict(self.__dict__)
        state.update(_engine=None, _engine_key=None, _dev_fresh=False, _host_fresh=True)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        for name in ("_links", "_test_links"):
            t = self.__dict__.get(name)
            if t is not None and not isinstance(t, TrackedLinks):
                # (a new version: _fold_fresh then reads the copied table, not the parse)
                self.__dict__[name] = TrackedLinks(t)

    def _fold_fresh(self, which):
        """The parsed arrays still hold table `which` (nothing edited or replaced it)."""
        if self._fold is None or self._fold_v[which] is None:
            return False
        tab = self._links if which == 0 else self._test_links
        return tab is None or tab.version.n == self._fold_v[which]

    def _link_arrays(self, which):
        """(ids int32[E][3] in key order, counts int32[E][R]) of the train (0) / test (1) links."""
        if self._fold_fresh(which):
            f = self._fold
            return (f.train_ids, f.train_counts) if which == 0 else (f.test_ids, f.test_counts)
        return links_to_arrays(self.links if which == 0 else self.test_links, self.R)

    def _n_links(self, which=0):
        if self._fold_fresh(which):
            return int((self._fold.train_ids if which == 0 else self._fold.test_ids).shape[0])
        return len(self.links if which == 0 else self.test_links)

    def _ensure_engine(self):
        from .engine import EMEngine  # imports torch + the HIP library
        key = (self.K, self.P, self._links_version, version_of(self._links), version_of(self._test_links))
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._pull()
                self._engine.close()
            eng = EMEngine(self.K, self.P, B=1, R=self.R, eps=self.eps, device=self._device)
            eng.set_links(_lib.SET_TRAIN, *self._link_arrays(0))
            eng.set_links(_lib.SET_TEST, *self._link_arrays(1))
            self._engine = eng
            self._engine_key = key
            self._dev_fresh = False
        return self._engine

    def _push(self):
        eng = self._ensure_engine()
        if not self._dev_fresh:
            self._pull()
            eng.upload(np.array(self._theta, dtype=np.float64)[None],
                       np.array(self._pr, dtype=np.float64)[None])
            self._dev_fresh = True
        return eng

    @property
    def engine(self):
        return self._push()

    # --------------------------------------------------- :106-170 (host RNG)
    def initialize_parameters(self, k_value=10):
        try:
            self.K = int(k_value)
        except ValueError:
            self.K = 10
        K, R, rnd = self.K, self.R, random.random
        self.vlikelihood = []
        self._theta = [[rnd() for _ in range(K)] for _ in range(self.P)]
        self.ntheta = [[0.0] * K for _ in range(self.P)]
        self._pr = [[[[rnd() for _ in range(R)] for _ in range(K)] for _ in range(K)] for _ in range(K)]
        self.npr = [[[[0.] * R for _ in range(K)] for _ in range(K)] for _ in range(K)]
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
        for plane in self._pr:
            for line in plane:
                for cell in line:
                    total = 0.
                    for v in cell:
                        total += v
                    for r in range(R):
                        cell[r] = cell[r] / total if total != 0 else cell[r] / (total + self.eps)
        self._host_fresh = True
        self._dev_fresh = False

    # ------------------------------------------------- :218-318, :321-423
    def _register(self, names, gid):
        ids = []
        for g in names:
            if g not in self.gene_id:
                self.gene_id[g] = gid
                self.id_gene[gid] = g
                self.uniqueg[gid] = 0
                gid += 1
            n = self.gene_id[g]
            self.uniqueg[n] += 1
            ids.append(str(n))
        return ids, gid

    def _add(self, table, key, r):
        row = table.get(key)
        if row is None:
            table[key] = [0] * 2
            row = table[key]   # a tracked table stores its own row object
        row[r] += 1

    def get_input(self, argfilename, selectedinteractiontype="trigenic", cutoffvalue=-0.08, discard=0,
                  interactions='ALL'):
        try:
            gid = 0
            if selectedinteractiontype not in ('trigenic', 'digenic', '*'):
                raise ValueError("argument 2 selectedInteractionType must be trigenic, digenic or *")
            with codecs.open(argfilename, encoding='utf-8', mode='r') as fileref:
                first = fileref.readline()
                raw = len(re.split(r'\t+', first)) == 12
                for line in fileref.readlines():
                    fields = re.split(r'\t+', line)
                    if raw:
                        fields.pop(5)
                    if selectedinteractiontype != "*" and fields[4] != selectedinteractiontype:
                        continue
                    if interactions == 'ALL':
                        r = 1 if (float(fields[6]) < 0.05 and float(fields[5]) < cutoffvalue) else 0
                    else:
                        if float(fields[6]) >= 0.05:
                            continue
                        if float(fields[5]) < cutoffvalue:
                            r = 1
                        elif discard:
                            continue
                        else:
                            r = 0
                    names = fields[1].split('+') + [fields[3]]
                    ids, gid = self._register(names, gid)
                    names.sort()
                    ids.sort()
                    self._add(self.links, '_'.join(ids), r)
                    self._add(self.nlinks, '_'.join(names), r)
                self.P = len(self.id_gene)
        except ValueError as error:
            print(error)
        except IOError as error:
            print('Error, file does not exist or can\'t be read')
            print(error)
        self._links_version += 1

    def get_traintest(self, trainfile, testfile):
        # native reader (include/mmsbm_io.h) for the canonical format on a fresh Model; any other
        # input takes the reference-semantics loop below
        fold = None
        if NATIVE_INGEST and not self.gene_id and not self._n_links(0) and not self._n_links(1):
            from .ingest import parse_fold
            fold = parse_fold(trainfile, testfile)
        if fold is not None:
            self._fold = fold
            self.id_gene = dict(enumerate(fold.names))
            self.gene_id = {g: i for i, g in enumerate(fold.names)}
            self.uniqueg = dict(enumerate(fold.uniqueg.tolist()))
            self._links = self._nlinks = self._test_links = None
            self._fold_v = [0, 0]
            self.P = fold.P
            self._links_version += 1
            n_train = self._n_links(0)
            print('READ DATA train', n_train, n_train)
            print('READ DATA test', self._n_links(1))
            return
        try:
            gid = 0
            with codecs.open(trainfile, encoding='utf-8', mode='r') as fileref:
                for line in fileref.readlines():
                    fields = line.strip().split('\t')
                    names = fields[0].split('_')
                    r = int(fields[1])
                    ids, gid = self._register(names, gid)
                    names.sort()
                    ids.sort()
                    self._add(self.links, '_'.join(ids), r)
                    self._add(self.nlinks, '_'.join(names), r)
                self.P = len(self.id_gene)
            with codecs.open(testfile, encoding='utf-8', mode='r') as fileref:
                for line in fileref.readlines():
                    fields = re.split(r'\t+', line)
                    names = fields[0].split('_')
                    r = int(fields[1])
                    ids, gid = self._register(names, gid)
                    ids.sort()
                    self._add(self.test_links, '_'.join(ids), r)
                self.P = len(self.id_gene)
        except ValueError as error:
            print(error)
        except IOError as error:
            print('Error, file does not exist or can\'t be read')
            print(error)
            exit(1)
        self._links_version += 1
        print('READ DATA train', len(self.links), len(self.nlinks))
        print('READ DATA test', len(self.test_links))

    # ------------------------------------------------------------- :447-523
    def fold(self, fraction=0.2):
        test_set_size = int(len(self.links) * fraction)
        num_folds = int(1 / fraction)
        keys = list(self.links.keys())
        np.random.shuffle(keys)
        chunks = [keys[test_set_size * i: test_set_size * (i + 1)] for i in range(num_folds)]
        chunks[num_folds - 1] += keys[test_set_size * num_folds:]

        def line(triplet):
            rating = 0 if self.links[triplet][0] else 1
            names = sorted(self.id_gene[int(x)] for x in triplet.split("_"))
            return '_'.join(names) + '\t' + str(rating) + '\n'

        for f in range(num_folds):
            with codecs.open('test' + str(f) + '.dat', encoding='utf-8', mode="w+") as out:
                for t in chunks[f]:
                    out.write(line(t))
            with codecs.open('train' + str(f) + '.dat', encoding='utf-8', mode="w+") as out:
                for other in chunks[:f] + chunks[f + 1:]:
                    for t in other:
                        out.write(line(t))

    # ------------------------------------------------------ hot path (GPU)
    def make_iteration(self):
        """One EM iteration on the GPU (:984-1043).  ZeroDivisionError when a
        gene has no train link, like :1018."""
        eng = self._push()
        eng.iterate(1)
        self._host_fresh = False

    def make_iterations(self, n):
        """`n` back-to-back iterations without host round trips."""
        eng = self._push()
        eng.iterate(int(n))
        self._host_fresh = False

    def compute_likelihood(self, selected_set='train'):
        eng = self._push()
        which = _lib.SET_TRAIN if selected_set == 'train' else _lib.SET_TEST
        log_l = float(eng.loglik(which)[0])
        if selected_set == 'train':
            self.likelihood = log_l
        else:
            self.heldoutlikelihood = log_l
        return log_l

    # ------------------------------------------------------- :530-637
    def do_prediction(self, id1, id2, id3):
        try:
            ids = [int(id1), int(id2), int(id3)]
        except ValueError:
            ids = [self.gene_id[id1], self.gene_id[id2], self.gene_id[id3]]
        # the reference indexes the theta list (:537): an id >= P raises IndexError and a
        # negative id counts from the end; the device kernel is only ever handed ids in [0, P)
        for n, g in enumerate(ids):
            if not -self.P <= g < self.P:
                raise IndexError("list index out of range")
            ids[n] = g % self.P
        eng = self._push()
        return float(eng.predict(np.array([ids], dtype=np.int32))[0, 0])

    def calculate_test_set_results(self):
        tids, _ = self._link_arrays(1)
        keys = list(self.test_links.keys())
        probs = self._push().predict(tids)[0] if keys else []
        self.results = []
        for p, key in zip(probs, keys):
            self.results.append([float(p), key, 0 if self.test_links[key][0] else 1])
        self.results.sort()
        self.results.reverse()

    def calculate_metrics(self):
        if self._fold_fresh(0):
            positives = int((self._fold.train_counts[:, 1] == 1).sum())
        else:
            positives = sum(1 for n in self.links.values() if n[1] == 1)
        positives_fraction = positives / self._n_links(0)
        positives_number = int(positives_fraction * self._n_links(1))
        cut_value = 0
        if positives_number < len(self.results):
            cut_value = self.results[positives_number][0]
        pos = np.array([row[0] for row in self.results if row[2]], dtype=np.float64)
        neg = np.sort(np.array([row[0] for row in self.results if not row[2]], dtype=np.float64))
        # pairs with positive strictly above negative (:611-615), by rank instead of O(n+ n-)
        better = int(np.searchsorted(neg, pos, side='left').sum())
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

    # ------------------------------------------------------- :793-904
    def to_string(self):
        def print_tuples(tuples):
            txt = '\nPredicted Interaction\tID of genes\tReal Interaction\n'
            for row in tuples:
                txt += str(row[0]) + '\t' + str(row[1]) + '\t' + str(row[2]) + '\n'
            return txt

        text = "Max Likelihood:\t" + str(self.likelihood) + "\n"
        text += "Held-out Likelihood:\t" + str(self.compute_likelihood('test')) + "\n"
        text += "Number of genes (P):\t" + str(self.P) + "\n"
        text += "Number of links:\t" + str(self._n_links(0)) + "\n"
        text += "Number of groups of genes (K):\n" + str(self.K) + "\n"
        text += "Number of possible ratings (R):\n" + str(self.R) + "\n\n"
        self.calculate_test_set_results()
        metrics = self.calculate_metrics()
        text += "\nMetrics:\nPrecision\tRecall\tFallout\tAUC\n"
        text += str(metrics[0]) + "\t" + str(metrics[1]) + "\t" + str(metrics[2]) + "\t" + str(metrics[3])
        text += "\nTest set:" + str(print_tuples(self.results))
        return text

    def to_file(self, name_file=None):
        try:
            if name_file is None:
                name_file = "out.txt"
            # the file is created before the text is built (:898-899): if to_string raises, an
            # empty file stays behind, which the CLI's resume rule (:1256) then skips
            with codecs.open(name_file, encoding='utf-8', mode="w+") as fileref:
                fileref.write(self.to_string())
        except IOError:
            print("I/O error")

    # ------------------------------------------------------- :915-1067
    def compare_links(self, arg_model):
        return [link for link in self.nlinks.keys() if link not in arg_model.nlinks]

    def compare_genes(self, arg_model):
        return [gene for gene in self.gene_id.keys() if gene not in arg_model.gene_id]

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
