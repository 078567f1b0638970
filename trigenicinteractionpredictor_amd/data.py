"""Synthetic fold files in the reference's on-disk format.

The reference's real folds (`data/DATA_FOLDS/{train,test}{0-4}.dat`) are Git-LFS
pointers, so every configuration is stood in for by a generated fold with the
same file format: one line per link, ``name1_name2_name3\\t<r>\\n`` with the three
gene names sorted (format written by `src/TrigenicInteractionPredictor.py:486-491`
and `:516-521`, read by `get_traintest` `:321-423`).

Genes are named ``g%05d`` (zero padded, so string order == numeric order),
positives are Bernoulli(``pos_frac``) and the first ``test_frac`` of the
non-coverage triples go to the test file.  Every gene is placed in at least one
train triple: a gene seen only in the test file makes the reference's
``make_iteration`` divide by a zero degree (`:1016-1018`).
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass

import numpy as np

__all__ = ["FoldSpec", "FOLD0", "write_fold", "gene_name", "JointFoldSpec", "write_joint_fold"]


def gene_name(idx: int) -> str:
    return "g%05d" % idx


@dataclass(frozen=True)
class FoldSpec:
    """Shape of a synthetic fold.  ``E`` counts unique triples (train + test)."""

    P: int
    E: int
    seed: int = 7
    pos_frac: float = 0.05
    test_frac: float = 0.2
    multi_frac: float = 0.0   # train links given 1..3 extra copies of their line
    both_frac: float = 0.0    # train links given one extra line with the other rating
    dup_frac: float = 0.0     # triples with a repeated gene, e.g. a_a_c
    # hub-heavy degrees, like the trigenic screens behind get_input (:218-318), where a few query
    # genes sit in many triples: hub_share of the non-coverage triples take one gene from the
    # first hub_frac of a gene permutation (0 = uniform, the default)
    hub_frac: float = 0.0
    hub_share: float = 0.0


# "fold0 stand-in", sized from the LFS byte counts
# (train0.dat 1,793,824 B + test0.dat 448,744 B at ~25 B/line).
FOLD0 = FoldSpec(P=1500, E=90000, seed=7)


def _line(names, r) -> str:
    return "_".join(names) + "\t" + str(r) + "\n"


def _python_triples(spec: FoldSpec, rng: random.Random):
    P = spec.P
    seen = set()
    cover = []
    perm = list(range(P))
    rng.shuffle(perm)
    for s in range(0, P, 3):
        tri = perm[s:s + 3]
        while len(tri) < 3:
            g = rng.randrange(P)
            if g not in tri:
                tri.append(g)
        key = tuple(sorted(tri))
        if key not in seen:
            seen.add(key)
            cover.append(key)
    rest = []
    hubs = perm[: max(1, int(P * spec.hub_frac))] if spec.hub_frac else []
    while len(cover) + len(rest) < spec.E:
        if spec.dup_frac and rng.random() < spec.dup_frac:
            a, c = rng.sample(range(P), 2)
            key = tuple(sorted((a, a, c)))
        elif hubs and rng.random() < spec.hub_share:
            h = hubs[rng.randrange(len(hubs))]
            a, c = rng.sample(range(P), 2)
            if h in (a, c):
                continue
            key = tuple(sorted((h, a, c)))
        else:
            key = tuple(sorted(rng.sample(range(P), 3)))
        if key in seen:
            continue
        seen.add(key)
        rest.append(key)
    return cover, rest


def _numpy_triples(spec: FoldSpec):
    """Vectorised variant for large E (10M-link stress config).  Takes the hub options (the
    same rule as the Python path: hub_share of the drawn triples take their first gene from the
    first hub_frac of the permutation); the per-line options (multi / both / dup) belong to the
    Python path only and raise here."""
    P, E = spec.P, spec.E
    if spec.multi_frac or spec.both_frac or spec.dup_frac:
        raise NotImplementedError("multi_frac / both_frac / dup_frac: only for E < 1,000,000 "
                                  "(the per-line Python generator)")
    rs = np.random.default_rng(spec.seed)
    perm = rs.permutation(P)
    hubs = perm[: max(1, int(P * spec.hub_frac))] if spec.hub_frac else None
    nfull = P // 3
    cover = np.sort(perm[: nfull * 3].reshape(nfull, 3), axis=1)
    if P % 3:
        tail = list(perm[nfull * 3:])
        others = [g for g in rs.permutation(P) if g not in tail][: 3 - len(tail)]
        cover = np.vstack([cover, np.sort(np.array(tail + others))[None, :]])
    enc = lambda t: (t[:, 0].astype(np.int64) * P + t[:, 1]) * P + t[:, 2]
    cover_codes = np.unique(enc(cover))
    need = E - cover_codes.size
    codes = np.empty(0, dtype=np.int64)
    while codes.size < need:
        m = int((need - codes.size) * 1.1) + 1024
        t = rs.integers(0, P, size=(m, 3))
        if hubs is not None:      # (no extra draws without hubs: the uniform folds are unchanged)
            hub = rs.random(m) < spec.hub_share
            t[hub, 0] = hubs[rs.integers(0, hubs.size, size=int(hub.sum()))]
        t = t[(t[:, 0] != t[:, 1]) & (t[:, 0] != t[:, 2]) & (t[:, 1] != t[:, 2])]
        t.sort(axis=1)
        c = np.unique(enc(t))
        c = c[~np.isin(c, cover_codes)]
        codes = np.unique(np.concatenate([codes, c]))
    codes = rs.permutation(codes)[:need]
    dec = lambda c: np.stack([c // (P * P), (c // P) % P, c % P], axis=1)
    return dec(cover_codes), dec(codes), rs


def write_fold(spec: FoldSpec, train_path: str, test_path: str) -> tuple[int, int]:
    """Write a synthetic train/test fold pair; returns (#train lines, #test lines)."""
    if spec.E >= 1_000_000:
        return _write_fold_numpy(spec, train_path, test_path)
    rng = random.Random(spec.seed)
    cover, rest = _python_triples(spec, rng)
    n_test = int(spec.E * spec.test_frac)
    n_test = min(n_test, len(rest))
    test, train_rest = rest[:n_test], rest[n_test:]
    train = cover + train_rest
    rng.shuffle(train)
    rating = {}
    for key in train + test:
        rating[key] = 1 if rng.random() < spec.pos_frac else 0
    names = lambda key: sorted(gene_name(g) for g in key)
    train_lines = [_line(names(k), rating[k]) for k in train]
    extra = []
    for k in train:
        if spec.multi_frac and rng.random() < spec.multi_frac:
            extra += [_line(names(k), rating[k])] * rng.randint(1, 3)
        if spec.both_frac and rng.random() < spec.both_frac:
            extra.append(_line(names(k), 1 - rating[k]))
    rng.shuffle(extra)
    train_lines += extra
    test_lines = [_line(names(k), rating[k]) for k in test]
    for path, lines in ((train_path, train_lines), (test_path, test_lines)):
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w", encoding="utf-8") as f:
            f.writelines(lines)
    return len(train_lines), len(test_lines)


def _write_fold_numpy(spec: FoldSpec, train_path: str, test_path: str):
    cover, rest, rs = _numpy_triples(spec)
    n_test = min(int(spec.E * spec.test_frac), rest.shape[0])
    test = rest[:n_test]
    train = np.vstack([cover, rest[n_test:]])
    train = train[rs.permutation(train.shape[0])]
    width = len(gene_name(spec.P - 1))

    def dump(path, tri):
        if tri.shape[0] == 0:                      # (test_frac 0: an empty test file)
            open(path, "w").close()
            return
        r = (rs.random(tri.shape[0]) < spec.pos_frac).astype(np.int64)
        names = np.char.add("g", np.char.zfill(tri.astype(str), width - 1))
        lines = np.char.add(np.char.add(np.char.add(names[:, 0], "_"),
                                        np.char.add(names[:, 1], "_")),
                            np.char.add(names[:, 2], np.char.add("\t", r.astype(str))))
        with open(path, "w", encoding="utf-8") as f:
            chunk = 1 << 20
            for s in range(0, lines.size, chunk):
                f.write("\n".join(lines[s:s + chunk].tolist()))
                f.write("\n")

    dump(train_path, train)
    dump(test_path, test)
    return int(train.shape[0]), int(test.shape[0])


def synthetic_links(spec: FoldSpec):
    """Train link table of a synthetic fold as arrays, without writing files (the 10M-link
    stress configuration): ids int32[E_train][3] (each triple sorted ascending), counts
    int32[E_train][2] with one observation per link, rating Bernoulli(``pos_frac``)."""
    cover, rest, rs = _numpy_triples(spec)
    n_test = min(int(spec.E * spec.test_frac), rest.shape[0])
    train = np.vstack([cover, rest[n_test:]])
    train = train[rs.permutation(train.shape[0])].astype(np.int32)
    r = (rs.random(train.shape[0]) < spec.pos_frac).astype(np.int32)
    counts = np.zeros((train.shape[0], 2), dtype=np.int32)
    counts[np.arange(train.shape[0]), r] = 1
    return np.ascontiguousarray(train), counts


# ---- joint digenic + trigenic folds (src/TrigenicInteractionPredictor_23.py) ----
HO_DELTA = "hoΔ"   # filler allele the joint reader drops from every key (:405-410)


@dataclass(frozen=True)
class JointFoldSpec:
    """A fold with triplet lines ``a_b_c\\t<r>`` and pair lines ``a_b\\t<r>`` mixed in one
    file, as `get_train_test` (:393-546) reads them.  Triplets use genes ``[0, P - pair_only)``;
    the last ``pair_only`` genes appear only in pairs, so their degree comes from the pair loop
    alone (:1616-1617).  ``ho_frac`` of the pair lines carry the filler allele as a third name."""

    P: int
    E3: int
    E2: int
    seed: int = 7
    pos_frac: float = 0.05
    pair_pos_frac: float = 0.1
    test_frac: float = 0.2
    multi_frac: float = 0.0
    both_frac: float = 0.0
    pair_only: int = 0
    ho_frac: float = 0.0


def write_joint_fold(spec: JointFoldSpec, train_path: str, test_path: str) -> tuple[int, int]:
    """Write a synthetic joint train/test fold; returns (#train lines, #test lines)."""
    rng = random.Random(spec.seed)
    P3 = spec.P - spec.pair_only
    if spec.E3:
        cover, rest = _python_triples(FoldSpec(P=P3, E=spec.E3, seed=spec.seed), rng)
    else:
        cover, rest = [], []
    pairs, seen = [], set()
    only = list(range(P3, spec.P))
    for s in range(0, len(only)):   # cover: each pair-only gene with a random partner
        b = rng.randrange(spec.P - 1)
        b = b if b < only[s] else b + 1
        key = tuple(sorted((only[s], b)))
        if key not in seen:
            seen.add(key)
            pairs.append(key)
    while len(pairs) < spec.E2:
        key = tuple(sorted(rng.sample(range(spec.P), 2)))
        if key not in seen:
            seen.add(key)
            pairs.append(key)
    ncover = len(only)
    n3_test = min(int(spec.E3 * spec.test_frac), len(rest))
    n2_test = min(int(spec.E2 * spec.test_frac), len(pairs) - ncover)
    test_keys = rest[:n3_test] + pairs[len(pairs) - n2_test:]
    train_keys = cover + rest[n3_test:] + pairs[:len(pairs) - n2_test]
    rating = {}
    for key in train_keys + test_keys:
        frac = spec.pos_frac if len(key) == 3 else spec.pair_pos_frac
        rating[key] = 1 if rng.random() < frac else 0

    def names(key):
        n = [gene_name(g) for g in key]
        if len(key) == 2 and spec.ho_frac and rng.random() < spec.ho_frac:
            n.append(HO_DELTA)
        return sorted(n)

    train_lines = [_line(names(k), rating[k]) for k in train_keys]
    for k in train_keys:
        if spec.multi_frac and rng.random() < spec.multi_frac:
            train_lines += [_line(names(k), rating[k])] * rng.randint(1, 3)
        if spec.both_frac and rng.random() < spec.both_frac:
            train_lines.append(_line(names(k), 1 - rating[k]))
    test_lines = [_line(names(k), rating[k]) for k in test_keys]
    rng.shuffle(train_lines)
    rng.shuffle(test_lines)
    for path, lines in ((train_path, train_lines), (test_path, test_lines)):
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w", encoding="utf-8") as f:
            f.writelines(lines)
    return len(train_lines), len(test_lines)
