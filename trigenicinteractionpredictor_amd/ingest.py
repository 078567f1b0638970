"""Native fold-file ingestion (include/mmsbm_io.h, libmmsbm_io.so): the canonical-format fast path
of `Model.get_traintest` (src/TrigenicInteractionPredictor.py:321-423), SURVEY.md §8f rank 3.

`parse_fold` returns a `Fold` (gene names in id order, `uniqueg`, train / test ids in key order
and their per-rating counts) or None when the input is outside the native reader's canonical
format; the Model then runs its reference-semantics Python reader.  The reference's dicts are
rebuilt from a Fold on demand: `links_dict` / `nlinks_dict` / `test_links_dict` give the same
keys, values and insertion order as the reference's loop.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .build import LIB_IO

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_IO):
            from .build import build_io
            build_io()
        lib = ctypes.CDLL(LIB_IO)
        vp, i64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)
        lib.mmsbm_fold_parse.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp)]
        lib.mmsbm_fold_parse.restype = ctypes.c_int
        lib.mmsbm_fold_sizes.argtypes = [vp, i64p, i64p, i64p, i64p]
        lib.mmsbm_fold_sizes.restype = ctypes.c_int
        lib.mmsbm_fold_export.argtypes = [vp] + [vp] * 6
        lib.mmsbm_fold_export.restype = ctypes.c_int
        lib.mmsbm_fold_free.argtypes = [vp]
        lib.mmsbm_fold_free.restype = None
        _lib = lib
    return _lib


@dataclass
class Fold:
    names: list            # id -> gene name
    uniqueg: np.ndarray    # int32[P]
    train_ids: np.ndarray  # int32[E][3], key order
    train_counts: np.ndarray
    test_ids: np.ndarray
    test_counts: np.ndarray

    @property
    def P(self) -> int:
        return len(self.names)

    def links_dict(self) -> dict:
        return _as_dict(self.train_ids, self.train_counts)

    def test_links_dict(self) -> dict:
        return _as_dict(self.test_ids, self.test_counts)

    def nlinks_dict(self) -> dict:
        """Keyed by the sorted gene NAMES (:354-366); same rows, order and counts as links."""
        nm = self.names
        return {"_".join(sorted((nm[a], nm[b], nm[c]))): [int(x), int(y)]
                for (a, b, c), (x, y) in zip(self.train_ids.tolist(), self.train_counts.tolist())}


def _as_dict(ids, counts) -> dict:
    return {"%d_%d_%d" % (a, b, c): [x, y] for (a, b, c), (x, y) in zip(ids.tolist(), counts.tolist())}


def parse_fold(trainfile, testfile):
    """-> Fold, or None when the native reader does not take this input (use the Python path)."""
    lib = _load()
    h = ctypes.c_void_p()
    rc = lib.mmsbm_fold_parse(os.fsencode(trainfile), os.fsencode(testfile), ctypes.byref(h))
    if rc != 0:
        return None
    try:
        P, Etr, Ete, nb = (ctypes.c_int64() for _ in range(4))
        lib.mmsbm_fold_sizes(h, ctypes.byref(P), ctypes.byref(Etr), ctypes.byref(Ete), ctypes.byref(nb))
        names = ctypes.create_string_buffer(max(nb.value, 1))
        uq = np.zeros(P.value, np.int32)
        tri, trc = np.zeros((Etr.value, 3), np.int32), np.zeros((Etr.value, 2), np.int32)
        tei, tec = np.zeros((Ete.value, 3), np.int32), np.zeros((Ete.value, 2), np.int32)
        ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
        lib.mmsbm_fold_export(h, names, ptr(uq), ptr(tri), ptr(trc), ptr(tei), ptr(tec))
        raw = names.raw[:nb.value]
        gene_names = raw.decode("ascii").split("\0")[:-1] if nb.value else []
        return Fold(gene_names, uq, tri, trc, tei, tec)
    finally:
        lib.mmsbm_fold_free(h)
