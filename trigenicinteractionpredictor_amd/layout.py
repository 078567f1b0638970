"""Host link table of the device engine (include/mmsbm.h, mmsbm_set_links).

The reference keeps its link sets as ordered dictionaries ``"i_j_k" -> [n_0, n_1]``
(`links` / `test_links`, filled by `get_traintest`, src/TrigenicInteractionPredictor.py
:321-423).  The engine takes them as two int32 arrays in the same order: the key's gene ids
in its string-sorted order (``'10_2_9'`` -> (10, 2, 9), :349-358: that order decides which
gene sits in which slot of the asymmetric p lattice) and the per-rating counts.  The work plan
(observation streams ordered by each slot's gene, chunks, units, partial rows) is built from
these inside the library (csrc/plan.h).
"""
from __future__ import annotations

import numpy as np


def links_to_arrays(links: dict, R: int = 2):
    """Ordered ``"i_j_k" -> [n_0..n_{R-1}]`` dict -> ids int32[E][3], counts int32[E][R]."""
    E = len(links)
    if E == 0:
        return np.zeros((0, 3), np.int32), np.zeros((0, R), np.int32)
    keys = "_".join(links.keys())
    ids = np.array(keys.split("_"), dtype=np.int64).astype(np.int32).reshape(E, 3)
    counts = np.array(list(links.values()), dtype=np.int64).astype(np.int32).reshape(E, R)
    return ids, counts


def n_observations(counts: np.ndarray) -> int:
    """Observed (link, rating) pairs: the reference's per-link loop does work only for n_r > 0
    (an unobserved rating adds exactly +0.0, :1002-1012)."""
    return int((np.asarray(counts) > 0).sum())
