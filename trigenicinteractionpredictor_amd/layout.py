"""Host-side construction of the device edge list (include/mmsbm.h, "Device layouts").

From the reference's link dictionaries (`links` / `test_links`, filled by
`get_traintest`, src/TrigenicInteractionPredictor.py:321-423) this builds:

* ``obs``  int32[n_obs_pad][4] = (id1, id2, id3, n): one row per observed
  (link, rating) pair, grouped by rating, each group padded to a multiple of
  MMSBM_TILE with (0,0,0,0) rows so that every workgroup tile is rating-uniform;
* ``seg``  int64[R+1] row offsets of the rating groups;
* the gene incidence CSR (``gene_ptr``, ``gene_inc``) of the theta M-step:
  entry ``row*3 + slot`` for every (observation, slot) of a gene, ascending;
* ``deg``  int32[P]: the reference's ``counter`` (:986-994) — one per LINK slot,
  independent of the counts.

Links are taken in dictionary insertion order; ids come from the string-sorted
key (``'10_2_9'`` -> (10, 2, 9), :349-358), which fixes which gene sits in
which slot of the (asymmetric) p lattice.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

TILE = 256


def links_to_arrays(links: dict, R: int = 2):
    """Ordered ``"i_j_k" -> [n_0..n_{R-1}]`` dict -> ids int32[E][3], counts int32[E][R]."""
    E = len(links)
    if E == 0:
        return np.zeros((0, 3), np.int32), np.zeros((0, R), np.int32)
    keys = "_".join(links.keys())
    ids = np.array(keys.split("_"), dtype=np.int64).astype(np.int32).reshape(E, 3)
    counts = np.array(list(links.values()), dtype=np.int64).astype(np.int32).reshape(E, R)
    return ids, counts


@dataclass
class ObsLayout:
    obs: np.ndarray        # int32[n_obs_pad][4]
    seg: np.ndarray        # int64[R+1]
    n_obs: int             # real (unpadded) observations
    link_of_row: np.ndarray  # int64[n_obs_pad] link index of each row, -1 for padding


def build_obs(ids: np.ndarray, counts: np.ndarray, tile: int = TILE,
              by_gene: bool = True) -> ObsLayout:
    """by_gene: within a rating, order the observations by their slot-0 gene (stable): a wave
    group's slot-0 rows then fall in one stretch of that gene's CSR run and its th_i loads
    repeat (summation order only; every sum stays fixed-order)."""
    R = counts.shape[1]
    blocks, owners, seg = [], [], [0]
    for r in range(R):
        sel = np.nonzero(counts[:, r] > 0)[0]
        if by_gene:
            sel = sel[np.argsort(ids[sel, 0], kind="stable")]
        n = sel.size
        pad = (-n) % tile
        blk = np.zeros((n + pad, 4), dtype=np.int32)
        blk[:n, :3] = ids[sel]
        blk[:n, 3] = counts[sel, r]
        own = np.full(n + pad, -1, dtype=np.int64)
        own[:n] = sel
        blocks.append(blk)
        owners.append(own)
        seg.append(seg[-1] + n + pad)
    obs = np.concatenate(blocks) if blocks else np.zeros((0, 4), np.int32)
    owner = np.concatenate(owners) if owners else np.zeros(0, np.int64)
    return ObsLayout(obs=np.ascontiguousarray(obs), seg=np.array(seg, dtype=np.int64),
                     n_obs=int((owner >= 0).sum()), link_of_row=owner)


@dataclass
class GeneCSR:
    ptr: np.ndarray   # int32[P+1]
    inc: np.ndarray   # int32[nnz]
    deg: np.ndarray   # int32[P]


def build_gene_csr(layout: ObsLayout, ids: np.ndarray, P: int) -> GeneCSR:
    real = np.nonzero(layout.link_of_row >= 0)[0]
    genes = layout.obs[real, :3].astype(np.int64)          # [n_obs][3]
    entry = (real[:, None] * 3 + np.arange(3)[None, :])     # row*3 + slot
    g_flat = genes.ravel()
    e_flat = entry.ravel()
    order = np.argsort(g_flat, kind="stable")               # ascending entry within a gene
    inc = e_flat[order].astype(np.int32)
    ptr = np.zeros(P + 1, dtype=np.int64)
    np.cumsum(np.bincount(g_flat, minlength=P)[:P], out=ptr[1:])
    deg = np.bincount(ids.ravel().astype(np.int64), minlength=P)[:P].astype(np.int32)
    return GeneCSR(ptr=ptr.astype(np.int32), inc=inc, deg=deg)
