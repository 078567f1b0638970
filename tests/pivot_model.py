"""Numpy model of the engine's pivot-run factorisation (test infrastructure, CPU).

The reference EM step (src/TrigenicInteractionPredictor.py:984-1043) spends K^3 work per link.
The engine regroups the same sums by gene ("Pivot-run factorisation"):

  stream s (s = 0, 1, 2): the observations of rating r sorted by their slot-s gene (the pivot);
  u, v = the two other slots.  For the observations o with pivot gene g:

    V_g[b][h]   = sum_a th_g[a] p_r[a][b][h]                         (per gene, K^3)
    Z_o[b]      = sum_h V_g[b][h] th_k(o)[h]                          (stream 0, K^2 per obs)
    d_o         = eps + sum_b th_j(o)[b] Z_o[b]                       (= :996-1000)
    c_o         = n_o / d_o
    M^s_g[x][y] = sum_o c_o th_u(o)[x] th_v(o)[y]                    (K^2 per obs)

  then, per gene and rating (K^3 per gene, not per link):
    X0_g[a] = sum_bh p[a][b][h] M^0_g[b][h],  X1_g[b] = sum_ah p[a][b][h] M^1_g[a][h],
    X2_g[h] = sum_ab p[a][b][h] M^2_g[a][b]
    theta'_g = theta_g * sum_r (X0 + X1 + X2) / deg_g                  (:1009-1018)
    S_r = sum_g theta_g (x) M^0_g,  p' = p S / (eps + sum_r p S)        (:1012, :1021-1028)

The large-K kernels (K > 12, mmsbm.hip) keep only stream 0's pivot grouping and take the j- and
k-slot sums from the stream-0 pass itself, per observation:

    sum_ah T[a][b][h] = th_j[b] Z_o[b],   sum_ab T[a][b][h] = th_k[h] Z'_o[h],
    Z'_o[h] = sum_b th_j(o)[b] V_i[b][h]                               (K^2 per obs)

so the pass writes Y entries c_o Z_o (for gene j) and c_o Z'_o (for gene k) and
    theta'_g = theta_g * (sum_r X0_g + sum of g's Y entries) / deg_g
(`iterate_y`).

This model sums in numpy order; tests/test_pivot_model.py checks it against the C oracle.
"""
from __future__ import annotations

import numpy as np


def iterate(ids, counts, theta, pr, eps=1e-10):
    """One EM step.  ids int32[E][3], counts int32[E][R], theta [P][K], pr [K][K][K][R]."""
    ids = np.asarray(ids, np.int64)
    counts = np.asarray(counts)
    P, K = theta.shape
    R = pr.shape[-1]
    deg = np.bincount(ids.ravel(), minlength=P)[:P]
    if np.any(deg == 0):
        raise ZeroDivisionError("float division by zero")
    acc = np.zeros((P, K))
    S = np.zeros((R, K, K, K))
    p_new = np.empty_like(pr)
    for r in range(R):
        obs = np.nonzero(counts[:, r] > 0)[0]
        if obs.size == 0:
            continue
        p = pr[..., r]
        i, j, k = ids[obs, 0], ids[obs, 1], ids[obs, 2]
        n = counts[obs, r].astype(np.float64)
        V = np.einsum("ga,abh->gbh", theta, p)              # per gene
        Z = np.einsum("obh,oh->ob", V[i], theta[k])
        d = eps + np.einsum("ob,ob->o", theta[j], Z)
        c = n / d
        slots = ((i, j, k), (j, i, k), (k, i, j))          # (pivot, u, v)
        M = []
        for piv, u, v in slots:
            m = np.zeros((P, K, K))
            np.add.at(m, piv, c[:, None, None] * theta[u][:, :, None] * theta[v][:, None, :])
            M.append(m)
        acc += np.einsum("abh,gbh->ga", p, M[0])
        acc += np.einsum("abh,gah->gb", p, M[1])
        acc += np.einsum("abh,gab->gh", p, M[2])
        S[r] = np.einsum("ga,gbh->abh", theta, M[0])
    theta_new = theta * acc / deg[:, None]
    npr = np.moveaxis(S, 0, -1) * pr
    p_new = npr / (eps + npr.sum(axis=-1, keepdims=True))
    return theta_new, p_new


def iterate_y(ids, counts, theta, pr, eps=1e-10):
    """One EM step in the large-K kernels' grouping: stream-0 pivot rows for X0 and S, per-
    observation Y entries c Z (slot-1 gene) and c Z' (slot-2 gene) for the other two slots."""
    ids = np.asarray(ids, np.int64)
    counts = np.asarray(counts)
    P, K = theta.shape
    R = pr.shape[-1]
    deg = np.bincount(ids.ravel(), minlength=P)[:P]
    if np.any(deg == 0):
        raise ZeroDivisionError("float division by zero")
    acc = np.zeros((P, K))
    S = np.zeros((R, K, K, K))
    for r in range(R):
        obs = np.nonzero(counts[:, r] > 0)[0]
        if obs.size == 0:
            continue
        p = pr[..., r]
        i, j, k = ids[obs, 0], ids[obs, 1], ids[obs, 2]
        n = counts[obs, r].astype(np.float64)
        V = np.einsum("ga,abh->gbh", theta, p)
        Z = np.einsum("obh,oh->ob", V[i], theta[k])
        Zp = np.einsum("obh,ob->oh", V[i], theta[j])
        c = n / (eps + np.einsum("ob,ob->o", theta[j], Z))
        M0 = np.zeros((P, K, K))
        np.add.at(M0, i, c[:, None, None] * theta[j][:, :, None] * theta[k][:, None, :])
        acc += np.einsum("abh,gbh->ga", p, M0)
        np.add.at(acc, j, c[:, None] * Z)
        np.add.at(acc, k, c[:, None] * Zp)
        S[r] = np.einsum("ga,gbh->abh", theta, M0)
    theta_new = theta * acc / deg[:, None]
    npr = np.moveaxis(S, 0, -1) * pr
    return theta_new, npr / (eps + npr.sum(axis=-1, keepdims=True))


def loglik(ids, counts, theta, pr, eps=1e-10):
    ids = np.asarray(ids, np.int64)
    L = 0.0
    for r in range(pr.shape[-1]):
        obs = np.nonzero(counts[:, r] > 0)[0]
        if obs.size == 0:
            continue
        V = np.einsum("ga,abh->gbh", theta, pr[..., r])
        Z = np.einsum("obh,oh->ob", V[ids[obs, 0]], theta[ids[obs, 2]])
        d = eps + np.einsum("ob,ob->o", theta[ids[obs, 1]], Z)
        L += float(np.sum(counts[obs, r] * np.log(d)))
    return L
