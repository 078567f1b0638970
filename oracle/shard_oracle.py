"""ORACLE — TEST INFRASTRUCTURE ONLY.  The reference EM step (src/TrigenicInteractionPredictor.py
:984-1043) written as the two halves the link-sharded path splits it into, in numpy:

  accumulate  (:986-1012) over a block of links: per gene the sum of c * (Y | Z | W) (theta not
              applied: ntheta[g] = theta[g] * nth[g]), and S_r[a][b][g] += c th_i[a] th_j[b] th_k[g]
              with c = n_r / d_r, d_r = eps + sum th_i th_j th_k p_r (:996-1000)
  mstep       (:1016-1028) from the summed halves: theta <- theta nth / deg,
              p_r <- p_r S_r / (eps + sum_r p_r S_r)

Summed over any partition of the links, accumulate + mstep is the reference iteration
(tests/test_linkshard.py checks it against oracle/mmsbm_oracle.c to 1e-12).  Layouts: ids
int32[E][3], counts int32[E][R], theta f64[P][K], pr f64[K][K][K][R] (reference nesting),
nth f64[P][K], S f64[R][K^3] (cell = (a K + b) K + g).
"""
from __future__ import annotations

import numpy as np


def accumulate(ids, counts, theta, pr, eps=1e-10):
    P, K = theta.shape
    R = pr.shape[-1]
    nth = np.zeros((P, K))
    S = np.zeros((R, K, K, K))
    for (i, j, k), n in zip(np.asarray(ids), np.asarray(counts)):
        ti, tj, tk = theta[i], theta[j], theta[k]
        for r in range(R):
            if n[r] <= 0:          # an unobserved rating adds exactly +0.0 (:1002-1012)
                continue
            p = pr[..., r]
            d = eps + np.einsum("abg,a,b,g->", p, ti, tj, tk)
            c = n[r] / d
            nth[i] += c * np.einsum("abg,b,g->a", p, tj, tk)
            nth[j] += c * np.einsum("abg,a,g->b", p, ti, tk)
            nth[k] += c * np.einsum("abg,a,b->g", p, ti, tj)
            S[r] += c * np.einsum("a,b,g->abg", ti, tj, tk)
    return nth, S.reshape(R, K ** 3)


def mstep(theta, pr, nth, S, deg, eps=1e-10):
    """-> (theta', pr'); ZeroDivisionError for a zero degree, as :1018."""
    if np.any(np.asarray(deg) <= 0):
        raise ZeroDivisionError("float division by zero")
    K = theta.shape[1]
    R = pr.shape[-1]
    theta = theta * nth / np.asarray(deg, np.float64)[:, None]
    p = pr.reshape(K ** 3, R).T                     # [R][K^3]
    npr = p * S
    p = npr / (eps + npr.sum(axis=0))
    return theta, np.ascontiguousarray(p.T.reshape(K, K, K, R))
