"""ORACLE — TEST INFRASTRUCTURE ONLY.  ctypes binding of oracle/mmsbm_oracle.c.

Array-level view of the reference path (`src/TrigenicInteractionPredictor.py`
:952-974 loglik, :984-1043 EM step, :530-547 prediction), bit-identical to
`oracle/mmsbm_oracle.py`.  Layouts: ids int32[E][3], counts int32[E][R],
theta f64[P][K], pr f64[K][K][K][R] (the reference's nesting).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmmsbm_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P_i32 = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        P_f64 = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        L.oracle_loglik.restype = ctypes.c_double
        L.oracle_loglik.argtypes = [ctypes.c_int64, P_i32, P_i32, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_double, P_f64, P_f64]
        L.oracle_make_iteration.restype = ctypes.c_int
        L.oracle_make_iteration.argtypes = [ctypes.c_int64, P_i32, P_i32, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_double, P_f64, P_f64]
        L.oracle_accumulate.restype = None
        L.oracle_accumulate.argtypes = [ctypes.c_int64, P_i32, P_i32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_double, P_f64, P_f64, P_f64, P_f64]
        L.oracle_predict.restype = None
        L.oracle_predict.argtypes = [ctypes.c_int64, P_i32, ctypes.c_int, ctypes.c_int,
                                     P_f64, P_f64, P_f64]
        L.oracle_pair_loglik.restype = ctypes.c_double
        L.oracle_pair_loglik.argtypes = [ctypes.c_int64, P_i32, P_i32, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_double, P_f64, P_f64, ctypes.c_double]
        L.oracle_joint_make_iteration.restype = ctypes.c_int
        L.oracle_joint_make_iteration.argtypes = [ctypes.c_int64, P_i32, P_i32, ctypes.c_int64, P_i32,
                                                  P_i32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_double, P_f64, P_f64, P_f64]
        L.oracle_pair_predict.restype = None
        L.oracle_pair_predict.argtypes = [ctypes.c_int64, P_i32, ctypes.c_int, ctypes.c_int,
                                          P_f64, P_f64, P_f64]
        _lib = L
    return _lib


def links_to_arrays(links: dict, R: int = 2, arity: int = 3):
    """`links` dict ("i_j_k" -> [n0, n1]; "i_j" for `dlinks`, arity 2) in insertion order
    -> (ids, counts)."""
    E = len(links)
    ids = np.empty((E, arity), dtype=np.int32)
    counts = np.empty((E, R), dtype=np.int32)
    for e, (key, n) in enumerate(links.items()):
        ids[e] = [int(s) for s in key.split("_")]
        counts[e] = n[:R]
    return ids, counts


def loglik(ids, counts, theta, pr, eps=1e-10):
    K = theta.shape[1]
    R = counts.shape[1]
    return lib().oracle_loglik(ids.shape[0], ids, counts, K, R, eps,
                               np.ascontiguousarray(theta), np.ascontiguousarray(pr))


def make_iteration(ids, counts, theta, pr, eps=1e-10):
    """Returns new (theta, pr); raises ZeroDivisionError like :1018."""
    theta = np.array(theta, dtype=np.float64, copy=True, order="C")
    pr = np.array(pr, dtype=np.float64, copy=True, order="C")
    P, K = theta.shape
    R = counts.shape[1]
    rc = lib().oracle_make_iteration(ids.shape[0], ids, counts, P, K, R, eps, theta, pr)
    if rc != 0:
        raise ZeroDivisionError("float division by zero")
    return theta, pr


def accumulate(ids, counts, theta, pr, eps=1e-10):
    """The per-link sums of :986-1012 over these links -> (nth [P][K], npr [K][K][K][R]); the
    C loop releases the GIL, so disjoint link blocks can run on threads."""
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    pr = np.ascontiguousarray(pr, dtype=np.float64)
    P, K = theta.shape
    R = counts.shape[1]
    nth = np.zeros((P, K), dtype=np.float64)
    npr = np.zeros(pr.shape, dtype=np.float64)
    lib().oracle_accumulate(ids.shape[0], np.ascontiguousarray(ids, dtype=np.int32),
                            np.ascontiguousarray(counts, dtype=np.int32), P, K, R, eps, theta, pr, nth, npr)
    return nth, npr


def predict(ids, theta, pr):
    K = theta.shape[1]
    out = np.empty(ids.shape[0], dtype=np.float64)
    lib().oracle_predict(ids.shape[0], np.ascontiguousarray(ids), K, pr.shape[-1],
                         np.ascontiguousarray(theta), np.ascontiguousarray(pr), out)
    return out


# ---- joint digenic + trigenic model (src/TrigenicInteractionPredictor_23.py) ----
# ids2 int32[E2][2], counts2 int32[E2][R], qr f64[K][K][R].

def pair_loglik(ids2, counts2, theta, qr, eps=1e-10, start=0.0):
    K = theta.shape[1]
    R = counts2.shape[1]
    return lib().oracle_pair_loglik(ids2.shape[0], np.ascontiguousarray(ids2, dtype=np.int32),
                                    np.ascontiguousarray(counts2, dtype=np.int32), K, R, eps,
                                    np.ascontiguousarray(theta), np.ascontiguousarray(qr), start)


def joint_loglik(ids3, counts3, ids2, counts2, theta, pr, qr, eps=1e-10):
    """compute_likelihood of the joint model (:1534-1562): one running sum, triplets then pairs."""
    return pair_loglik(ids2, counts2, theta, qr, eps, start=loglik(ids3, counts3, theta, pr, eps))


def joint_make_iteration(ids3, counts3, ids2, counts2, theta, pr, qr, eps=1e-10):
    """Returns new (theta, pr, qr) of :1572-1687; raises ZeroDivisionError like :1642."""
    theta = np.array(theta, dtype=np.float64, copy=True, order="C")
    pr = np.array(pr, dtype=np.float64, copy=True, order="C")
    qr = np.array(qr, dtype=np.float64, copy=True, order="C")
    P, K = theta.shape
    R = qr.shape[-1]
    ids3 = np.ascontiguousarray(ids3, dtype=np.int32).reshape(-1, 3)
    counts3 = np.ascontiguousarray(counts3, dtype=np.int32).reshape(-1, R)
    ids2 = np.ascontiguousarray(ids2, dtype=np.int32).reshape(-1, 2)
    counts2 = np.ascontiguousarray(counts2, dtype=np.int32).reshape(-1, R)
    rc = lib().oracle_joint_make_iteration(ids3.shape[0], ids3, counts3, ids2.shape[0], ids2, counts2,
                                           P, K, R, eps, theta, pr, qr)
    if rc != 0:
        raise ZeroDivisionError("float division by zero")
    return theta, pr, qr


def pair_predict(ids2, theta, qr):
    K = theta.shape[1]
    out = np.empty(ids2.shape[0], dtype=np.float64)
    lib().oracle_pair_predict(ids2.shape[0], np.ascontiguousarray(ids2, dtype=np.int32), K, qr.shape[-1],
                              np.ascontiguousarray(theta), np.ascontiguousarray(qr), out)
    return out
