"""Device engine: PyTorch-ROCm tensors for storage, libmmsbm.so for all compute.

One ``EMEngine`` = one GPU context (include/mmsbm.h) holding the train/test
edge lists, the gene incidence CSR, a workspace and B batched samples
(independent EM restarts) of theta f64[B][P][K] and p f64[B][R][K^3].
Nothing here computes on the host: every numeric step is a HIP kernel.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .layout import TILE, build_gene_csr, build_obs


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _stream(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class EMEngine:
    def __init__(self, K: int, P: int, B: int = 1, R: int = 2, eps: float = 1e-10, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("EMEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.K, self.P, self.B, self.R, self.eps = int(K), int(P), int(B), int(R), float(eps)
        self.K3 = self.K ** 3
        ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.mmsbm_create(self.device.index, ctypes.byref(ctx)))
        self.ctx = ctx
        _lib.check(self.lib.mmsbm_set_shape(self.ctx, self.K, self.R, self.B, self.P, self.eps))
        self._sets = {}
        self._csr = None
        self.zero_degree = False
        self.workspace = None
        self.theta = torch.zeros((self.B, self.P, self.K), dtype=torch.float64, device=self.device)
        self.pr = torch.zeros((self.B, self.R, self.K3), dtype=torch.float64, device=self.device)

    # ---------------------------------------------------------------- setup
    def _dev(self, a: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def set_links(self, which: int, ids: np.ndarray, counts: np.ndarray, deg: np.ndarray = None):
        """deg: the reference's `counter` over ALL train links; defaults to the one of `ids`
        (a link-sharded rank passes the global one)."""
        lay = build_obs(ids, counts, TILE)
        obs_d = self._dev(lay.obs)
        seg = (ctypes.c_int64 * (self.R + 1))(*[int(x) for x in lay.seg])
        _lib.check(self.lib.mmsbm_set_links(self.ctx, which, _ptr(obs_d) if obs_d.numel() else None,
                                            int(lay.obs.shape[0]), seg))
        self._sets[which] = (lay, obs_d)
        if which == _lib.SET_TRAIN:
            csr = build_gene_csr(lay, ids, self.P)
            if deg is not None:
                csr.deg = np.ascontiguousarray(deg, dtype=np.int32)
            ptr_d, inc_d, deg_d = self._dev(csr.ptr), self._dev(csr.inc), self._dev(csr.deg)
            self._csr = (csr, ptr_d, inc_d, deg_d)
            rc = self.lib.mmsbm_set_genes(self.ctx, _ptr(ptr_d), _ptr(inc_d) if inc_d.numel() else None,
                                          int(csr.inc.size), _ptr(deg_d))
            self.zero_degree = rc == _lib.MMSBM_ERR_ZERO_DEGREE
            if not self.zero_degree:
                _lib.check(rc)
        self._alloc_workspace()

    def _alloc_workspace(self):
        nbytes = ctypes.c_int64()
        _lib.check(self.lib.mmsbm_workspace_bytes(self.ctx, ctypes.byref(nbytes)))
        need = max(int(nbytes.value), 256)
        if self.workspace is None or self.workspace.numel() < need:
            self.workspace = torch.empty(need, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.mmsbm_set_workspace(self.ctx, _ptr(self.workspace), self.workspace.numel()))

    # ------------------------------------------------------------ parameters
    def upload(self, theta: np.ndarray, pr: np.ndarray):
        """theta [B][P][K]; pr in the reference nesting [B][K][K][K][R]."""
        theta = np.asarray(theta, dtype=np.float64).reshape(self.B, self.P, self.K)
        pr = np.asarray(pr, dtype=np.float64).reshape(self.B, self.K3, self.R)
        self.theta.copy_(torch.from_numpy(np.ascontiguousarray(theta)))
        self.pr.copy_(torch.from_numpy(np.ascontiguousarray(pr.transpose(0, 2, 1))))

    def download(self):
        """-> theta [B][P][K], pr [B][K][K][K][R] (host numpy)."""
        th = self.theta.cpu().numpy()
        pr = self.pr.cpu().numpy().transpose(0, 2, 1).reshape(self.B, self.K, self.K, self.K, self.R)
        return th, np.ascontiguousarray(pr)

    # --------------------------------------------------------------- compute
    def iterate(self, n_iters: int = 1, stream=None):
        if self.zero_degree:
            raise ZeroDivisionError("float division by zero")
        if _lib.SET_TRAIN not in self._sets:
            raise RuntimeError("train links not set")
        _lib.check(self.lib.mmsbm_iterate(self.ctx, _ptr(self.theta), _ptr(self.pr), int(n_iters),
                                          _stream(stream)))

    def accumulate(self, nth: torch.Tensor, S: torch.Tensor, stream=None):
        """Link-sharded step 1 (include/mmsbm.h): this context's sums nth [B][P][K], S [B][R][K^3]."""
        if _lib.SET_TRAIN not in self._sets:
            raise RuntimeError("train links not set")
        _lib.check(self.lib.mmsbm_accumulate(self.ctx, _ptr(self.theta), _ptr(self.pr), _ptr(nth),
                                             _ptr(S), _stream(stream)))

    def mstep(self, nth: torch.Tensor, S: torch.Tensor, stream=None):
        """Link-sharded step 2: M-step from the summed nth / S (ZeroDivisionError like :1018)."""
        if self.zero_degree:
            raise ZeroDivisionError("float division by zero")
        _lib.check(self.lib.mmsbm_mstep(self.ctx, _ptr(self.theta), _ptr(self.pr), _ptr(nth), _ptr(S),
                                        _stream(stream)))

    def loglik_async(self, which: int = _lib.SET_TRAIN, out: torch.Tensor = None, stream=None):
        if out is None:
            out = torch.empty(self.B, dtype=torch.float64, device=self.device)
        _lib.check(self.lib.mmsbm_loglik(self.ctx, which, _ptr(self.theta), _ptr(self.pr), _ptr(out),
                                         _stream(stream)))
        return out

    def loglik(self, which: int = _lib.SET_TRAIN) -> np.ndarray:
        if which not in self._sets:
            return np.zeros(self.B)
        return self.loglik_async(which).cpu().numpy()

    def predict(self, ids: np.ndarray) -> np.ndarray:
        """P(r=1) for each row of ids int32[n][3] -> [B][n] (host)."""
        n = int(ids.shape[0])
        out = torch.empty((self.B, max(n, 1)), dtype=torch.float64, device=self.device)
        if n:
            ids_d = self._dev(ids.astype(np.int32))
            _lib.check(self.lib.mmsbm_predict(self.ctx, _ptr(ids_d), n, _ptr(self.theta), _ptr(self.pr),
                                              _ptr(out), _stream(None)))
        return out[:, :n].cpu().numpy()

    # ---------------------------------------------------------- measurement
    KERNELS = ("estep", "m1", "m2")

    @property
    def fused(self) -> bool:
        """True when iterate() runs the fused FP64-MFMA E-step (E-step + S in one kernel)."""
        return self.fused_kind in (1, 2)

    @property
    def fused_kind(self) -> int:
        """0 VALU E-step + M1, 1 fused KR-image kernel (emx), 2 fused lean kernel (eml),
        3 large-K MFMA E-step (emb) + MFMA S accumulation (m1x)."""
        v = ctypes.c_int32()
        _lib.check(self.lib.mmsbm_fused(self.ctx, ctypes.byref(v)))
        return int(v.value)

    def time_estep(self, n: int = 50, stream=None) -> float:
        """Average device ms of n back-to-back E-step launches (measurement; parameters unchanged)."""
        ms = ctypes.c_double()
        _lib.check(self.lib.mmsbm_time_estep(self.ctx, _ptr(self.theta), _ptr(self.pr), int(n),
                                             _stream(stream), ctypes.byref(ms)))
        return ms.value

    def timing(self, stride: int = 1):
        """Record HIP event pairs around the kernels of every `stride`-th iteration (0: off)."""
        _lib.check(self.lib.mmsbm_timing(self.ctx, int(stride)))

    def timing_result(self, kernel: str = "estep"):
        """-> (summed device ms, launches) of one kernel since timing(True)."""
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.lib.mmsbm_timing_result(self.ctx, self.KERNELS.index(kernel),
                                                ctypes.byref(tot), ctypes.byref(cnt)))
        return tot.value, cnt.value

    def synchronize(self):
        torch.cuda.synchronize(self.device)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mmsbm_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
