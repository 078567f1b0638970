"""Device engine: PyTorch-ROCm tensors for storage, libmmsbm.so for all compute.

One ``EMEngine`` = one GPU context (include/mmsbm.h) holding the train/test link sets (as the
engine's work plan), a workspace and B batched samples (independent EM restarts) of
theta f64[B][P][K] and p f64[B][R][K^3].  Nothing here computes on the host: every numeric step
is a HIP kernel.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _host_ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a.size else None


class EMEngine:
    KERNELS = ("pass_a", "pass_b", "fin")   # kernel ids of include/mmsbm.h's timing calls
    # what each id launches, by plan family (plan_info "small_k"): the large-K kernels (0) run
    # pass A, the gene kernel and the update; the small-K plan (1) pass A, pass B and fin; the
    # fused small-K plans (2: three streams, 3: stream 0 with Y entries) one E-step and fin
    LABELS = {0: {"pass_a": 0, "gene": 1, "fin": 2},
              1: {"pass_a": 0, "pass_b": 1, "fin": 2},
              2: {"fused": 0, "fin": 2},
              3: {"fused": 0, "fin": 2}}

    FAMILIES = {None: _lib.FAMILY_AUTO, "auto": _lib.FAMILY_AUTO, "sku": _lib.FAMILY_SKU,
                "sky": _lib.FAMILY_SKY}

    def __init__(self, K: int, P: int, B: int = 1, R: int = 2, eps: float = 1e-10, device=None,
                 family=None):
        """family (K <= 12, include/mmsbm.h mmsbm_set_family): "sku", "sky" or None / "auto"
        (SK_U at B = 1, SK_Y from B = 2).  A sample's bits depend on the family and on nothing
        else, so a driver whose engines differ in B for one run fixes it (family_for_batch)."""
        if not torch.cuda.is_available():
            raise RuntimeError("EMEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        if device is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            d = torch.device(device)
            self.device = torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())
        self.K, self.P, self.B, self.R, self.eps = int(K), int(P), int(B), int(R), float(eps)
        self.K3 = self.K ** 3
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.mmsbm_create(self.device.index, ctypes.byref(ctx)))
        self.ctx = ctx
        _lib.check(self.lib.mmsbm_set_shape(self.ctx, self.K, self.R, self.B, self.P, self.eps))
        if family not in self.FAMILIES:
            raise ValueError("family %r: one of sku, sky, auto" % (family,))
        _lib.check(self.lib.mmsbm_set_family(self.ctx, self.FAMILIES[family]))
        self.active = self.B
        self._sets = set()
        self.workspace = None
        self.theta = torch.zeros((self.B, self.P, self.K), dtype=torch.float64, device=self.device)
        self.pr = torch.zeros((self.B, self.R, self.K3), dtype=torch.float64, device=self.device)

    def _stream(self, stream=None) -> int:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return s.cuda_stream

    # ---------------------------------------------------------------- setup
    def set_links(self, which: int, ids: np.ndarray, counts: np.ndarray, deg: np.ndarray = None):
        """ids int32[E][3] (the keys' string-sorted gene ids), counts int32[E][R], in the link
        dict's insertion order.  deg: the reference's `counter` over ALL train links (a
        link-sharded rank passes the global one); by default the engine counts `ids`."""
        ids = np.ascontiguousarray(ids, dtype=np.int32).reshape(-1, 3)
        counts = np.ascontiguousarray(counts, dtype=np.int32).reshape(-1, self.R)
        if deg is not None and which == _lib.SET_TRAIN:
            d = np.ascontiguousarray(deg, dtype=np.int32)
            _lib.check(self.lib.mmsbm_set_degree(self.ctx, _host_ptr(d)))
        _lib.check(self.lib.mmsbm_set_links(self.ctx, which, _host_ptr(ids), _host_ptr(counts),
                                            int(ids.shape[0])))
        self._sets.add(which)
        self._alloc_workspace()

    def _alloc_workspace(self):
        nbytes = ctypes.c_int64()
        _lib.check(self.lib.mmsbm_workspace_bytes(self.ctx, ctypes.byref(nbytes)))
        need = max(int(nbytes.value), 256)
        if self.workspace is None or self.workspace.numel() < need:
            self.workspace = torch.empty(need, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.mmsbm_set_workspace(self.ctx, _ptr(self.workspace), self.workspace.numel()))

    def plan_info(self, which: int = _lib.SET_TRAIN) -> dict:
        v = (ctypes.c_int64 * 16)()
        _lib.check(self.lib.mmsbm_plan_info(self.ctx, which, v))
        keys = ("observations", "rows", "rows_stream0", "wg_stream0", "wg_stream12", "wg_spartial",
                "partial_rows", "genes_per_wg_max", "v_genes", "partial_rows_stream0", "small_k",
                "units", "plan_cus", "unit_target", "y_entries", "gm_groups")
        return dict(zip(keys, [int(x) for x in v]))

    # ------------------------------------------------------------ parameters
    def upload(self, theta: np.ndarray, pr: np.ndarray):
        """theta [B][P][K]; pr in the reference nesting [B][K][K][K][R]."""
        theta = np.asarray(theta, dtype=np.float64).reshape(self.B, self.P, self.K)
        pr = np.asarray(pr, dtype=np.float64).reshape(self.B, self.K3, self.R)
        self.theta.copy_(torch.from_numpy(np.ascontiguousarray(theta)))
        self.pr.copy_(torch.from_numpy(np.ascontiguousarray(pr.transpose(0, 2, 1))))

    # ---------------------------------------------------------- sample slots
    # A restart pool (restarts.run_pool) retires converged samples: it refills a slot with the next
    # pending sample, or moves the last live slot into it and shrinks the active prefix.
    def set_active(self, n: int):
        """Iterate / evaluate samples [0, n) only (include/mmsbm.h mmsbm_set_active)."""
        if not 0 < n <= self.B:
            raise ValueError("active samples %d outside [1, %d]" % (n, self.B))
        _lib.check(self.lib.mmsbm_set_active(self.ctx, int(n)))
        self.active = int(n)

    def upload_slot(self, b: int, theta: np.ndarray, pr: np.ndarray):
        """One sample's theta [P][K] and pr [K][K][K][R] into slot b."""
        th = np.asarray(theta, dtype=np.float64).reshape(self.P, self.K)
        p = np.asarray(pr, dtype=np.float64).reshape(self.K3, self.R)
        self.theta[b].copy_(torch.from_numpy(np.ascontiguousarray(th)))
        self.pr[b].copy_(torch.from_numpy(np.ascontiguousarray(p.T)))

    def download_slot(self, b: int):
        """-> theta [P][K], pr [K][K][K][R] of slot b (host numpy)."""
        th = self.theta[b].cpu().numpy()
        pr = self.pr[b].cpu().numpy().T.reshape(self.K, self.K, self.K, self.R)
        return th, np.ascontiguousarray(pr)

    def move_slot(self, dst: int, src: int):
        """Slot src's parameters into slot dst (a device copy: the bits travel unchanged)."""
        if dst != src:
            self.theta[dst].copy_(self.theta[src])
            self.pr[dst].copy_(self.pr[src])

    def download(self):
        """-> theta [B][P][K], pr [B][K][K][K][R] (host numpy)."""
        th = self.theta.cpu().numpy()
        pr = self.pr.cpu().numpy().transpose(0, 2, 1).reshape(self.B, self.K, self.K, self.K, self.R)
        return th, np.ascontiguousarray(pr)

    # --------------------------------------------------------------- compute
    def iterate(self, n_iters: int = 1, stream=None):
        if _lib.SET_TRAIN not in self._sets:
            raise RuntimeError("train links not set")
        _lib.check(self.lib.mmsbm_iterate(self.ctx, _ptr(self.theta), _ptr(self.pr), int(n_iters),
                                          self._stream(stream)))

    def accumulate(self, nth: torch.Tensor, S: torch.Tensor, stream=None):
        """Link-sharded step 1 (include/mmsbm.h): this context's sums nth [B][P][K], S [B][R][K^3]."""
        if _lib.SET_TRAIN not in self._sets:
            raise RuntimeError("train links not set")
        _lib.check(self.lib.mmsbm_accumulate(self.ctx, _ptr(self.theta), _ptr(self.pr), _ptr(nth),
                                             _ptr(S), self._stream(stream)))

    def mstep(self, nth: torch.Tensor, S: torch.Tensor, stream=None):
        """Link-sharded step 2: M-step from the summed nth / S (ZeroDivisionError like :1018)."""
        _lib.check(self.lib.mmsbm_mstep(self.ctx, _ptr(self.theta), _ptr(self.pr), _ptr(nth), _ptr(S),
                                        self._stream(stream)))

    def loglik_async(self, which: int = _lib.SET_TRAIN, out: torch.Tensor = None, stream=None):
        """[B] device tensor; the kernels write the active prefix only, slots outside it read NaN
        (the fill touches no word the launch writes, so its stream does not matter)."""
        if out is None:
            out = torch.empty(self.B, dtype=torch.float64, device=self.device)
        if self.active < self.B:
            out[self.active:] = float("nan")
        _lib.check(self.lib.mmsbm_loglik(self.ctx, which, _ptr(self.theta), _ptr(self.pr), _ptr(out),
                                         self._stream(stream)))
        return out

    def loglik(self, which: int = _lib.SET_TRAIN) -> np.ndarray:
        """[B] host array; slots outside the active prefix read NaN."""
        if which not in self._sets:
            out = np.zeros(self.B)
        else:
            out = self.loglik_async(which).cpu().numpy()
        out[self.active:] = np.nan
        return out

    def predict(self, ids: np.ndarray) -> np.ndarray:
        """P(r=1) for each row of ids int32[n][3] -> [B][n] (host); rows of slots outside the
        active prefix are NaN (the kernel covers the active samples only)."""
        n = int(ids.shape[0])
        out = torch.empty((self.B, max(n, 1)), dtype=torch.float64, device=self.device)
        if self.active < self.B:
            out[self.active:] = float("nan")
        if n:
            ids_d = torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int32)).to(self.device)
            _lib.check(self.lib.mmsbm_predict(self.ctx, _ptr(ids_d), n, _ptr(self.theta), _ptr(self.pr),
                                              _ptr(out), self._stream()))
        return out[:, :n].cpu().numpy()

    # ---------------------------------------------------------- measurement
    def kernels(self) -> dict:
        """{label: kernel id} of the kernels one iteration launches, in launch order (LABELS)."""
        return dict(self.LABELS[self.plan_info(_lib.SET_TRAIN)["small_k"]])

    def _kid(self, kernel) -> int:
        if kernel in self.KERNELS:
            return self.KERNELS.index(kernel)
        for labels in self.LABELS.values():
            if kernel in labels:
                return labels[kernel]
        raise KeyError(kernel)

    def time_kernel(self, kernel: str, n: int = 50, stream=None) -> float:
        """Average device ms of n back-to-back launches of one kernel of the iteration (a label
        of kernels() or an id name of KERNELS); the parameters are unchanged."""
        ms = ctypes.c_double()
        _lib.check(self.lib.mmsbm_time_kernel(self.ctx, self._kid(kernel), _ptr(self.theta),
                                              _ptr(self.pr), int(n), self._stream(stream),
                                              ctypes.byref(ms)))
        return ms.value

    def timing(self, stride: int = 1):
        """Record HIP event pairs around the kernels of every `stride`-th iteration (0: off)."""
        _lib.check(self.lib.mmsbm_timing(self.ctx, int(stride)))

    def timing_result(self, kernel: str = "pass_a"):
        """-> (summed device ms, launches) of one kernel since timing(stride)."""
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.lib.mmsbm_timing_result(self.ctx, self._kid(kernel),
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
